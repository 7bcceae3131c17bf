"""CPU restatement of the y-slab decomposed vortex-merger step (TEST INFRASTRUCTURE ONLY).

The reference is single-process (no parallelism of any kind).  This module
restates, in NumPy, the decomposition libcfdj.so implements for multi-GPU runs
(cfd_julia_amd/csrc/cfdj_api.hip: cfdj_vm::poisson / halo / alltoall, pack/unpack
kernels) so the CPU test suite can check its index arithmetic over real process groups
(torch.distributed gloo, world_size >= 2) against the single-domain oracle:

  rank p owns rows j in [p*rows, (p+1)*rows), rows = ny/P;
  Poisson: row r2c along x -> pack S[q][jl][kl] = X[q*kb+kl, jl] (kb = ceil((nx/2+1)/P),
  zero padded) -> all-to-all -> Y[y][kl] (y = p*rows + jl) -> c2c along y -> divide by the
  symbol at global kx = rank*kb + kl -> inverse c2c -> all-to-all -> unpack -> c2r;
  stencil: 1-row halos of omega and psi from ranks p-1 / p+1 (periodic).
"""
from __future__ import annotations

import numpy as np
import scipy.fft as sfft

from . import vm_oracle as vo


class LocalComm:
    """P virtual ranks in one process (lists of per-rank arrays).  `calls` counts the
    collectives by kind."""

    def __init__(self, P):
        self.P = P
        self.calls = {"alltoall": 0, "allgather": 0}

    def alltoall(self, chunks):
        # chunks[p][q] (rank p's chunk for rank q) -> out[q][p]
        P = self.P
        self.calls["alltoall"] += 1
        return {q: [chunks[p][q] for p in range(P)] for q in range(P)}

    def allgather(self, parts):
        # parts[p] (rank p's array) -> [parts[0], ..., parts[P-1]]
        self.calls["allgather"] += 1
        return [parts[p] for p in range(self.P)]


class DistComm:
    """One rank of a torch.distributed process group (gloo on CPU)."""

    def __init__(self):
        import torch.distributed as dist
        self.dist = dist
        self.P = dist.get_world_size()
        self.rank = dist.get_rank()
        self.local_ranks = [self.rank]
        self.calls = {"alltoall": 0, "allgather": 0, "halo": 0}

    def alltoall(self, chunks):
        import torch
        self.calls["alltoall"] += 1
        mine = chunks[self.rank]
        shape = mine[0].shape
        send = torch.from_numpy(np.ascontiguousarray(np.stack(mine)).view(np.float64).copy())
        recv = torch.empty_like(send)
        self.dist.all_to_all_single(recv.view(-1), send.view(-1))
        arr = recv.numpy().view(np.complex128).reshape((self.P,) + shape)
        return {self.rank: [arr[p] for p in range(self.P)]}

    def allgather(self, parts):
        import torch
        self.calls["allgather"] += 1
        mine = np.ascontiguousarray(parts[self.rank])
        t = torch.from_numpy(mine.view(np.float64).copy())
        out = [torch.empty_like(t) for _ in range(self.P)]
        self.dist.all_gather(out, t)
        return [o.numpy().view(np.complex128).reshape(mine.shape) for o in out]

    def halo(self, slabs):
        import torch
        self.calls["halo"] += 1
        (w,) = slabs
        P, r = self.P, self.rank
        prev, nxt = (r - 1) % P, (r + 1) % P
        first = torch.from_numpy(np.ascontiguousarray(w[:, 0]))
        last = torch.from_numpy(np.ascontiguousarray(w[:, -1]))
        lo, hi = torch.empty_like(first), torch.empty_like(first)
        # tags give the role, so prev == next (P = 2) is unambiguous
        reqs = [self.dist.isend(first, prev, tag=1), self.dist.isend(last, nxt, tag=2),
                self.dist.irecv(hi, nxt, tag=1), self.dist.irecv(lo, prev, tag=2)]
        for q in reqs:
            q.wait()
        return [(lo.numpy(), hi.numpy())]


def slab_layout(nx, ny, P):
    if ny % P:
        raise ValueError("ny must be divisible by P")
    nxh = nx // 2 + 1
    kb = -(-nxh // P)
    return ny // P, nxh, kb


def pack(X, P, kb):
    """X (nxh, rows) -> S (P, rows, kb) with S[q, jl, kl] = X[q*kb+kl, jl] (0 padding)."""
    nxh, rows = X.shape
    S = np.zeros((P, rows, kb), dtype=np.complex128)
    for q in range(P):
        lo, hi = q * kb, min((q + 1) * kb, nxh)
        if hi > lo:
            S[q, :, :hi - lo] = X[lo:hi, :].T
    return S


def unpack(S, nxh):
    P, rows, kb = S.shape
    X = np.zeros((nxh, rows), dtype=np.complex128)
    for q in range(P):
        lo, hi = q * kb, min((q + 1) * kb, nxh)
        if hi > lo:
            X[lo:hi, :] = S[q, :, :hi - lo].T
    return X


def divide_block(Y, rank, kb, nx, ny, dx, dy, eps, neg):
    """Y[y, kl] / symbol(kx = rank*kb + kl, y); padding and (0,0) -> 0 (Common.jl:118-121)."""
    nxh = nx // 2 + 1
    aa = -2.0 / (dx * dx) - 2.0 / (dy * dy)
    bb = 2.0 / (dx * dx)
    cc = 2.0 / (dy * dy)
    ck = vo.cos_table(vo.kx_table(nx, eps))
    kx = rank * kb + np.arange(kb)
    valid = kx < nxh
    cxv = np.where(valid, ck[np.minimum(kx, nxh - 1)], 1.0)
    d = (aa + bb * cxv[None, :]) + cc * ck[:ny, None]
    v = -Y if neg else Y
    out = np.empty_like(Y)
    out.real = v.real / d
    out.imag = v.imag / d
    out[:, ~valid] = 0.0
    if rank == 0:
        out[0, 0] = 0.0
    return out


def slab_poisson_all(w_slabs, nx, ny, dx, dy, eps, comm, neg=True, workers=1):
    """psi slabs for all ranks of a LocalComm (or the single local rank of a DistComm)."""
    P = comm.P
    rows, nxh, kb = slab_layout(nx, ny, P)
    ranks = getattr(comm, "local_ranks", list(range(P)))
    S = {p: pack(sfft.rfft(w_slabs[i], axis=0, workers=workers), P, kb)
         for i, p in enumerate(ranks)}
    recv = comm.alltoall({p: [S[p][q] for q in range(P)] for p in ranks})
    Ys = {}
    for q in ranks:
        Y = np.concatenate(recv[q], axis=0)  # (ny, kb): y = p*rows + jl
        Y = sfft.fft(Y, axis=0, workers=workers)
        Y = divide_block(Y, q, kb, nx, ny, dx, dy, eps, neg)
        Ys[q] = sfft.ifft(Y, axis=0, workers=workers)
    back = comm.alltoall({q: [Ys[q][p * rows:(p + 1) * rows] for p in range(P)]
                          for q in ranks})
    out = []
    for p in ranks:
        X = unpack(np.stack(back[p], axis=0), nxh)
        out.append(sfft.irfft(X, n=nx, axis=0, workers=workers))
    return out


def slab_poisson_schur(w_slabs, nx, ny, dx, dy, eps, comm, neg=True, workers=1):
    """The substructured y-slab solve (cfdj_vm::poisson_schur, schur.hip): per rank, row
    r2c; all-gather of the x-mode 0 / nx/2 columns (solved by a full y-FFT with the
    reference symbol) and of 4 trace numbers per other x-mode; separator + interior solves;
    row c2r.  Square grids only (oracle/schur_oracle.py)."""
    from . import schur_oracle as so

    P = comm.P
    rows = ny // P
    L = nx // 2
    ranks = getattr(comm, "local_ranks", list(range(P)))
    c = so.mode_constants(nx, ny, dx, dy, P, eps)
    ms, lam = so.interior_lambda(c)
    sgn = -1.0 if neg else 1.0
    F = {p: sfft.rfft(sgn * w_slabs[i], axis=0, workers=workers) for i, p in enumerate(ranks)}
    cols = comm.allgather({p: np.stack([F[p][0], F[p][L]]) for p in ranks})
    G = np.concatenate(cols, axis=1)
    g0, gL = so.column_solve(G[0], c, 0, eps), so.column_solve(G[1], c, L, eps)
    T = comm.allgather({p: so.slab_traces(F[p][ms], lam) for p in ranks})
    out = []
    for p in ranks:
        X = np.empty_like(F[p])
        X[0] = g0[p * rows:(p + 1) * rows]
        X[L] = gL[p * rows:(p + 1) * rows]
        X[ms] = so.slab_solve(F[p][ms], lam, T, p, c, ms, dy, ny)
        out.append(sfft.irfft(X, n=nx, axis=0, workers=workers))
    return out


def slab_poisson_schur_one_gather(w_slabs, nx, ny, dx, dy, eps, comm, neg=True, workers=1):
    """The substructured solve as cfdj_vm::poisson_schur runs it by default: ONE all-gather per
    solve whose block per rank is [3 trace numbers per x-mode 1..L-1][the slab's column sums,
    nx reals, untransformed][its piece of the x-mode 0 and nx/2 columns][its first and last
    input rows]; no other communication.  Returns, per local rank, (psi, psi_lo, psi_hi, w_lo,
    w_hi): the slab and the four halo rows the stencil needs --
      w_lo / w_hi   the neighbours' last / first rows, taken out of the gathered blocks;
      psi_hi        the row after the slab = the next slab's separator row, whose value s_q
                    every rank has from the separator system;
      psi_lo        the row before the slab, from the operator's equation at the slab's own
                    separator row: (psi[-1] + psi[1]) / dy^2 + d_m psi[0] = f[0] per x-mode;
    the x-modes 0 and nx/2 of both rows come from the solved gathered column; the constant-mode
    correction from the transform of the ranks' column sums added up AFTER the gather."""
    from . import schur_oracle as so

    P = comm.P
    rows = ny // P
    L = nx // 2
    ranks = getattr(comm, "local_ranks", list(range(P)))
    c = so.mode_constants(nx, ny, dx, dy, P, eps)
    ms, lam = so.interior_lambda(c)
    sgn = -1.0 if neg else 1.0
    F = {p: sfft.rfft(sgn * w_slabs[i], axis=0, workers=workers) for i, p in enumerate(ranks)}

    def block(i, p):
        tr = so.slab_traces(F[p][ms], lam)[:3]  # separator row, the two interior traces
        cs = (sgn * w_slabs[i]).sum(axis=1)      # column sums of the slab, physical space
        return np.concatenate([tr.ravel(), cs.astype(np.complex128), F[p][0], F[p][L],
                               w_slabs[i][:, 0].astype(np.complex128),
                               w_slabs[i][:, -1].astype(np.complex128)])

    blocks = comm.allgather({p: block(i, p) for i, p in enumerate(ranks)})
    nm = len(ms)
    o_cs, o_c0, o_cL, o_w0, o_w1 = 3 * nm, 3 * nm + nx, 3 * nm + nx + rows, \
        3 * nm + nx + 2 * rows, 3 * nm + 2 * nx + 2 * rows
    T = [b[:o_cs].reshape(3, nm) for b in blocks]
    cs_hat = sfft.rfft(sum(b[o_cs:o_c0].real for b in blocks))[ms]  # rank 0 first
    g0 = so.column_solve(np.concatenate([b[o_c0:o_cL] for b in blocks]), c, 0, eps)
    gL = so.column_solve(np.concatenate([b[o_cL:o_w0] for b in blocks]), c, L, eps)
    dy2 = dy * dy
    out = []
    for i, p in enumerate(ranks):
        # slab_solve wants the column sums per rank in T[q][3]: hand it the total once
        T4 = [np.vstack([T[q], cs_hat if q == 0 else np.zeros(nm)]) for q in range(P)]
        core = so.slab_solve(F[p][ms], lam, T4, p, c, ms, dy, ny)
        cst = (cs_hat / ny) * c["corr"][ms]
        X = np.empty_like(F[p])
        X[0] = g0[p * rows:(p + 1) * rows]
        X[L] = gL[p * rows:(p + 1) * rows]
        X[ms] = core
        psi = sfft.irfft(X, n=nx, axis=0, workers=workers)
        # the two rows just outside the slab
        rhs = np.stack([T[q][0] - (T[(q - 1) % P][2] + T[q][1]) / dy2 for q in range(P)])
        sq = np.einsum("mq,qm->m", c["minv"][ms][:, (p + 1) % P, :], rhs)
        u0, u1 = core[:, 0] - cst, core[:, 1] - cst  # T^{-1} f at rows 0 and 1
        lo = dy2 * (F[p][ms, 0] - c["d"][ms] * u0) - u1
        Xlo, Xhi = np.zeros(L + 1, dtype=np.complex128), np.zeros(L + 1, dtype=np.complex128)
        Xlo[ms], Xhi[ms] = lo + cst, sq + cst
        jlo, jhi = (p * rows - 1) % ny, ((p + 1) * rows) % ny
        Xlo[0], Xlo[L], Xhi[0], Xhi[L] = g0[jlo], gL[jlo], g0[jhi], gL[jhi]
        w_lo = blocks[(p - 1) % P][o_w1:].real
        w_hi = blocks[(p + 1) % P][o_w0:o_w1].real
        out.append((psi, sfft.irfft(Xlo, n=nx), sfft.irfft(Xhi, n=nx), w_lo, w_hi))
    return out


def slab_rk3_step_one_gather(wn, dt, nx, ny, dx, dy, re, eps, comm):
    """One RK3 step whose only communication is the solve's all-gather, three per step
    (slab_poisson_schur_one_gather): the stencil's halo rows come with the solve."""

    def rhs(w):
        out = []
        for wi, (s, sl, sh, wl, wh) in zip(w, slab_poisson_schur_one_gather(
                w, nx, ny, dx, dy, eps, comm)):
            we = np.concatenate([wl[:, None], wi, wh[:, None]], axis=1)
            se = np.concatenate([sl[:, None], s, sh[:, None]], axis=1)
            out.append(vo.arakawa_rhs(we, se, dx, dy, re)[:, 1:-1])
        return out

    r = rhs(wn)
    wt = [a + dt * b for a, b in zip(wn, r)]
    r = rhs(wt)
    wt = [(0.75 * a + 0.25 * b) + (0.25 * dt) * c for a, b, c in zip(wn, wt, r)]
    r = rhs(wt)
    return [(a / 3.0 + (2.0 / 3.0) * b) + ((2.0 / 3.0) * dt) * c for a, b, c in zip(wn, wt, r)]


def halo_rows(slabs, comm):
    """(lo, hi) ghost rows per local rank: lo = last row of p-1, hi = first row of p+1."""
    if hasattr(comm, "halo"):
        return comm.halo(slabs)
    P = comm.P
    return [(slabs[(p - 1) % P][:, -1], slabs[(p + 1) % P][:, 0]) for p in range(P)]


def slab_rhs(w_slabs, psi_slabs, dx, dy, re, comm):
    hw = halo_rows(w_slabs, comm)
    hs = halo_rows(psi_slabs, comm)
    out = []
    for w, s, (wl, wh), (sl, sh) in zip(w_slabs, psi_slabs, hw, hs):
        we = np.concatenate([wl[:, None], w, wh[:, None]], axis=1)
        se = np.concatenate([sl[:, None], s, sh[:, None]], axis=1)
        out.append(vo.arakawa_rhs(we, se, dx, dy, re)[:, 1:-1])
    return out


def slab_rk3_step(wn, dt, nx, ny, dx, dy, re, eps, comm, poisson="transpose"):
    solve = slab_poisson_schur if poisson == "schur" else slab_poisson_all

    def rhs(w):
        return slab_rhs(w, solve(w, nx, ny, dx, dy, eps, comm), dx, dy, re, comm)

    r = rhs(wn)
    wt = [a + dt * b for a, b in zip(wn, r)]
    r = rhs(wt)
    wt = [(0.75 * a + 0.25 * b) + (0.25 * dt) * c for a, b, c in zip(wn, wt, r)]
    r = rhs(wt)
    return [(a / 3.0 + (2.0 / 3.0) * b) + ((2.0 / 3.0) * dt) * c for a, b, c in zip(wn, wt, r)]


def split(w, P):
    rows = w.shape[1] // P
    return [np.array(w[:, p * rows:(p + 1) * rows]) for p in range(P)]
