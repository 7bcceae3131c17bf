"""TEST INFRASTRUCTURE ONLY -- never imported by the product path (cfd_julia_amd/).

CPU restatement of the multi-GPU Poisson decomposition that libcfdj.so runs on y-slabs:
the reference's periodic FD-FFT solve (Common.jl:97-125, restated in
vm_oracle.fps) rewritten as

  1. real FFT along x (local to a y-slab);
  2. per x-mode m >= 1, the y-direction operator of the reference symbol,
        psi[j-1]/dy^2 + d_m psi[j] + psi[j+1]/dy^2,   d_m = aa + bb cos(kx_m),
     which is the periodic tridiagonal circulant whose eigenvalues are
     d_m + cc cos(2 pi k / ny) -- EXCEPT at k = 0, where Common.jl's ky[1] = eps makes the
     reference eigenvalue d_m + cc cos(eps).  That is a rank-one (constant-mode) change,
     applied exactly: psi = T^{-1} f + mean(f) (1/D_ref - 1/D_tri).
     T^{-1} f is solved by substructuring: rank p owns rows [p rl, (p+1) rl); row p rl is
     its separator, rows p rl + 1 .. p rl + rl - 1 its interior (rl - 1 unknowns, a
     Dirichlet block diagonalised by the DST-I = an FFT of length 2 rl on the odd
     extension).  Interior traces + separator values of all ranks (O(nx P) numbers, not
     the O(nx ny) of a transpose) give a P x P periodic system for the separator values;
     a second interior solve with those boundary values completes psi;
  3. the x-modes m = 0 (kx = eps) and m = nx/2 (the real DC / Nyquist columns, which the
     GPU packs into one complex column) are solved with the reference symbol by a full
     FFT along y after gathering that one column (e[1,1] = 0 included);
  4. inverse real FFT along x.

Equal to vm_oracle.fps up to round-off for nx == ny (for ny < nx the reference's
ky = kx aliasing gives a symbol that is not a y-stencil, so this decomposition applies to
square grids only -- the library then uses the all-to-all transpose path).
"""
import math

import numpy as np
import scipy.fft as sfft

from oracle import vm_oracle as vo


def mode_constants(nx, ny, dx, dy, P, eps=1e-6):
    """Per x-mode constants shared by every rank: d_m, the Dirichlet-block Green's
    function corner values a1 = T_int^{-1}[1,1], an = T_int^{-1}[1,n] and the inverse of the
    P x P separator system.  Long-double sums (the GPU library builds the same tables on
    the host in long double)."""
    rl = ny // P
    n = rl - 1
    aa = -2.0 / (dx * dx) - 2.0 / (dy * dy)
    bb = 2.0 / (dx * dx)
    cc = 2.0 / (dy * dy)
    cx = vo.cos_table(vo.kx_table(nx, eps))[: nx // 2 + 1]
    d = aa + bb * cx
    k = np.arange(1, n + 1, dtype=np.longdouble)
    pi = np.longdouble(math.pi)
    s2 = np.sin(pi * k / rl) ** 2
    lam = d.astype(np.longdouble)[:, None] + np.longdouble(cc) * np.cos(pi * k / rl)[None, :]
    a1 = (2.0 / np.longdouble(rl)) * np.sum(s2[None, :] / lam, axis=1)
    sgn = np.where(k.astype(np.int64) % 2 == 1, 1.0, -1.0).astype(np.longdouble)
    an = (2.0 / np.longdouble(rl)) * np.sum((sgn * s2)[None, :] / lam, axis=1)
    dy2 = np.longdouble(dy) * np.longdouble(dy)
    diag = d.astype(np.longdouble) - 2.0 * a1 / (dy2 * dy2)
    off = -an / (dy2 * dy2)
    # the periodic separator system is circulant: invert through its eigenvalues
    # mu_j = diag + 2 off cos(2 pi j / P), in long double -- diag and off are O(1/dy^2)
    # while the smallest mu is O(1), so a double-precision inverse loses ~log10(1/dy^2)
    # digits to cancellation
    j = np.arange(P, dtype=np.longdouble)
    mu = diag[:, None] + 2.0 * off[:, None] * np.cos(2.0 * pi * j / P)[None, :]
    L = nx // 2 + 1
    minv = np.zeros((L, P, P))
    for dpq in range(P):
        col = np.sum(np.cos(2.0 * pi * j * dpq / P)[None, :] / mu, axis=1) / P
        for p in range(P):
            minv[:, p, (p + dpq) % P] = col.astype(np.float64)
    minv[0] = 0.0  # mode 0 is solved by the gathered-column FFT
    d_ref0 = (aa + bb * cx) + cc * math.cos(eps)  # reference D(m, 0), Common.jl:120 order
    d_tri0 = d + cc
    return dict(rl=rl, n=n, aa=aa, bb=bb, cc=cc, cx=cx, d=d, a1=a1.astype(np.float64),
                an=an.astype(np.float64), minv=minv, corr=1.0 / d_ref0 - 1.0 / d_tri0)


def _dst_solve(rhs, lam):
    """Interior Dirichlet solve along axis 1 (rows 1..n of a slab): DST-I diagonalisation."""
    return sfft.idst(sfft.dst(rhs, type=1, axis=1) / lam, type=1, axis=1)


def interior_lambda(c):
    ms = np.arange(1, len(c["d"]) - 1)
    kk = np.arange(1, c["n"] + 1)
    return ms, c["d"][ms][:, None] + c["cc"] * np.cos(np.pi * kk / c["rl"])[None, :]


def column_solve(col, c, m, eps=1e-6):
    """x-mode m in {0, nx/2}: the gathered full column, FFT along y, reference symbol."""
    ny = col.size
    ky = vo.cos_table(vo.kx_table(2 * (len(c["d"]) - 1), eps))[:ny]
    z = np.fft.fft(col)
    if m == 0:
        z[0] = 0.0  # e[1,1] = 0 (Common.jl:118)
    den = (c["aa"] + c["bb"] * c["cx"][m]) + c["cc"] * ky
    return np.fft.ifft(vo._cdiv_real(z, den))


def slab_traces(blk, lam):
    """Pass 0 of one slab (x-modes 1..L-1 as rows of `blk`): separator row, interior traces of
    the zero-Dirichlet solve, column sum -> (4, L-1)."""
    psi0 = _dst_solve(blk[:, 1:], lam)
    return np.stack([blk[:, 0], psi0[:, 0], psi0[:, -1], blk.sum(axis=1)])


def slab_solve(blk, lam, T, rank, c, ms, dy, ny):
    """Pass 1 of slab `rank` given the traces T[q] of every rank: separator values from the
    circulant inverse, interior solve with them as Dirichlet data, constant-mode fix."""
    P = len(T)
    dy2 = dy * dy
    rhs = np.stack([T[q][0] - (T[(q - 1) % P][2] + T[q][1]) / dy2 for q in range(P)])
    minv = c["minv"][ms]  # (L-1, P, P)
    sp = np.einsum("mq,qm->m", minv[:, rank, :], rhs)
    sq = np.einsum("mq,qm->m", minv[:, (rank + 1) % P, :], rhs)
    fbar = sum(T[q][3] for q in range(P)) / ny
    r = blk[:, 1:].copy()
    r[:, 0] -= sp / dy2
    r[:, -1] -= sq / dy2
    psi = np.empty_like(blk)
    psi[:, 0] = sp
    psi[:, 1:] = _dst_solve(r, lam)
    return psi + (fbar * c["corr"][ms])[:, None]


def schur_fps(f, dx, dy, P, eps=1e-6):
    """Decomposed solve of vm_oracle.fps(f, dx, dy) on P y-slabs (single process)."""
    nx, ny = f.shape
    if nx != ny:
        raise ValueError("substructured y-solve needs nx == ny (see module docstring)")
    c = mode_constants(nx, ny, dx, dy, P, eps)
    rl = c["rl"]
    F = np.fft.rfft(f, axis=0)  # F[m, y], m = 0..nx/2
    out = np.empty_like(F)
    for m in (0, nx // 2):
        out[m, :] = column_solve(F[m, :], c, m, eps)
    ms, lam = interior_lambda(c)
    blks = [F[ms, p * rl:(p + 1) * rl] for p in range(P)]
    T = [slab_traces(b, lam) for b in blks]
    for p in range(P):
        out[ms, p * rl:(p + 1) * rl] = slab_solve(blks[p], lam, T, p, c, ms, dy, ny)
    return np.fft.irfft(out, n=nx, axis=0)
