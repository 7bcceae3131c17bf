"""TEST INFRASTRUCTURE ONLY -- never imported by the product path (cfd_julia_amd/).

CPU restatement of the multi-GPU Poisson decomposition that libcfdj.so runs on y-slabs
(DESIGN.md §5): the reference's periodic FD-FFT solve (Common.jl:97-125, restated in
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


def schur_fps(f, dx, dy, P, eps=1e-6):
    """Decomposed solve of vm_oracle.fps(f, dx, dy) on P y-slabs (single process)."""
    nx, ny = f.shape
    if nx != ny:
        raise ValueError("substructured y-solve needs nx == ny (see module docstring)")
    c = mode_constants(nx, ny, dx, dy, P, eps)
    rl, n = c["rl"], c["n"]
    F = np.fft.rfft(f, axis=0)  # F[m, y], m = 0..nx/2
    out = np.empty_like(F)
    # modes 0 and nx/2: full y-FFT with the reference symbol (the gathered column)
    ky = vo.cos_table(vo.kx_table(nx, eps))[:ny]
    for m in (0, nx // 2):
        col = np.fft.fft(F[m, :])
        if m == 0:
            col[0] = 0.0  # e[1,1] = 0 (Common.jl:118)
        den = (c["aa"] + c["bb"] * c["cx"][m]) + c["cc"] * ky
        out[m, :] = np.fft.ifft(vo._cdiv_real(col, den))
    ms = np.arange(1, nx // 2)
    d = c["d"][ms]
    kk = np.arange(1, n + 1)
    lam = d[:, None] + c["cc"] * np.cos(np.pi * kk / rl)[None, :]
    dy2 = dy * dy
    # pass A: interior traces with zero boundaries; separator right-hand sides
    t1 = np.empty((P, ms.size), complex)
    tn = np.empty((P, ms.size), complex)
    fs = np.empty((P, ms.size), complex)
    for p in range(P):
        blk = F[ms, p * rl:(p + 1) * rl]
        psi0 = _dst_solve(blk[:, 1:], lam)
        t1[p], tn[p], fs[p] = psi0[:, 0], psi0[:, -1], blk[:, 0]
    rhs = fs - (np.roll(tn, 1, axis=0) + t1) / dy2  # tn[p-1] + t1[p]
    s = np.einsum("mpq,qm->pm", c["minv"][ms], rhs)
    fbar = F[ms, :].mean(axis=1)
    # pass B: interior with the separator values as Dirichlet data, + constant-mode fix
    for p in range(P):
        blk = F[ms, p * rl:(p + 1) * rl].copy()
        sp, sq = s[p], s[(p + 1) % P]
        r = blk[:, 1:]
        r[:, 0] -= sp / dy2
        r[:, -1] -= sq / dy2
        psi = np.empty_like(blk)
        psi[:, 0] = sp
        psi[:, 1:] = _dst_solve(r, lam)
        out[ms, p * rl:(p + 1) * rl] = psi + (fbar * c["corr"][ms])[:, None]
    return np.fft.irfft(out, n=nx, axis=0)
