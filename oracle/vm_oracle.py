"""CPU oracle: NumPy/SciPy restatement of the reference's 2D vorticity-streamfunction
Navier-Stokes hot path (t-bltg/CFD_Julia, `Common.jl` + `19_NS2D_Vortex_Merger/vm.jl`).

TEST INFRASTRUCTURE ONLY.  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg may import this module, and only as the checker / the timed CPU
baseline.  The product path (`cfd_julia_amd`, `libcfdj.so`) never imports or calls it.

Parity pinning: the Julia reference cannot run in this image (no `julia`,
unregistered `Unroll`/`Utils` deps, unpinned FFTW.jl).  This restatement is pinned by
  * the only published numbers of the reference: the FD-FFT Poisson L2 errors hard-coded
    at `13_Poisson_Solver_FFT_Spectral/specrtral_vs_FDM/order.jl:11` (fft_p.jl MMS,
    N = 32..512) -- reproduced to <= 3e-12 relative by `fft_p_mms_error` below;
  * the spectral Poisson errors at `order.jl:10` (fft_s.jl) -- round-off level;
  * the analytic Taylor-Green decay used by `19_NS2D_Vortex_Merger/tgv.jl:82-90`;
  * the qualitative peak vorticity ~0.74 at 128^2, t = 20 (`Python_Vectorized/field_fdm.png`).
The vortex-merger field itself has no stored golden vector in the reference: for it the
parity is "pinned by the KATs above", not by reference output.

Conventions: fields are periodic nx-by-ny arrays indexed [i, j] with i along x (Julia's
first, contiguous dimension), 0-based, WITHOUT ghost layers.  Element [i, j] here is the
reference's w[i+2, j+2] (Julia 1-based, ghosted).  `to_ghosted` / `from_ghosted` convert.
Floating-point evaluation order mirrors the reference source text exactly (no FMA:
NumPy never contracts), so the GPU kernels compiled with -ffp-contract=off reproduce the
stencil and the spectral divide bit-for-bit; only the FFT implementations differ
(pocketfft here, FFTW in the reference, rocFFT on the GPU).
"""
from __future__ import annotations

import math
import os

import numpy as np
import scipy.fft as sfft

TWO_PI = 2 * math.pi  # Julia `2π` == Float64(2) * Float64(π)


def _workers(workers):
    return os.cpu_count() if workers is None else workers


# --------------------------------------------------------------------------------------
# Grid / IC  (vm.jl:93-128, Common.jl:208-219)
# --------------------------------------------------------------------------------------
def vm_grid(nx, ny, x_l=0.0, x_r=TWO_PI, y_b=0.0, y_t=TWO_PI):
    """vm.jl:94-115: Δx = (x_r-x_l)/nx, x[i] = Δx(i-1) for i = 1..nx+1."""
    dx = (x_r - x_l) / nx
    dy = (y_t - y_b) / ny
    x = dx * np.arange(nx + 1, dtype=np.float64)
    y = dy * np.arange(ny + 1, dtype=np.float64)
    return dx, dy, x, y


def vm_ic(nx, ny, x, y):
    """Common.jl:208-219 (vm_ic): two Gaussian vortices, σ = π, centres (π ∓ π/4, π).

    Returns the periodic interior nx-by-ny field (reference w[2:nx+1, 2:ny+1]); the
    reference also evaluates column/row nx+2 but vm.jl:121-128 overwrites it with the
    periodic copy, so the interior is authoritative."""
    sigma = math.pi
    xc1, yc1 = math.pi - math.pi / 4.0, math.pi
    xc2, yc2 = math.pi + math.pi / 4.0, math.pi
    X = x[:nx, None]
    Y = y[None, :ny]
    return (np.exp(-sigma * ((X - xc1) ** 2 + (Y - yc1) ** 2))
            + np.exp(-sigma * ((X - xc2) ** 2 + (Y - yc2) ** 2)))


def to_ghosted(w):
    """Interior (nx, ny) -> reference (nx+2, ny+2) array, Fortran order (Julia layout),
    ghosts filled in the order of vm.jl:121-128 (all periodic copies)."""
    nx, ny = w.shape
    g = np.zeros((nx + 2, ny + 2), dtype=np.float64, order="F")
    g[1:nx + 1, 1:ny + 1] = w
    g[0, :] = g[nx, :]
    g[:, 0] = g[:, ny]
    g[nx + 1, :] = g[1, :]
    g[:, ny + 1] = g[:, 1]
    return g


def from_ghosted(g):
    return np.array(g[1:-1, 1:-1], dtype=np.float64)


def with_duplicate_node(w):
    """Interior (nx, ny) -> the (nx+1, ny+1) array vm.jl:89 returns (wn[2:nx+2, 2:ny+2])."""
    nx, ny = w.shape
    out = np.empty((nx + 1, ny + 1), dtype=np.float64, order="F")
    out[:nx, :ny] = w
    out[nx, :ny] = w[0, :]
    out[:nx, ny] = w[:, 0]
    out[nx, ny] = w[0, 0]
    return out


# --------------------------------------------------------------------------------------
# FFT Poisson (Common.jl:97-125 `fps`, 12_Poisson_Solver_FFT/fft_p.jl:8-42 `ps_fft`)
# --------------------------------------------------------------------------------------
def kx_table(nx, eps=1e-6):
    """Common.jl:106-113: hx = 2π/nx; kx[i] = hx(i-1) (i ≤ nx/2), kx[i+nx/2] = hx(i-nx/2-1);
    kx[1] = ε.  0-based here: kx[0] = ε, kx[m] = hx·m (m < nx/2), kx[m] = hx·(m-nx) (m ≥ nx/2)."""
    if nx % 2:
        raise ValueError("fps requires even nx (Common.jl:108 loops to nx÷2)")
    hx = TWO_PI / nx
    h = nx // 2
    kx = np.empty(nx, dtype=np.float64)
    for i in range(1, h + 1):
        kx[i - 1] = hx * float(i - 1)
        kx[i + h - 1] = hx * float(i - h - 1)
    kx[0] = eps
    return kx


def cos_table(k):
    # math.cos (glibc, correctly rounded in practice) -- not np.cos, whose SIMD kernels
    # may differ by an ulp; the GPU tables are built with the same libm on the host.
    return np.array([math.cos(v) for v in k], dtype=np.float64)


def fps_denominator(nx, ny, dx, dy, eps=1e-6):
    """aa + bb·cos(kx_i) + cc·cos(ky_j) with ky = kx (Common.jl:101-103,113,120)."""
    if ny > nx:
        raise IndexError("Common.jl:113 aliases ky = kx: ny > nx is a BoundsError")
    aa = -2.0 / (dx * dx) - 2.0 / (dy * dy)
    bb = 2.0 / (dx * dx)
    cc = 2.0 / (dy * dy)
    ck = cos_table(kx_table(nx, eps))
    return (aa + bb * ck[:, None]) + cc * ck[None, :ny]


def _cdiv_real(e, d):
    # Julia Complex/Real divides each component (not numpy's Smith complex division).
    out = np.empty(e.shape, dtype=np.complex128)
    out.real = e.real / d
    out.imag = e.imag / d
    return out


def fps(f, dx, dy, eps=1e-6, workers=None):
    """Common.jl:97-125: returns s[2:nx+1, 2:ny+1] (the interior) for ∇²s = f."""
    nx, ny = f.shape
    den = fps_denominator(nx, ny, dx, dy, eps)
    e = sfft.fft2(f.astype(np.complex128), workers=_workers(workers))
    e[0, 0] = 0.0
    data1 = _cdiv_real(e, den)
    return sfft.ifft2(data1, workers=_workers(workers)).real.copy()


ps_fft = fps  # fft_p.jl:8-42 is the same arithmetic, returning real(ifft) nx-by-ny


def ps_spectral(f, dx, dy, eps=1e-6, workers=None):
    """13_Poisson_Solver_FFT_Spectral/fft_s.jl:8-37: divisor -(kx²+ky²), hx = 2π/(nx·Δx)."""
    nx, ny = f.shape
    hx = TWO_PI / (nx * dx)
    h = nx // 2
    kx = np.empty(nx)
    for i in range(1, h + 1):
        kx[i - 1] = hx * float(i - 1)
        kx[i + h - 1] = hx * float(i - h - 1)
    kx[0] = eps
    ky = kx
    e = sfft.fft2(f.astype(np.complex128), workers=_workers(workers))
    e[0, 0] = 0.0
    den = -(kx[:, None] ** 2 + ky[None, :ny] ** 2)
    return sfft.ifft2(_cdiv_real(e, den), workers=_workers(workers)).real.copy()


def compute_l2norm_bnds(r):
    """Common.jl:234-237: sqrt(Σ r[1:nx+1,1:ny+1]² / ((nx+1)(ny+1)))."""
    return math.sqrt(float(np.sum(r * r)) / r.size)


def fft_d_order_tolerance(nx, ref):
    """Relative tolerance for comparing the L2 error of 14/fft_d.jl's DST-I solve with the
    order.jl:11 value `ref` of 12/fft_p.jl on the same manufactured solution: 1e-9, or --
    on the finer grids -- the rounding of the two scripts' symbols, which cancel from
    O(nx^2) terms to 8 pi^2 for the dominant mode (relative error 4 nx^2 eps / (8 pi^2) of
    the mode's unit amplitude, seen in an error norm of size ref)."""
    sym = 4.0 * nx * nx * np.finfo(np.float64).eps / (8.0 * math.pi ** 2)
    return max(1e-9, sym / ref)


def fft_p_mms(nx, km=16):
    """fft_p.jl:45-82 MMS on [0,1]² (returns f, ue on the (nx+1)² node grid, and Δx)."""
    ny = nx
    dx = 1.0 / nx
    dy = 1.0 / ny
    x = 0.0 + dx * np.arange(nx + 1)
    y = 0.0 + dy * np.arange(ny + 1)
    c1 = (1.0 / km) ** 2
    c2 = -8 * math.pi ** 2
    X, Y = x[:, None], y[None, :]
    ue = (np.sin(TWO_PI * X) * np.sin(TWO_PI * Y)
          + c1 * np.sin(km * TWO_PI * X) * np.sin(km * TWO_PI * Y))
    f = (c2 * np.sin(TWO_PI * X) * np.sin(TWO_PI * Y)
         + c2 * np.sin(km * TWO_PI * X) * np.sin(km * TWO_PI * Y))
    return f, ue, dx, dy


def fft_p_mms_error(nx, solver=None):
    """fft_p.jl:90-101: solve on the nx² periodic part, copy the periodic node, L2 error.
    `solver(f_interior, dx, dy) -> u` defaults to this oracle's `ps_fft`."""
    f, ue, dx, dy = fft_p_mms(nx)
    solver = solver or ps_fft
    un = np.zeros_like(f)
    un[:nx, :nx] = solver(np.ascontiguousarray(f[:nx, :nx]), dx, dy)
    un[nx, :] = un[0, :]
    un[:, nx] = un[:, 0]
    err = un - ue
    return compute_l2norm_bnds(err), float(np.max(np.abs(err)))


# Published reference errors (order.jl:10-11), N = 32, 64, 128, 256, 512.
ORDER_JL_GRID = (32, 64, 128, 256, 512)
ORDER_JL_FFT_FDM = (0.0015607100315532957, 0.0005987381110678801, 0.00014313734718665358,
                    3.549617203207291e-5, 8.865373334924762e-6)
ORDER_JL_FFT_SPECTRAL = (1.339154672220572e-16, 1.342489800590083e-16,
                         1.3269947532677886e-16, 1.4514549677756118e-16,
                         1.485803753784319e-16)


# --------------------------------------------------------------------------------------
# Arakawa Jacobian + 5-point Laplacian (Common.jl:148-181)
# --------------------------------------------------------------------------------------
def vm_coefs(dx, dy, re):
    """Common.jl:149-152."""
    aa = 1.0 / (re * (dx * dx))
    bb = 1.0 / (re * (dy * dy))
    gg = 1.0 / ((4 * dx) * dy)
    hh = 1.0 / 3.0
    return aa, bb, gg, hh


def arakawa_rhs(w, s, dx, dy, re):
    """r = -J_Arakawa(w, s) + (1/re)∇²w on the periodic grid, float order of
    Common.jl:154-181 (j1, j2, j3 left-associated; jac = gg*(j1+j2+j3)*hh)."""
    aa, bb, gg, hh = vm_coefs(dx, dy, re)
    R = np.roll
    wE, wW = R(w, -1, 0), R(w, 1, 0)          # w[i+1,j], w[i-1,j]
    wN, wS = R(w, -1, 1), R(w, 1, 1)          # w[i,j+1], w[i,j-1]
    wNE, wSE = R(wE, -1, 1), R(wE, 1, 1)      # w[i+1,j+1], w[i+1,j-1]
    wNW, wSW = R(wW, -1, 1), R(wW, 1, 1)      # w[i-1,j+1], w[i-1,j-1]
    sE, sW = R(s, -1, 0), R(s, 1, 0)
    sN, sS = R(s, -1, 1), R(s, 1, 1)
    sNE, sSE = R(sE, -1, 1), R(sE, 1, 1)
    sNW, sSW = R(sW, -1, 1), R(sW, 1, 1)
    j1 = (wE - wW) * (sN - sS) - (wN - wS) * (sE - sW)
    j2 = wE * (sNE - sSE) - wW * (sNW - sSW) - wN * (sNE - sNW) + wS * (sSE - sSW)
    j3 = wNE * (sN - sE) - wSW * (sW - sS) - wNW * (sN - sW) + wSE * (sE - sS)
    jac = gg * (j1 + j2 + j3) * hh
    return -jac + (aa * (wE - 2 * w + wW) + bb * (wN - 2 * w + wS))


def vm_rhs(w, dx, dy, re, eps=1e-6, workers=None):
    """Common.jl:132-182: f = -w; s = fps(f); r = -J(w,s) + ν∇²w.  Returns (r, s)."""
    s = fps(-w, dx, dy, eps, workers)
    return arakawa_rhs(w, s, dx, dy, re), s


# --------------------------------------------------------------------------------------
# SSP-RK3 time loop (vm.jl:12-90)
# --------------------------------------------------------------------------------------
def rk3_step(wn, dt, dx, dy, re, eps=1e-6, workers=None):
    """One Shu-Osher RK3 step, stage formulas and float order of vm.jl:26-76."""
    r, _ = vm_rhs(wn, dx, dy, re, eps, workers)
    wt = wn + dt * r                                            # vm.jl:28
    r, _ = vm_rhs(wt, dx, dy, re, eps, workers)
    wt = (0.75 * wn + 0.25 * wt) + (0.25 * dt) * r              # vm.jl:43-47
    r, _ = vm_rhs(wt, dx, dy, re, eps, workers)
    return (wn / 3.0 + (2.0 / 3.0) * wt) + ((2.0 / 3.0) * dt) * r  # vm.jl:62-66


def numerical(wn, nt, dt, dx, dy, re, eps=1e-6, workers=None, callback=None):
    """vm.jl:12-90 without the text snapshots; returns the interior after nt steps."""
    w = np.array(wn, dtype=np.float64)
    for k in range(1, nt + 1):
        w = rk3_step(w, dt, dx, dy, re, eps, workers)
        if callback is not None:
            callback(k, w)
    return w


def exact_tgv(x, y, time, re, nq=4):
    """tgv.jl:82-90: ω = 2nq·cos(nq x)cos(nq y)·exp(-2nq² t / re) on the (nx+1)² nodes."""
    return (2 * nq * np.cos(nq * x[:, None]) * np.cos(nq * y[None, :])
            * math.exp(-2 * nq ** 2 * time / re))


def tgv_error(nx=64, re=10.0, dt=0.01, tf=1.0, stepper=None):
    """tgv.jl:92-139: run the vm RK3 loop on Taylor-Green; returns (L2, Linf) errors."""
    dx, dy, x, y = vm_grid(nx, nx)
    nt = int(round(tf / dt))
    w0 = exact_tgv(x, y, 0.0, re)[:nx, :nx].copy()
    if stepper is None:
        w = numerical(w0, nt, dt, dx, dy, re)
    else:
        w = stepper(w0, nt, dt, dx, dy, re)
    un = with_duplicate_node(w)
    ue = exact_tgv(x, y, tf, re)
    err = un - ue
    return compute_l2norm_bnds(err), float(np.max(np.abs(err)))
