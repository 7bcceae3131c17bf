"""CPU oracle: NumPy/SciPy restatement of the reference's spectral-space NS2D solvers,
`20_NS2D_Hybrid_Solver/hybrid.jl`, `21_NS2D_PseudoSpectral_32_Rule/pseudospectral_32_rule.jl`
and `22_NS2D_PseudoSpectral_23_Rule/pseudospectral_23_rule.jl`.

TEST INFRASTRUCTURE ONLY.  Only `tests/` may import this module, as the checker of
libcfdj.so's `cfdj_spec_*` handle; the product path never imports or calls it.

All three scripts share one time loop (hybrid.jl:14-86 = pseudospectral_*.jl:13-89): the
vorticity lives in Fourier space as a full complex nx-by-ny array (`fft` of the real
field, [0, 0] zeroed), advanced by a low-storage RK3 with Crank-Nicolson viscosity,
d_k = α_k (.5Δt k² / re); they differ only in `jacobian` (jf = fft(-J(w, ψ))):
  * hybrid.jl:92-152      -- ψ̂ = ŵ / k², w and ψ back to physical space, the Arakawa
                             Jacobian (per-term gg, Common.jl's stencil), forward FFT;
  * pseudospectral_23_rule.jl:95-144 -- ψ_x, w_y, ψ_y, w_x as spectral derivatives, the
                             modes beyond 2/3 of the grid zeroed, products in physical space;
  * pseudospectral_32_rule.jl:94-186 -- the same derivatives zero-padded to a 3/2-size
                             grid (quadrant copies), products there, truncated back.
Complex arrays throughout, `real(ifft(...))` as written (the reference never assumes
Hermitian symmetry, and its ε at kx[1] and its Nyquist derivatives are not Hermitian).

Parity pinning: the reference cannot run here (no `julia`) and ships no
output for these scripts, so this restatement is pinned by known answers instead:
  * Taylor-Green (tgv.jl:82-90's ω = 2n cos(nx) cos(ny)): the Jacobian is zero (ω = 2n²ψ
    is a function of ψ), so every solver must reproduce the scheme's exact viscous decay
    Π_k (1 - d_k)/(1 + d_k) (tests/test_oracle.py);
  * the three Jacobians agree with each other and with vm_oracle's FD Arakawa to the
    truncation error on smooth fields, and the pseudospectral ones are exact for a
    product of two band-limited modes.
Floating-point order follows the source text (Julia Real*Complex and Complex/Real act
componentwise); the reference marks these loops @fastmath, so its own rounding is not
pinned either -- the GPU is compared to this oracle with a 1e-10 tolerance.
"""
from __future__ import annotations

import numpy as np
import scipy.fft as sfft

from oracle.vm_oracle import TWO_PI

HYBRID, PS23, PS32 = 0, 1, 2
ALPHA = (8.0 / 15.0, 2.0 / 15.0, 1.0 / 3.0)   # hybrid.jl:30
GAMMA = (8.0 / 15.0, 5.0 / 12.0, 3.0 / 4.0)   # hybrid.jl:31
RHO = (None, -17.0 / 60.0, -5.0 / 12.0)        # hybrid.jl:32


def wave_kx(nx, dx, eps=1e-6):
    """Common.jl:184-203 / pseudospectral_*.jl:96-106: hx = 2π/(nx Δx);
    kx[i] = hx(i-1), kx[i+nx/2] = hx(i-nx/2-1); kx[1] = ε.  0-based here."""
    hx = TWO_PI / (nx * dx)
    h = nx // 2
    kx = np.empty(nx, dtype=np.float64)
    for i in range(1, h + 1):
        kx[i - 1] = hx * (i - 1.0)
        kx[i + h - 1] = hx * float(i - h - 1)
    kx[0] = eps
    return kx


def wavespace(nx, ny, dx, dy, eps=1e-6):
    """Common.jl:184-203: k2[i, j] = kx[i]^2 + ky[j]^2 with ky = kx (square grids)."""
    if ny != nx:
        raise ValueError("the spectral solvers alias ky = kx: square grids only")
    kx = wave_kx(nx, dx, eps)
    return kx[:, None] * kx[:, None] + (kx * kx)[None, :]


def _cdiv(e, d):
    out = np.empty(np.broadcast(e, d).shape, dtype=np.complex128)
    out.real = e.real / d
    out.imag = e.imag / d
    return out


def _cmul(a, e):
    """Real * Complex, componentwise (Julia)."""
    out = np.empty(np.broadcast(a, e).shape, dtype=np.complex128)
    out.real = a * e.real
    out.imag = a * e.imag
    return out


def _times_i(e):
    out = np.empty(e.shape, dtype=np.complex128)
    out.real = -e.imag
    out.imag = e.real
    return out


def _ifft_real(f):
    return np.ascontiguousarray(sfft.ifft2(f, axes=(0, 1)).real)


def _fft_real(r):
    return sfft.fft2(r.astype(np.complex128), axes=(0, 1))


# --------------------------------------------------------------------------------------
# Jacobians, jf = fft(-J(w, ψ))
# --------------------------------------------------------------------------------------
def jacobian_hybrid(wf, k2, dx, dy):
    """hybrid.jl:92-152."""
    gg = 1.0 / (4.0 * dx * dy)
    hh = 1.0 / 3.0
    w = _ifft_real(wf)
    s = _ifft_real(_cdiv(wf, k2))
    R = np.roll
    wE, wW = R(w, -1, 0), R(w, 1, 0)
    wN, wS = R(w, -1, 1), R(w, 1, 1)
    wNE, wSE = R(wE, -1, 1), R(wE, 1, 1)
    wNW, wSW = R(wW, -1, 1), R(wW, 1, 1)
    sE, sW = R(s, -1, 0), R(s, 1, 0)
    sN, sS = R(s, -1, 1), R(s, 1, 1)
    sNE, sSE = R(sE, -1, 1), R(sE, 1, 1)
    sNW, sSW = R(sW, -1, 1), R(sW, 1, 1)
    j1 = gg * ((wE - wW) * (sN - sS) - (wN - wS) * (sE - sW))
    j2 = gg * (wE * (sNE - sSE) - wW * (sNW - sSW) - wN * (sNE - sNW) + wS * (sSE - sSW))
    j3 = gg * (wNE * (sN - sE) - wSW * (sW - sS) - wNW * (sN - sW) + wSE * (sE - sS))
    return _fft_real(-(j1 + j2 + j3) * hh)


def _derivs(wf, k2, dx, eps):
    """pseudospectral_*.jl:96-122: ψ_x, w_y, ψ_y, w_x spectra (j1f .. j4f)."""
    nx, ny = wf.shape
    kx = wave_kx(nx, dx, eps)
    ky = kx[None, :ny]
    kxc = kx[:, None]
    iw = _times_i(wf)
    j1f = _cdiv(_cmul(kxc, iw), k2)
    j4f = _cmul(kxc, iw)
    j2f = _cmul(ky, iw)
    j3f = _cdiv(_cmul(ky, iw), k2)
    return j1f, j2f, j3f, j4f


def jacobian_ps23(wf, k2, dx, dy, eps=1e-6):
    """pseudospectral_23_rule.jl:95-144."""
    nx, ny = wf.shape
    js = list(_derivs(wf, k2, dx, eps))
    nxe, nye = (2 * nx) // 3, (2 * ny) // 3
    lo_x, hi_x = nxe // 2 + 1, nx - nxe // 2          # 1-based inclusive
    lo_y, hi_y = nye // 2 + 1, ny - nye // 2
    for f in js:
        f[lo_x - 1:hi_x, :] = 0.0
        f[:, lo_y - 1:hi_y] = 0.0
    j1, j2, j3, j4 = (_ifft_real(f) for f in js)
    return _fft_real(j1 * j2 - j3 * j4)


def jacobian_ps32(wf, k2, dx, dy, eps=1e-6):
    """pseudospectral_32_rule.jl:94-186."""
    nx, ny = wf.shape
    nxe, nye = (3 * nx) // 2, (3 * ny) // 2
    qx, qy = nxe - nx // 2, nye - ny // 2             # 0-based starts of the upper blocks
    hx, hy = nx // 2, ny // 2
    sc = float(nxe * nye)
    sd = float(nx * ny)

    def pad(f):
        p = np.zeros((nxe, nye), dtype=np.complex128)
        p[:hx, :hy] = f[:hx, :hy]
        p[qx:, :hy] = f[hx:, :hy]
        p[:hx, qy:] = f[:hx, hy:]
        p[qx:, qy:] = f[hx:, hy:]
        return p

    j1, j2, j3, j4 = (_ifft_real(pad(f) * sc / sd) for f in _derivs(wf, k2, dx, eps))
    jp = _fft_real(j1 * j2 - j3 * j4)
    jf = np.empty((nx, ny), dtype=np.complex128)
    jf[:hx, :hy] = jp[:hx, :hy]
    jf[hx:, :hy] = jp[qx:, :hy]
    jf[:hx, hy:] = jp[:hx, qy:]
    jf[hx:, hy:] = jp[qx:, qy:]
    return jf * sd / sc


JACOBIANS = {HYBRID: jacobian_hybrid, PS23: jacobian_ps23, PS32: jacobian_ps32}


# --------------------------------------------------------------------------------------
# Time loop (hybrid.jl:14-86)
# --------------------------------------------------------------------------------------
def to_spectral(w):
    """hybrid.jl:24-28: ŵ = fft(complex(w)); ŵ[1,1] = 0."""
    wf = _fft_real(np.asarray(w, dtype=np.float64))
    wf[0, 0] = 0.0
    return wf


def to_physical(wf):
    """hybrid.jl:71: real(ifft(ŵ)) (interior nx-by-ny)."""
    return _ifft_real(wf)


def step(wnf, k2, dt, re, dx, dy, kind):
    """One RK3-CN step, hybrid.jl:41-67 (float order of the source)."""
    jac = JACOBIANS[kind]
    z = 0.5 * dt * k2 / re
    d1, d2, d3 = (a * z for a in ALPHA)
    jn = jac(wnf, k2, dx, dy)
    w1 = _cmul((1.0 - d1) / (1.0 + d1), wnf) + _cdiv(_cmul(GAMMA[0] * dt, jn), 1.0 + d1)
    w1[0, 0] = 0.0
    j1 = jac(w1, k2, dx, dy)
    w2 = _cmul((1.0 - d2) / (1.0 + d2), w1) + _cdiv(
        _cmul(RHO[1] * dt, jn) + _cmul(GAMMA[1] * dt, j1), 1.0 + d2)
    w2[0, 0] = 0.0
    j2 = jac(w2, k2, dx, dy)
    return _cmul((1.0 - d3) / (1.0 + d3), w2) + _cdiv(
        _cmul(RHO[2] * dt, j1) + _cmul(GAMMA[2] * dt, j2), 1.0 + d3)


def numerical(w0, nt, dt, dx, dy, re, kind, eps=1e-6):
    """hybrid.jl:14-86 without the snapshots: physical interior in, physical out."""
    nx, ny = w0.shape
    k2 = wavespace(nx, ny, dx, dy, eps)
    wf = to_spectral(w0)
    for _ in range(nt):
        wf = step(wf, k2, dt, re, dx, dy, kind)
    return to_physical(wf)


def cn_decay(nx, dx, dt, re, nt, kx_mode, ky_mode, eps=1e-6):
    """The scheme's exact amplification of one Fourier mode with J = 0: Π_k (1-d_k)/(1+d_k)
    per step, d_k = α_k .5Δt k²/re."""
    kx = wave_kx(nx, dx, eps)
    k2 = kx[kx_mode] * kx[kx_mode] + kx[ky_mode] * kx[ky_mode]
    g = 1.0
    for a in ALPHA:
        d = a * (0.5 * dt * k2 / re)
        g *= (1.0 - d) / (1.0 + d)
    return g ** nt
