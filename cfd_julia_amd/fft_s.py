"""Host-side mirror of `13_Poisson_Solver_FFT_Spectral/fft_s.jl` (spectral FFT Poisson)."""
from __future__ import annotations

import numpy as np

from .common import compute_l2norm_bnds
from .fft_p import mms
from .solver import PoissonFFT


def ps_spectral(nx, ny, dx, dy, f, eps=1e-6, device=-1):
    """fft_s.jl:8-37: real(ifft(fft(f) / (-kx^2 - ky^2))), kx = 2pi/(nx dx) * index."""
    with PoissonFFT(nx, ny, dx, dy, eps, device, symbol="spectral") as h:
        return h.solve(np.asfortranarray(f[:nx, :ny]))


def main(grids=(32, 64, 128, 256, 512), device=-1):
    """fft_s.jl:39-116 without the text files: returns {N: (L2, Linf)} (same MMS as fft_p)."""
    out = {}
    for nx in grids:
        f, ue, dx, dy = mms(nx)
        un = np.zeros_like(f)
        un[:nx, :nx] = ps_spectral(nx, nx, dx, dy, f, device=device)
        un[nx, :] = un[0, :]
        un[:, nx] = un[:, 0]
        err = un - ue
        out[nx] = (compute_l2norm_bnds(nx, nx, err), float(np.max(np.abs(err))))
    return out
