"""Host-side mirror of `12_Poisson_Solver_FFT/fft_p.jl` (FD-FFT periodic Poisson, MMS)."""
from __future__ import annotations

import math

import numpy as np

from .common import compute_l2norm_bnds
from .solver import PoissonFFT


def ps_fft(nx, ny, dx, dy, f, eps=1e-6, device=-1):
    """fft_p.jl:8-42: returns real(ifft(fft(f)/symbol)) as an nx-by-ny array."""
    with PoissonFFT(nx, ny, dx, dy, eps, device) as h:
        return h.solve(np.asfortranarray(f[:nx, :ny]))


def mms(nx, km=16):
    """fft_p.jl:45-82: unit box, ue = sin2πx sin2πy + (1/km)² sin(km2πx) sin(km2πy)."""
    ny = nx
    dx, dy = 1.0 / nx, 1.0 / ny
    x = 0.0 + dx * np.arange(nx + 1)
    y = 0.0 + dy * np.arange(ny + 1)
    c1 = (1.0 / km) ** 2
    c2 = -8 * math.pi ** 2
    X, Y = x[:, None], y[None, :]
    tp = 2 * math.pi
    ue = np.sin(tp * X) * np.sin(tp * Y) + c1 * np.sin(km * tp * X) * np.sin(km * tp * Y)
    f = c2 * np.sin(tp * X) * np.sin(tp * Y) + c2 * np.sin(km * tp * X) * np.sin(km * tp * Y)
    return np.asfortranarray(f), np.asfortranarray(ue), dx, dy


def main(grids=(32, 64, 128, 256, 512), device=-1):
    """fft_p.jl:44-119 without the text files: returns {N: (L2, Linf)}."""
    out = {}
    for nx in grids:
        f, ue, dx, dy = mms(nx)
        un = np.zeros_like(f)
        un[:nx, :nx] = ps_fft(nx, nx, dx, dy, f, device=device)
        un[nx, :] = un[0, :]
        un[:, nx] = un[:, 0]
        err = un - ue
        out[nx] = (compute_l2norm_bnds(nx, nx, err), float(np.max(np.abs(err))))
    return out
