"""Host-side mirror of `14_Poisson_Solver_FST/fft_d.jl` (fast-sine-transform Dirichlet
Poisson, MMS) over `cfdj_fps_sine`."""
from __future__ import annotations

import math

import numpy as np

from .cavity import fps_sine
from .common import compute_l2norm_bnds


def ps_fst(nx, ny, dx, dy, f):
    """fft_d.jl:7-23: the (nx-1)-by-(ny-1) interior solution of the 5-point Dirichlet
    Poisson problem with right-hand side f[2:nx, 2:ny] (f is (nx+1)-by-(ny+1)): DST-I,
    division by the symbol (2/dx^2)(cos(pi i/nx) - 1) + (2/dy^2)(cos(pi j/ny) - 1), DST-I,
    / (2nx 2ny).  The reference divides (fft_d.jl:15-20) where the cavity's fps_sine
    multiplies by the tabulated reciprocal (lid_driven_cavity.jl:17): the two differ by one
    rounding per spectral coefficient."""
    s = fps_sine(nx, ny, dx, dy, np.asfortranarray(f, dtype=np.float64))
    return np.asfortranarray(s[1:nx, 1:ny])


def mms(nx, km=16):
    """fft_d.jl:26-62: unit box, ue = sin2πx sin2πy + (1/km)² sin(km2πx) sin(km2πy)."""
    ny = nx
    dx, dy = (1.0 - 0.0) / nx, (1.0 - 0.0) / ny
    x = 0.0 + dx * np.arange(nx + 1)
    y = 0.0 + dy * np.arange(ny + 1)
    c1 = (1.0 / km) ** 2
    c2 = -8 * math.pi ** 2
    X, Y = x[:, None], y[None, :]
    tp = 2 * math.pi
    ue = np.sin(tp * X) * np.sin(tp * Y) + c1 * np.sin(km * tp * X) * np.sin(km * tp * Y)
    f = c2 * np.sin(tp * X) * np.sin(tp * Y) + c2 * np.sin(km * tp * X) * np.sin(km * tp * Y)
    return np.asfortranarray(f), np.asfortranarray(ue), dx, dy


def main(grids=(128,)):
    """fft_d.jl:25-94 without the text files: returns {N: (L2, Linf)} (the reference runs
    N = 128 only)."""
    out = {}
    for nx in grids:
        f, ue, dx, dy = mms(nx)
        un = np.zeros_like(f)
        un[1:nx, 1:nx] = ps_fst(nx, nx, dx, dy, f)
        err = un - ue
        out[nx] = (compute_l2norm_bnds(nx, nx, err), float(np.max(np.abs(err))))
    return out
