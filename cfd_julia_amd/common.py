"""Host-side mirror of the hot-path subset of the reference's `Common.jl`.

Same function names, positional arguments and in-place semantics as the Julia module,
with 0-based NumPy arrays in the reference's column-major (Fortran) layout:

    Julia                                              here
    fps(nx,ny,Δx,Δy,u,e,data,data1,f,s)  (Common.jl:97)   fps(nx,ny,dx,dy,u,e,data,data1,f,s)
    vm_rhs(nx,ny,Δx,Δy,re,w,u,e,data,data1,r,s,f) (:132) vm_rhs(...same...)
    vm_ic(nx,ny,x,y,w)                   (Common.jl:208)   vm_ic(nx,ny,x,y,w)
    compute_l2norm(nx,ny,r)              (Common.jl:229)   compute_l2norm(nx,ny,r)
    compute_l2norm_bnds(nx,ny,r)         (Common.jl:234)   compute_l2norm_bnds(nx,ny,r)

The FFT scratch arguments (u, e, data, data1) of the reference are accepted and ignored:
the GPU handle owns its spectrum buffers.  All compute runs in libcfdj.so on the GPU;
there is no CPU fallback.  Handles (rocFFT plans, device buffers) are cached per grid, so
repeated calls do not re-plan (the reference re-plans FFTW on every call).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np

from ._lib import ArgumentError
from .solver import PoissonFFT, VortexMerger

_CACHE: "OrderedDict[tuple, object]" = OrderedDict()
_CACHE_MAX = 4


def _cached(key, factory):
    obj = _CACHE.get(key)
    if obj is None:
        obj = factory()
        _CACHE[key] = obj
        while len(_CACHE) > _CACHE_MAX:
            _CACHE.popitem(last=False)[1].close()
    else:
        _CACHE.move_to_end(key)
    return obj


def clear_cache():
    while _CACHE:
        _CACHE.popitem()[1].close()


def fps(nx, ny, dx, dy, u, e, data, data1, f, s, eps=1e-6):
    """Common.jl:97-125.  Reads f[0:nx, 0:ny]; writes s[1:nx+1, 1:ny+1] (Julia
    s[2:nx+1, 2:ny+1]) with the FD-consistent periodic Poisson solution of ∇²s = f."""
    if s.shape[0] < nx + 2 or s.shape[1] < ny + 2:
        raise ArgumentError(-1, "fps", "s must be at least (nx+2, ny+2) (BoundsError)")
    h = _cached(("fps", nx, ny, dx, dy, eps), lambda: PoissonFFT(nx, ny, dx, dy, eps))
    s[1:nx + 1, 1:ny + 1] = h.solve(np.asfortranarray(f[:nx, :ny]))
    return None


def vm_rhs(nx, ny, dx, dy, re, w, u, e, data, data1, r, s, f, eps=1e-6):
    """Common.jl:132-182: f = -w; s = fps(f) with periodic ghosts; r = -J(w,s) + ν∇²w.
    w, r, s are ghosted (nx+2, ny+2) arrays; f is (nx, ny).  Mutates r (interior), s
    (all) and f, like the reference."""
    h = _cached(("vm", nx, ny, dx, dy, re, eps),
                lambda: VortexMerger(nx, ny, dx, dy, re, eps))
    wg = np.asfortranarray(w, dtype=np.float64)
    rr, ss = h.rhs(wg)
    r[1:nx + 1, 1:ny + 1] = rr[1:nx + 1, 1:ny + 1]
    s[...] = ss
    f[:nx, :ny] = -wg[1:nx + 1, 1:ny + 1]
    return None


def vm_ic(nx, ny, x, y, w):
    """Common.jl:208-219: two Gaussian vortices (σ = π, centres (π∓π/4, π)) written to
    w[1:nx+2, 1:ny+2] (Julia w[2:nx+2, 2:ny+2]) from x[0:nx+1], y[0:ny+1]."""
    sigma = math.pi
    xc1, yc1 = math.pi - math.pi / 4.0, math.pi
    xc2, yc2 = math.pi + math.pi / 4.0, math.pi
    X = np.asarray(x[:nx + 1])[:, None]
    Y = np.asarray(y[:ny + 1])[None, :]
    w[1:nx + 2, 1:ny + 2] = (np.exp(-sigma * ((X - xc1) ** 2 + (Y - yc1) ** 2))
                             + np.exp(-sigma * ((X - xc2) ** 2 + (Y - yc2) ** 2)))


def periodic_ghosts(w, nx, ny):
    """vm.jl:121-128 / 68-76 ghost fill of a ghosted array (in place)."""
    w[nx + 1, :] = w[1, :]
    w[:, ny + 1] = w[:, 1]
    w[0, :] = w[nx, :]
    w[:, 0] = w[:, ny]


def compute_l2norm(nx, ny, r):
    """Common.jl:229-232: sqrt(Σ r[2:nx,2:ny]² / ((nx-1)(ny-1)))."""
    a = r[1:nx, 1:ny]
    return math.sqrt(float(np.sum(a * a)) / ((nx - 1) * (ny - 1)))


def compute_l2norm_bnds(nx, ny, r):
    """Common.jl:234-237: sqrt(Σ r[1:nx+1,1:ny+1]² / ((nx+1)(ny+1)))."""
    a = r[:nx + 1, :ny + 1]
    return math.sqrt(float(np.sum(a * a)) / ((nx + 1) * (ny + 1)))
