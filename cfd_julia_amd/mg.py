"""Host-side mirror of `17_Poisson_Solver_Multigrid/mg_N.jl` (n-level V-cycle) on
libcfdj.so.  The GPU smoother visits the Common.jl:78-92 update in red-black order."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, dptr


class Multigrid:
    def __init__(self, nx, ny, dx, dy, n_level, v1=2, v2=2, v3=2, device=-1):
        lib = _lib.load()
        _lib.require_gpu()
        h = C.c_void_p()
        check(lib.cfdj_mg_create(int(nx), int(ny), float(dx), float(dy), int(n_level), v1, v2,
                                 v3, int(device), C.byref(h)), "cfdj_mg_create")
        self._h, self.nx, self.ny = h, int(nx), int(ny)

    def solve(self, f, u, tol=1e-9, max_iter=100000):
        """u (in: boundary values / initial guess; out: solution) -> (iterations, rms)."""
        f = np.asfortranarray(f, dtype=np.float64)
        if not (isinstance(u, np.ndarray) and u.flags.f_contiguous and u.dtype == np.float64):
            raise TypeError("u must be a Fortran-ordered float64 array (updated in place)")
        hist = np.zeros(int(max_iter) + 1)
        it = C.c_int()
        check(_lib.load().cfdj_mg_solve(self._h, dptr(f), f.shape[0], dptr(u), u.shape[0],
                                        float(tol), int(max_iter), C.byref(it), dptr(hist)),
              "cfdj_mg_solve")
        return it.value, hist[:it.value + 1]

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().cfdj_mg_destroy(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def mg_N(dx, dy, nx, ny, r, f, u_n, v1, v2, v3, max_iter, tol, out=None, n_level=2, freq=1,
         device=-1):
    """mg_N.jl:7-114: solves into u_n in place; r receives the final fine residual norm
    history is returned as (iterations, rms list); `out` (a text stream) gets the
    reference's "L-2 Norm= / Iterations=" lines."""
    with Multigrid(nx, ny, dx, dy, n_level, v1, v2, v3, device) as mg:
        it, hist = mg.solve(f, u_n, tol, max_iter)
    if out is not None:
        out.write(f"L-2 Norm={hist[-1]}\n")
        out.write(f"Iterations={it}\n")
    return it, hist


def mms(nx, ny=None, ipr=1):
    """mg_N.jl:127-169 (unit box, Dirichlet data from the exact solution)."""
    import math

    ny = nx if ny is None else ny
    dx, dy = 1.0 / nx, 1.0 / ny
    x = dx * np.arange(nx + 1)
    y = dy * np.arange(ny + 1)
    X, Y = x[:, None], y[None, :]
    if ipr == 1:
        ue = (X ** 2 - 1) * (Y ** 2 - 1)
        f = -2 * (2 - X ** 2 - Y ** 2)
    else:
        c1 = (1.0 / 16) ** 2
        c2 = -2 * math.pi ** 2
        ue = (np.sin(2 * math.pi * X) * np.sin(2 * math.pi * Y)
              + c1 * np.sin(16 * math.pi * X) * np.sin(16 * math.pi * Y))
        f = (4 * c2 * np.sin(2 * math.pi * X) * np.sin(2 * math.pi * Y)
             + c2 * np.sin(16 * math.pi * X) * np.sin(16 * math.pi * Y))
    un = np.zeros_like(ue)
    un[:, 0], un[:, ny] = ue[:, 0], ue[:, ny]
    un[0, :], un[nx, :] = ue[0, :], ue[nx, :]
    return np.asfortranarray(f), np.asfortranarray(ue), np.asfortranarray(un), dx, dy
