"""Host-side mirror of `15_Poisson_Solver_Gauss_Seidel/gauss_seidel.jl` (a Jacobi sweep in
the reference, reproduced exactly) on libcfdj.so."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, dptr


def gauss_seidel(dx, dy, nx, ny, r, f, u_n, max_iter, tol, out=None, freq=10000, device=-1):
    """gauss_seidel.jl:8-54: solves into u_n in place; returns (iterations, rms)."""
    f = np.asfortranarray(f, dtype=np.float64)
    f, ldf = _lib.fortran_view(f, "f", (nx + 1, ny + 1))
    u_n, ldu = _lib.fortran_view(u_n, "u_n", (nx + 1, ny + 1), writable=True)
    _lib.require_gpu()
    it = C.c_long()
    rms = C.c_double()
    check(_lib.load().cfdj_jacobi_solve(int(nx), int(ny), float(dx), float(dy), dptr(f),
                                        ldf, dptr(u_n), ldu, int(max_iter),
                                        float(tol), int(freq), C.byref(it), C.byref(rms)),
          "cfdj_jacobi_solve")
    if out is not None:
        out.write(f"L-2 Norm={rms.value}\nIterations={it.value}\n")
    return it.value, rms.value
