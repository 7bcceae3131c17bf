"""Host-side mirrors of `17_Poisson_Solver_Multigrid/mg_N.jl` (n-level V-cycle) and
`17_Poisson_Solver_Multigrid/mg.jl` (two-level cycle) on libcfdj.so.  The GPU smoother
visits the Common.jl:78-92 update in red-black order."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _lib
from ._lib import check, dptr
from .fieldio import julia_str


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
        shape = (self.nx + 1, self.ny + 1)
        f = np.asfortranarray(f, dtype=np.float64)
        f, ldf = _lib.fortran_view(f, "f", shape)
        u, ldu = _lib.fortran_view(u, "u_n", shape, writable=True)
        hist = np.zeros(int(max_iter) + 1)
        it = C.c_int()
        check(_lib.load().cfdj_mg_solve(self._h, dptr(f), ldf, dptr(u), ldu,
                                        float(tol), int(max_iter), C.byref(it), dptr(hist)),
              "cfdj_mg_solve")
        return it.value, hist[:it.value + 1]

    def residual(self, r):
        """The fine residual of the last solve's final convergence check, into r in place."""
        r, ldr = _lib.fortran_view(r, "r", (self.nx + 1, self.ny + 1), writable=True)
        check(_lib.load().cfdj_mg_residual(self._h, dptr(r), ldr), "cfdj_mg_residual")
        return r

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().cfdj_mg_destroy(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def _run(n_level, sweeps, dx, dy, nx, ny, r, f, u_n, max_iter, tol, out, freq, res_name,
         outdir, device):
    with Multigrid(nx, ny, dx, dy, n_level, *sweeps, device=device) as mg_:
        it, hist = mg_.solve(f, u_n, tol, max_iter)
        if r is None:
            r = np.zeros((nx + 1, ny + 1), order="F")
        mg_.residual(r)
    if outdir is not None:  # the residual history file (every freq-th iteration)
        with open(os.path.join(outdir, res_name), "w") as res:
            for k in range(1, it + 1):
                if k % freq == 0:
                    res.write(f"{k} {julia_str(hist[k])} {julia_str(hist[k] / hist[0])}\n")
    if out is not None:
        out.write(f"L-2 Norm={julia_str(hist[-1])}\n")
        out.write(f"Maximum Norm={julia_str(float(np.abs(r).max()))}\n")
        out.write(f"Iterations={it}\n")
    return it, hist


def mg_N(dx, dy, nx, ny, r, f, u_n, v1, v2, v3, max_iter, tol, out=None, n_level=2, freq=1,
         device=-1, outdir=None):
    """mg_N.jl:7-114: solves into u_n in place and leaves the final fine residual in r (an
    (nx+1) x (ny+1) Fortran-ordered array, or None); `out` (a text stream) receives the
    reference's "L-2 Norm= / Maximum Norm= / Iterations=" lines (mg_N.jl:109-111) and, with
    `outdir`, `mg_residual.txt` the "it rms rms/rms0" history (mg_N.jl:8,64-67).  Returns
    (iterations, rms history incl. the initial residual)."""
    return _run(n_level, (v1, v2, v3), dx, dy, nx, ny, r, f, u_n, max_iter, tol, out, freq,
                "mg_residual.txt", outdir, device)


def mg(dx, dy, nx, ny, r, f, u_n, v1, v2, v3, max_iter, tol, out=None, freq=100, device=-1,
       outdir=None):
    """mg.jl:7-85, the two-level cycle: v1 pre-smoothing sweeps, v3 sweeps on the coarse grid
    (mg.jl:66), v2 sweeps after the correction (mg.jl:77) -- the coarse / post roles are the
    reverse of mg_N's, so the handle is created with (v1, v3, v2).  Writes `residual.txt`
    (mg.jl:9,52-56) under `outdir`."""
    return _run(2, (v1, v3, v2), dx, dy, nx, ny, r, f, u_n, max_iter, tol, out, freq,
                "residual.txt", outdir, device)


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
