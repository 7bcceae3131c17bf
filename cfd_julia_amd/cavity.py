"""Host-side mirror of `18_NS2D_Lid_Driven_Cavity/lid_driven_cavity.jl` on libcfdj.so.

Arrays are the reference's (nx+1, ny+1) node fields, 0-based, Fortran order.  All compute
runs on the GPU (`cfdj_cavity_*`); there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np

from . import _lib
from ._lib import check, dptr
from .fieldio import write_field, write_res_plot


class Cavity:
    """Device-resident cavity state (lid_driven_cavity.jl:58-118).  poisson="dst" is the
    reference's fps_sine; "mg" the V-cycle multigrid of mg_N.jl (warm-started)."""

    def __init__(self, nx, ny, dx, dy, re, device=-1, poisson="dst", n_level=None, v1=2,
                 v2=2, v3=2, tol=1e-9, max_iter=100000):
        lib = _lib.load()
        _lib.require_gpu()
        h = C.c_void_p()
        check(lib.cfdj_cavity_create(int(nx), int(ny), float(dx), float(dy), float(re),
                                     int(device), C.byref(h)), "cfdj_cavity_create")
        self._h, self.nx, self.ny = h, int(nx), int(ny)
        if poisson == "mg":
            if n_level is None:  # as deep as the grid allows (coarsest >= 2 cells)
                n_level = int(math.log2(min(nx, ny))) if nx == ny else 2
            check(lib.cfdj_cavity_set_poisson(h, _lib.CAVITY_MG, int(n_level), v1, v2, v3,
                                              float(tol), int(max_iter)),
                  "cfdj_cavity_set_poisson")
        elif poisson != "dst":
            raise ValueError(poisson)

    def _shape(self):
        return (self.nx + 1, self.ny + 1)

    def upload(self, wn, sn):
        w = np.asfortranarray(wn, dtype=np.float64)
        s = np.asfortranarray(sn, dtype=np.float64)
        _lib.fortran_view(w, "wn", self._shape())
        _lib.fortran_view(s, "sn", self._shape())
        check(_lib.load().cfdj_cavity_upload(self._h, dptr(w), w.shape[0], dptr(s),
                                             s.shape[0]), "cfdj_cavity_upload")

    def download(self):
        w = np.zeros(self._shape(), order="F")
        s = np.zeros(self._shape(), order="F")
        check(_lib.load().cfdj_cavity_download(self._h, dptr(w), w.shape[0], dptr(s),
                                               s.shape[0]), "cfdj_cavity_download")
        return w, s

    def step(self, dt, nsteps=1):
        rms = np.zeros(max(int(nsteps), 1))
        check(_lib.load().cfdj_cavity_step(self._h, float(dt), int(nsteps), dptr(rms)),
              "cfdj_cavity_step")
        return rms[:nsteps]

    def rhs(self, w, s):
        w = np.asfortranarray(w, dtype=np.float64)
        s = np.asfortranarray(s, dtype=np.float64)
        _lib.fortran_view(w, "w", self._shape())
        _lib.fortran_view(s, "s", self._shape())
        r = np.zeros(self._shape(), order="F")
        check(_lib.load().cfdj_cavity_rhs(self._h, dptr(w), w.shape[0], dptr(s), s.shape[0],
                                          dptr(r), r.shape[0]), "cfdj_cavity_rhs")
        return r

    def mg_iterations(self):
        return _lib.load().cfdj_cavity_mg_iterations(self._h)

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().cfdj_cavity_destroy(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def fps_sine(nx, ny, dx, dy, f, u=None, e=None, data=None, data1=None, iden=None, sn=None):
    """lid_driven_cavity.jl:11-21: sn[1:nx, 1:ny] (Julia sn[2:nx, 2:ny]) <- Dirichlet
    5-point Poisson solution with right-hand side f[1:nx, 1:ny]; returns sn."""
    f = np.asfortranarray(f, dtype=np.float64)
    sn = np.zeros((nx + 1, ny + 1), order="F") if sn is None else sn
    # the C side copies (nx+1) x (ny+1) nodes in and out: a short, C-ordered or non-float64
    # array would be read / written out of bounds or transposed
    f, ldf = _lib.fortran_view(f, "f", (nx + 1, ny + 1))
    sn, lds = _lib.fortran_view(sn, "sn", (nx + 1, ny + 1), writable=True)
    _lib.require_gpu()
    check(_lib.load().cfdj_fps_sine(int(nx), int(ny), float(dx), float(dy), dptr(f),
                                    ldf, dptr(sn), lds), "cfdj_fps_sine")
    return sn


def numerical(nx, ny, nt, dx, dy, dt, re, wn, sn, rms, device=-1, poisson="dst"):
    """lid_driven_cavity.jl:58-118: advances wn, sn in place for nt steps and fills rms."""
    _lib.fortran_view(wn, "wn", (nx + 1, ny + 1), writable=True)
    _lib.fortran_view(sn, "sn", (nx + 1, ny + 1), writable=True)
    if len(rms) < nt:
        raise _lib.ArgumentError(-1, "rms", f"length {len(rms)} < nt = {nt} (BoundsError)")
    with Cavity(nx, ny, dx, dy, re, device, poisson) as h:
        h.upload(wn, sn)
        rms[:nt] = h.step(dt, nt)
        w, s = h.download()
    wn[...] = w
    sn[...] = s
    return None


def main(nx=64, ny=64, dt=0.001, tf=10.0, re=100.0, poisson="dst", outdir=None):
    """lid_driven_cavity.jl:161-216: returns (wn, sn, rms); with outdir, also writes the
    reference's res_plot.txt ("n rms") and field_final.txt ("x y ω ψ") there."""
    dx = (1.0 - 0.0) / nx
    dy = (1.0 - 0.0) / ny
    nt = int(tf / dt)
    wn = np.zeros((nx + 1, ny + 1), order="F")
    sn = np.zeros((nx + 1, ny + 1), order="F")
    rms = np.empty(nt)
    numerical(nx, ny, nt, dx, dy, dt, re, wn, sn, rms, poisson=poisson)
    if outdir is not None:
        x = dx * np.arange(nx + 1, dtype=np.float64)
        y = dy * np.arange(ny + 1, dtype=np.float64)
        write_res_plot(os.path.join(outdir, "res_plot.txt"), rms)
        write_field(os.path.join(outdir, "field_final.txt"), x, y, wn, sn)
    return wn, sn, rms
