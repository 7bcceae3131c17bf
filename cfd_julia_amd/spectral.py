"""Host-side mirror of the reference's spectral-space NS2D scripts on libcfdj.so:

  hybrid          -- 20_NS2D_Hybrid_Solver/hybrid.jl (Arakawa Jacobian in physical space)
  pseudospectral  -- 22_NS2D_PseudoSpectral_23_Rule/pseudospectral_23_rule.jl (rule="2/3")
                     21_NS2D_PseudoSpectral_32_Rule/pseudospectral_32_rule.jl (rule="3/2")

`numerical(nx, ny, nt, dx, dy, dt, re, x, y, wn, ns)` keeps the reference signature and
return value (the (nx+1)x(ny+1) field real(ifft(w_f)) with its periodic row and column,
hybrid.jl:14-86); `main()` runs the reference's 128^2, t = 20 vortex merger.  All compute
runs on the GPU (`cfdj_spec_*`); there is no CPU path.  The "vm$m.txt" snapshots are
written only when `snapshot_dir` is given, in vm.py's "x y ω" line format.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib
from ._lib import check, dptr

KINDS = {"hybrid": _lib.SPEC_HYBRID, "2/3": _lib.SPEC_PS23, "3/2": _lib.SPEC_PS32}


class SpectralNS2D:
    """Device-resident spectral vorticity w_f of one of the three reference scripts."""

    def __init__(self, nx, ny, dx, dy, re, kind="hybrid", eps=1e-6, device=-1):
        lib = _lib.load()
        _lib.require_gpu()
        h = C.c_void_p()
        check(lib.cfdj_spec_create(int(nx), int(ny), float(dx), float(dy), float(re),
                                   float(eps), KINDS[kind], int(device), C.byref(h)),
              "cfdj_spec_create")
        self._h, self.nx, self.ny = h, int(nx), int(ny)

    def upload(self, wn):
        """hybrid.jl:24-28 from the ghosted (nx+2)x(ny+2) array of vm.jl's layout."""
        w = np.asfortranarray(wn, dtype=np.float64)
        _lib.fortran_view(w, "wn", (self.nx + 2, self.ny + 2))
        check(_lib.load().cfdj_spec_upload(self._h, dptr(w), w.shape[0]), "cfdj_spec_upload")

    def upload_interior(self, w):
        g = np.zeros((self.nx + 2, self.ny + 2), order="F")
        g[1:-1, 1:-1] = w
        self.upload(g)

    def step(self, dt, nsteps=1):
        check(_lib.load().cfdj_spec_step(self._h, float(dt), int(nsteps)), "cfdj_spec_step")

    def download(self):
        """hybrid.jl:71-76: (nx+1)x(ny+1) real(ifft(w_f)) with the periodic row/column."""
        ut = np.zeros((self.nx + 1, self.ny + 1), order="F")
        check(_lib.load().cfdj_spec_download(self._h, dptr(ut), ut.shape[0]),
              "cfdj_spec_download")
        return ut

    def spectrum(self):
        wf = np.zeros((self.nx, self.ny), dtype=np.complex128, order="F")
        check(_lib.load().cfdj_spec_get_spectrum(self._h, wf.ctypes.data_as(_lib._dp)),
              "cfdj_spec_get_spectrum")
        return wf

    def set_spectrum(self, wf):
        a = np.asfortranarray(wf, dtype=np.complex128)
        assert a.shape == (self.nx, self.ny)
        check(_lib.load().cfdj_spec_set_spectrum(self._h, a.ctypes.data_as(_lib._dp)),
              "cfdj_spec_set_spectrum")

    def jacobian(self, wf):
        """One reference `jacobian(nx, ny, dx, dy, wf, k2)`: fft(-J(w, psi))."""
        a = np.asfortranarray(wf, dtype=np.complex128)
        assert a.shape == (self.nx, self.ny)
        out = np.zeros_like(a, order="F")
        check(_lib.load().cfdj_spec_jacobian(self._h, a.ctypes.data_as(_lib._dp),
                                             out.ctypes.data_as(_lib._dp)),
              "cfdj_spec_jacobian")
        return out

    def close(self):
        if self._h:
            _lib.load().cfdj_spec_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def numerical(nx, ny, nt, dx, dy, dt, re, x, y, wn, ns, kind="hybrid", snapshot_dir=None):
    """hybrid.jl:14-86 / pseudospectral_*.jl:13-89 (same loop; `kind` picks the Jacobian).
    Snapshots every nt ÷ ns steps as the reference writes them ("vm$m.txt", m = 1, 2, ...)
    when snapshot_dir is given."""
    freq = nt // ns  # DivideError for ns > nt, as in the reference
    with SpectralNS2D(nx, ny, dx, dy, re, kind) as h:
        h.upload(wn)
        done, m = 0, 1
        while done < nt:
            k = min(freq - done % freq, nt - done)
            h.step(dt, k)
            done += k
            if done % freq == 0 and snapshot_dir is not None:
                from .vm import _write_field
                _write_field(f"{snapshot_dir}/vm{m}.txt", x, y, h.download())
                m += 1
        return h.download()


def setup(nx=128, ny=128, dt=0.01, tf=20.0, re=1000.0, ns=10):
    """hybrid.jl:154-190: grid, vm_ic and its ghost copies."""
    from .common import vm_ic

    dx, dy = 2 * math.pi / nx, 2 * math.pi / ny
    x = dx * np.arange(nx + 1)
    y = dy * np.arange(ny + 1)
    wn = np.zeros((nx + 2, ny + 2), order="F")
    vm_ic(nx, ny, x, y, wn)
    wn[0, :] = wn[nx, :]
    wn[:, 0] = wn[:, ny]
    wn[nx + 1, :] = wn[1, :]
    wn[:, ny + 1] = wn[:, 1]
    return dict(nx=nx, ny=ny, dx=dx, dy=dy, dt=dt, nt=int(round(tf / dt)), re=re, ns=ns,
                x=x, y=y, wn=wn)


def main(kind="hybrid", **kw):
    c = setup(**kw)
    return numerical(c["nx"], c["ny"], c["nt"], c["dx"], c["dy"], c["dt"], c["re"], c["x"],
                     c["y"], c["wn"], c["ns"], kind)
