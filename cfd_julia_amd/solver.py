"""Object wrappers of the libcfdj.so handles (device-resident solver state)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, dptr

_PATHS = {"auto": _lib.POISSON_AUTO, "rocfft": _lib.POISSON_ROCFFT, "fused": _lib.POISSON_FUSED,
          "schur": _lib.POISSON_SCHUR}
_PATH_NAMES = {v: k for k, v in _PATHS.items()}


class PoissonFFT:
    """Periodic FD-FFT Poisson solver, plan built once (Common.jl:97-125 `fps`,
    12_Poisson_Solver_FFT/fft_p.jl:8-42 `ps_fft`)."""

    def __init__(self, nx, ny, dx, dy, eps=1e-6, device=-1, symbol="fd"):
        """symbol: "fd" (Common.jl fps / fft_p.jl) or "spectral" (fft_s.jl ps_spectral)."""
        lib = _lib.load()
        _lib.require_gpu()
        h = C.c_void_p()
        check(lib.cfdj_fps_create(int(nx), int(ny), float(dx), float(dy), float(eps),
                                  int(device), C.byref(h)), "cfdj_fps_create")
        self._h, self.nx, self.ny = h, int(nx), int(ny)
        if symbol != "fd":
            kinds = {"spectral": _lib.SYMBOL_SPECTRAL}
            if symbol not in kinds:
                self.close()
                raise ValueError(f"unknown symbol {symbol!r}")
            check(lib.cfdj_fps_set_symbol(h, kinds[symbol]), "cfdj_fps_set_symbol")

    def solve(self, f, out=None):
        """f: (>=nx, >=ny) float64 array -> s: nx-by-ny (Fortran order)."""
        f = np.asfortranarray(f, dtype=np.float64)
        f, ldf = _lib.fortran_view(f, "f", (self.nx, self.ny))
        if out is None:
            out = np.empty((self.nx, self.ny), dtype=np.float64, order="F")
        out, lds = _lib.fortran_view(out, "s", (self.nx, self.ny), writable=True)
        check(_lib.load().cfdj_fps_solve(self._h, dptr(f), ldf, dptr(out), lds),
              "cfdj_fps_solve")
        return out

    def set_poisson(self, path):
        """path: "auto" | "rocfft" | "fused" (CFDJ_POISSON_*)."""
        check(_lib.load().cfdj_fps_set_poisson(self._h, _PATHS[path]), "cfdj_fps_set_poisson")

    def poisson(self):
        return _PATH_NAMES[
            _lib.load().cfdj_fps_get_poisson(self._h)]

    def solve_device(self, f_ptr, s_ptr):
        check(_lib.load().cfdj_fps_solve_device(self._h, C.c_void_p(f_ptr), C.c_void_p(s_ptr)),
              "cfdj_fps_solve_device")

    def solve_device_noalloc(self, f_ptr, s_ptr):
        """cfdj_fps_solve_device with the half spectrum in the library's static device
        array: allocates nothing (fused path, (nx/2)*ny <= 2**20)."""
        check(_lib.load().cfdj_fps_solve_device_noalloc(self._h, C.c_void_p(f_ptr),
                                                        C.c_void_p(s_ptr)),
              "cfdj_fps_solve_device_noalloc")

    def stream(self):
        """The plan's hipStream_t (as an integer) the device solves are enqueued on."""
        p = C.c_void_p()
        check(_lib.load().cfdj_fps_stream(self._h, C.byref(p)), "cfdj_fps_stream")
        return p.value

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().cfdj_fps_destroy(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class VortexMerger:
    """Device-resident periodic vortex-merger state (vm.jl:12-90 + Common.jl:132-182).

    kind = "single" (one GPU), "virtual" (nranks y-slabs on one GPU, transposes and halos
    by device copies) or "dist" (one process per GPU over RCCL; pass rank, nranks and the
    128-byte unique id from `unique_id()` on rank 0)."""

    def __init__(self, nx, ny, dx, dy, re, eps=1e-6, device=-1, kind="single", nranks=1,
                 rank=0, nccl_id=None):
        lib = _lib.load()
        _lib.require_gpu()
        h = C.c_void_p()
        args = (int(nx), int(ny), float(dx), float(dy), float(re), float(eps), int(device))
        if kind == "single":
            check(lib.cfdj_vm_create(*args, C.byref(h)), "cfdj_vm_create")
        elif kind == "virtual":
            check(lib.cfdj_vm_create_virtual(*args, int(nranks), C.byref(h)),
                  "cfdj_vm_create_virtual")
        elif kind == "dist":
            if nccl_id is None or len(nccl_id) != 128:
                raise ValueError("dist handles need the 128-byte RCCL unique id")
            check(lib.cfdj_vm_create_dist(*args, int(rank), int(nranks), bytes(nccl_id),
                                          C.byref(h)), "cfdj_vm_create_dist")
        else:
            raise ValueError(f"unknown kind {kind!r}")
        self._h = h
        self.nx, self.ny, self.kind, self.nranks, self.rank = int(nx), int(ny), kind, nranks, rank

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(_lib.load().cfdj_comm_unique_id(buf), "cfdj_comm_unique_id")
        return buf.raw

    def comm_ranks(self) -> int:
        """Ranks of the handle's RCCL communicator as RCCL reports them (0: none)."""
        n = C.c_int()
        check(_lib.load().cfdj_vm_comm_ranks(self._h, C.byref(n)), "cfdj_vm_comm_ranks")
        return n.value

    # ---- data movement (reference ghosted layout) -----------------------------------
    def upload(self, w_ghosted):
        w = np.asfortranarray(w_ghosted, dtype=np.float64)
        w, ldw = _lib.fortran_view(w, "w", (self.nx + 2, self.ny + 2))
        check(_lib.load().cfdj_vm_upload(self._h, dptr(w), ldw), "cfdj_vm_upload")

    def download(self, out=None):
        if out is None:
            out = np.zeros((self.nx + 2, self.ny + 2), dtype=np.float64, order="F")
        out, ldw = _lib.fortran_view(out, "w", (self.nx + 2, self.ny + 2), writable=True)
        check(_lib.load().cfdj_vm_download(self._h, dptr(out), ldw), "cfdj_vm_download")
        return out

    def upload_interior(self, w):
        """Convenience: periodic interior (nx, ny) -> device."""
        g = np.zeros((self.nx + 2, self.ny + 2), dtype=np.float64, order="F")
        g[1:-1, 1:-1] = w
        self.upload(g)

    def download_interior(self):
        return np.array(self.download()[1:-1, 1:-1])

    # ---- compute ----------------------------------------------------------------------
    def step(self, dt, nsteps=1):
        check(_lib.load().cfdj_vm_step(self._h, float(dt), int(nsteps)), "cfdj_vm_step")

    def step_async(self, dt, nsteps=1):
        check(_lib.load().cfdj_vm_step_async(self._h, float(dt), int(nsteps)),
              "cfdj_vm_step_async")

    def sync(self):
        check(_lib.load().cfdj_vm_sync(self._h), "cfdj_vm_sync")

    def rhs(self, w_ghosted, r=None, s=None):
        """One vm_rhs: returns (r, s) ghosted arrays (r's ghost layer untouched/zero)."""
        w = np.asfortranarray(w_ghosted, dtype=np.float64)
        w, ldw = _lib.fortran_view(w, "w", (self.nx + 2, self.ny + 2))
        shape = (self.nx + 2, self.ny + 2)
        r = np.zeros(shape, order="F") if r is None else r
        s = np.zeros(shape, order="F") if s is None else s
        r, ldr = _lib.fortran_view(r, "r", shape, writable=True)
        s, lds = _lib.fortran_view(s, "s", shape, writable=True)
        check(_lib.load().cfdj_vm_rhs(self._h, dptr(w), ldw, dptr(r), ldr, dptr(s), lds),
              "cfdj_vm_rhs")
        return r, s

    # ---- instrumentation -----------------------------------------------------------
    def set_timing(self, enable=True):
        check(_lib.load().cfdj_vm_set_timing(self._h, int(bool(enable))), "cfdj_vm_set_timing")

    def timing(self):
        ms = (C.c_double * _lib.K_COUNT)()
        n = (C.c_long * _lib.K_COUNT)()
        check(_lib.load().cfdj_vm_timing(self._h, ms, n), "cfdj_vm_timing")
        return {name: (ms[i], n[i]) for i, name in enumerate(_lib.K_NAMES)}

    def stage_timing(self):
        """[(ms, launches)] of the stage kernel per RK3 stage 1..3 (same recording as timing())."""
        ms = (C.c_double * 3)()
        n = (C.c_long * 3)()
        check(_lib.load().cfdj_vm_stage_timing(self._h, ms, n), "cfdj_vm_stage_timing")
        return [(ms[i], n[i]) for i in range(3)]

    def kernel_bench(self, kernel, dt, launches=20):
        """ms per launch of `launches` back-to-back launches of one kernel (CFDJ_KB_*);
        clobbers the stage buffers and advances the field: use after the timed runs."""
        ms = C.c_double()
        check(_lib.load().cfdj_vm_kernel_bench(self._h, int(kernel), float(dt), int(launches),
                                               C.byref(ms)), "cfdj_vm_kernel_bench")
        return ms.value

    def set_check_finite(self, enable=True):
        check(_lib.load().cfdj_vm_set_check_finite(self._h, int(bool(enable))),
              "cfdj_vm_set_check_finite")

    def set_rows_per_wave(self, rows):
        check(_lib.load().cfdj_vm_set_rows_per_wave(self._h, int(rows)),
              "cfdj_vm_set_rows_per_wave")

    def stage_row_group(self) -> bool:
        """True where a step launches the row-group stage kernel, False: the marching one."""
        f = C.c_int()
        check(_lib.load().cfdj_vm_stage_kernel(self._h, C.byref(f)), "cfdj_vm_stage_kernel")
        return bool(f.value)

    def set_graph(self, enable=True):
        check(_lib.load().cfdj_vm_set_graph(self._h, int(bool(enable))), "cfdj_vm_set_graph")

    def set_poisson(self, path):
        """path: "auto" | "rocfft" | "fused" (CFDJ_POISSON_*)."""
        check(_lib.load().cfdj_vm_set_poisson(self._h, _PATHS[path]), "cfdj_vm_set_poisson")

    def poisson(self):
        return _PATH_NAMES[
            _lib.load().cfdj_vm_get_poisson(self._h)]

    def field_device_ptr(self):
        p = C.c_void_p()
        check(_lib.load().cfdj_vm_field_device(self._h, C.byref(p)), "cfdj_vm_field_device")
        return p.value

    def slab(self):
        r0, n = C.c_int(), C.c_int()
        check(_lib.load().cfdj_vm_slab(self._h, C.byref(r0), C.byref(n)), "cfdj_vm_slab")
        return r0.value, n.value

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().cfdj_vm_destroy(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
