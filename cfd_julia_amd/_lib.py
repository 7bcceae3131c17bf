"""ctypes binding of libcfdj.so (include/cfdj.h).

The shared library is built in-tree (`python -c "import __graft_entry__ as g; g.build()"`
or `make -C cfd_julia_amd/csrc`).  There is no CPU fallback: if the library is missing or
no HIP device is visible the calls raise `CfdjError` -- the product path never silently
runs anything else.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CFDJ_LIB", os.path.join(_HERE, "libcfdj.so"))

CFDJ_OK = 0
ERR_NAMES = {-1: "CFDJ_ERR_ARG", -2: "CFDJ_ERR_HIP", -3: "CFDJ_ERR_ROCFFT",
             -4: "CFDJ_ERR_RCCL", -5: "CFDJ_ERR_NONFINITE", -6: "CFDJ_ERR_STATE"}
K_STAGE, K_FFT_FWD, K_DIVIDE, K_FFT_INV, K_COMM, K_COUNT = range(6)
K_NAMES = ("stage", "fft_fwd", "divide", "fft_inv", "comm")
# cfdj_vm_kernel_bench kernel ids (CFDJ_KB_*)
KB_NAMES = {1: "vm_stage<1>", 2: "vm_stage<2>", 3: "vm_stage<3>",
            4: "rows_fwd_kernel", 5: "cols_kernel", 6: "rows_inv_kernel"}
POISSON_AUTO, POISSON_ROCFFT, POISSON_FUSED, POISSON_SCHUR = 0, 1, 2, 3
SYMBOL_FD, SYMBOL_SPECTRAL = 0, 1
CAVITY_DST, CAVITY_MG = 0, 1
SPEC_HYBRID, SPEC_PS23, SPEC_PS32 = 0, 1, 2


class CfdjError(RuntimeError):
    def __init__(self, code, where, msg):
        self.code = code
        super().__init__(f"{where}: {ERR_NAMES.get(code, code)}: {msg}")


class ArgumentError(CfdjError, ValueError):
    """CFDJ_ERR_ARG -- the reference raises BoundsError/DivideError in these cases."""


_dp = C.POINTER(C.c_double)
_vp = C.c_void_p
_lp = C.POINTER(C.c_long)
_ip = C.POINTER(C.c_int)

# name -> (restype, argtypes); must list every symbol of include/cfdj.h.
SIGNATURES = {
    "cfdj_last_error": (C.c_char_p, []),
    "cfdj_version": (C.c_char_p, []),
    "cfdj_device_count": (C.c_int, []),
    "cfdj_fps_create": (C.c_int, [C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                  C.c_int, C.POINTER(_vp)]),
    "cfdj_fps_solve": (C.c_int, [_vp, _dp, C.c_long, _dp, C.c_long]),
    "cfdj_fps_solve_device": (C.c_int, [_vp, _vp, _vp]),
    "cfdj_fps_solve_device_noalloc": (C.c_int, [_vp, _vp, _vp]),
    "cfdj_fps_stream": (C.c_int, [_vp, C.POINTER(_vp)]),
    "cfdj_fps_destroy": (None, [_vp]),
    "cfdj_fps": (C.c_int, [C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, _dp,
                           C.c_long, _dp, C.c_long]),
    "cfdj_vm_create": (C.c_int, [C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                 C.c_double, C.c_int, C.POINTER(_vp)]),
    "cfdj_vm_create_dist": (C.c_int, [C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                      C.c_double, C.c_int, C.c_int, C.c_int, C.c_char_p,
                                      C.POINTER(_vp)]),
    "cfdj_comm_unique_id": (C.c_int, [C.c_char_p]),
    "cfdj_vm_comm_ranks": (C.c_int, [_vp, _ip]),
    "cfdj_vm_create_virtual": (C.c_int, [C.c_int, C.c_int, C.c_double, C.c_double,
                                         C.c_double, C.c_double, C.c_int, C.c_int,
                                         C.POINTER(_vp)]),
    "cfdj_vm_upload": (C.c_int, [_vp, _dp, C.c_long]),
    "cfdj_vm_download": (C.c_int, [_vp, _dp, C.c_long]),
    "cfdj_vm_step": (C.c_int, [_vp, C.c_double, C.c_int]),
    "cfdj_vm_step_async": (C.c_int, [_vp, C.c_double, C.c_int]),
    "cfdj_vm_sync": (C.c_int, [_vp]),
    "cfdj_vm_rhs": (C.c_int, [_vp, _dp, C.c_long, _dp, C.c_long, _dp, C.c_long]),
    "cfdj_vm_set_timing": (C.c_int, [_vp, C.c_int]),
    "cfdj_vm_timing": (C.c_int, [_vp, _dp, _lp]),
    "cfdj_vm_stage_timing": (C.c_int, [_vp, _dp, _lp]),
    "cfdj_vm_kernel_bench": (C.c_int, [_vp, C.c_int, C.c_double, C.c_int, _dp]),
    "cfdj_vm_set_check_finite": (C.c_int, [_vp, C.c_int]),
    "cfdj_vm_field_device": (C.c_int, [_vp, C.POINTER(_vp)]),
    "cfdj_vm_slab": (C.c_int, [_vp, _ip, _ip]),
    "cfdj_vm_set_rows_per_wave": (C.c_int, [_vp, C.c_int]),
    "cfdj_vm_stage_kernel": (C.c_int, [_vp, _ip]),
    "cfdj_vm_set_graph": (C.c_int, [_vp, C.c_int]),
    "cfdj_vm_set_poisson": (C.c_int, [_vp, C.c_int]),
    "cfdj_vm_get_poisson": (C.c_int, [_vp]),
    "cfdj_fps_set_poisson": (C.c_int, [_vp, C.c_int]),
    "cfdj_fps_get_poisson": (C.c_int, [_vp]),
    "cfdj_fps_set_symbol": (C.c_int, [_vp, C.c_int]),
    "cfdj_vm_destroy": (None, [_vp]),
    "cfdj_cavity_create": (C.c_int, [C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                     C.c_int, C.POINTER(_vp)]),
    "cfdj_cavity_set_poisson": (C.c_int, [_vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                          C.c_double, C.c_int]),
    "cfdj_cavity_upload": (C.c_int, [_vp, _dp, C.c_long, _dp, C.c_long]),
    "cfdj_cavity_download": (C.c_int, [_vp, _dp, C.c_long, _dp, C.c_long]),
    "cfdj_cavity_step": (C.c_int, [_vp, C.c_double, C.c_int, _dp]),
    "cfdj_cavity_rhs": (C.c_int, [_vp, _dp, C.c_long, _dp, C.c_long, _dp, C.c_long]),
    "cfdj_cavity_mg_iterations": (C.c_long, [_vp]),
    "cfdj_cavity_destroy": (None, [_vp]),
    "cfdj_fps_sine": (C.c_int, [C.c_int, C.c_int, C.c_double, C.c_double, _dp, C.c_long, _dp,
                                C.c_long]),
    "cfdj_mg_create": (C.c_int, [C.c_int, C.c_int, C.c_double, C.c_double, C.c_int, C.c_int,
                                 C.c_int, C.c_int, C.c_int, C.POINTER(_vp)]),
    "cfdj_mg_solve": (C.c_int, [_vp, _dp, C.c_long, _dp, C.c_long, C.c_double, C.c_int, _ip,
                                _dp]),
    "cfdj_mg_residual": (C.c_int, [_vp, _dp, C.c_long]),
    "cfdj_mg_destroy": (None, [_vp]),
    "cfdj_jacobi_solve": (C.c_int, [C.c_int, C.c_int, C.c_double, C.c_double, _dp, C.c_long,
                                    _dp, C.c_long, C.c_long, C.c_double, C.c_long, _lp, _dp]),
    "cfdj_ftcs": (C.c_int, [C.c_int, C.c_int, C.c_double, _dp, _dp, C.c_long]),
    "cfdj_spec_create": (C.c_int, [C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                   C.c_double, C.c_int, C.c_int, C.POINTER(_vp)]),
    "cfdj_spec_upload": (C.c_int, [_vp, _dp, C.c_long]),
    "cfdj_spec_step": (C.c_int, [_vp, C.c_double, C.c_int]),
    "cfdj_spec_download": (C.c_int, [_vp, _dp, C.c_long]),
    "cfdj_spec_get_spectrum": (C.c_int, [_vp, _dp]),
    "cfdj_spec_set_spectrum": (C.c_int, [_vp, _dp]),
    "cfdj_spec_jacobian": (C.c_int, [_vp, _dp, _dp]),
    "cfdj_spec_destroy": (None, [_vp]),
}

_lock = threading.Lock()
_lib = None


def load():
    """Load libcfdj.so (raises CfdjError if it has not been built)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise CfdjError(-6, "load", f"{LIB_PATH} not built: run "
                                "`make -C cfd_julia_amd/csrc` or __graft_entry__.build()")
            lib = C.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def check(rc, where):
    if rc != CFDJ_OK:
        msg = load().cfdj_last_error().decode(errors="replace")
        cls = ArgumentError if rc == -1 else CfdjError
        raise cls(rc, where, msg)


def require_gpu():
    n = load().cfdj_device_count()
    if n <= 0:
        raise CfdjError(-2, "device", "no HIP device visible: libcfdj has no CPU path")
    return n


def dptr(a: np.ndarray):
    assert a.dtype == np.float64
    return a.ctypes.data_as(_dp)


def fortran_view(a, name, shape_min, writable=False):
    """Validate a Julia-layout (column-major) float64 array; returns (array, ld)."""
    if not isinstance(a, np.ndarray) or a.dtype != np.float64:
        raise TypeError(f"{name} must be a float64 numpy array")
    if a.ndim != 2 or a.shape[0] < shape_min[0] or a.shape[1] < shape_min[1]:
        raise ArgumentError(-1, name, f"shape {a.shape} smaller than {shape_min} (BoundsError)")
    if not a.flags.f_contiguous:
        raise ArgumentError(-1, name, "must be Fortran-ordered (Julia column-major layout)")
    if writable and not a.flags.writeable:
        raise ArgumentError(-1, name, "must be writable")
    return a, a.shape[0]
