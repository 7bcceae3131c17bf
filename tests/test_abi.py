"""CPU tests of the C-ABI boundary: the library loads, exports exactly the entry points
include/cfdj.h declares, and validates arguments the way the reference fails
(BoundsError / DivideError analogues) without touching a GPU."""
import ctypes as C
import os
import re

import pytest

from cfd_julia_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(ROOT, "include", "cfdj.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(cfdj_\w+)\s*\(", text))


def test_header_and_binding_agree():
    assert header_functions() == set(_lib.SIGNATURES)


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert b"gfx950" in lib.cfdj_version()


def test_elf_dynamic_symbols():
    # the .so exports the C names unmangled
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (cfdj_\w+)", out))
    assert header_functions() <= exported


def test_device_count_never_fails():
    n = _lib.load().cfdj_device_count()
    assert n >= 0


def _create(nx, ny, dx=0.1, dy=0.1, re=1000.0):
    h = C.c_void_p()
    rc = _lib.load().cfdj_vm_create(nx, ny, dx, dy, re, 1e-6, -1, C.byref(h))
    return rc, h


@pytest.mark.parametrize("nx,ny,why", [(63, 63, "even"), (64, 128, "BoundsError"),
                                       (2, 2, ">= 4")])
def test_argument_errors_are_reported(nx, ny, why):
    rc, h = _create(nx, ny)
    assert rc == -1 and not h.value
    assert why in _lib.load().cfdj_last_error().decode()


def test_bad_spacing_and_reynolds():
    assert _create(64, 64, dx=-1.0)[0] == -1
    assert _create(64, 64, re=0.0)[0] == -1
    h = C.c_void_p()
    assert _lib.load().cfdj_fps_create(65, 64, 0.1, 0.1, 1e-6, -1, C.byref(h)) == -1


def test_null_handles_are_safe():
    lib = _lib.load()
    lib.cfdj_vm_destroy(None)
    lib.cfdj_fps_destroy(None)
    assert lib.cfdj_vm_step(None, 0.1, 1) == -1
    assert lib.cfdj_vm_sync(None) == -1


def test_python_wrappers_fail_loudly_without_gpu():
    if _lib.load().cfdj_device_count() > 0:
        pytest.skip("GPU present")
    from cfd_julia_amd import VortexMerger

    with pytest.raises(_lib.CfdjError):
        VortexMerger(64, 64, 0.1, 0.1, 1000.0)


def test_product_path_does_not_import_oracle():
    pkg = os.path.join(ROOT, "cfd_julia_amd")
    pat = re.compile(r"^\s*(import|from)\s+oracle|import_module\(.oracle|oracle/_ref|"
                     r"#include\s+\S*oracle", re.M)
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".cpp", ".h", "Makefile")):
                src = open(os.path.join(dirpath, f)).read()
                assert not pat.search(src), f
