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


def test_secondary_mirrors_validate_arrays_before_the_c_call():
    """cavity.fps_sine / numerical, mg.Multigrid.solve and gauss_seidel check shape, order and
    dtype of caller arrays (the C side copies (nx+1) x (ny+1) nodes in and out) -- raised
    before anything touches the GPU, so this runs on CPU."""
    import numpy as np

    from cfd_julia_amd import _lib, cavity, gauss_seidel
    from cfd_julia_amd import mg as mgmod

    n = 16
    f = np.zeros((n + 1, n + 1), order="F")
    with pytest.raises(_lib.ArgumentError):  # C-ordered output would come back transposed
        cavity.fps_sine(n, n, 1.0 / n, 1.0 / n, f, sn=np.zeros((n + 1, n + 2)))
    with pytest.raises(_lib.ArgumentError):  # short output: out-of-bounds host write
        cavity.fps_sine(n, n, 1.0 / n, 1.0 / n, f, sn=np.zeros((n, n), order="F"))
    with pytest.raises(_lib.ArgumentError):
        cavity.fps_sine(n, n, 1.0 / n, 1.0 / n, np.zeros((n, n), order="F"))
    with pytest.raises(TypeError):
        cavity.fps_sine(n, n, 1.0 / n, 1.0 / n, f, sn=np.zeros((n + 1, n + 1), np.float32, order="F"))
    with pytest.raises(_lib.ArgumentError):
        cavity.numerical(n, n, 2, 1.0 / n, 1.0 / n, 1e-3, 100.0, np.zeros((n, n), order="F"),
                         np.zeros((n + 1, n + 1), order="F"), np.zeros(2))
    with pytest.raises(_lib.ArgumentError):
        cavity.numerical(n, n, 2, 1.0 / n, 1.0 / n, 1e-3, 100.0, f.copy(order="F"),
                         f.copy(order="F"), np.zeros(1))
    with pytest.raises(_lib.ArgumentError):
        gauss_seidel.gauss_seidel(1.0 / n, 1.0 / n, n, n, None, f, np.zeros((n, n + 1), order="F"),
                                  10, 1e-9)
    with pytest.raises(_lib.ArgumentError):
        gauss_seidel.gauss_seidel(1.0 / n, 1.0 / n, n, n, None, np.zeros((n + 1, n)), f.copy(order="F"),
                                  10, 1e-9)
    m = mgmod.Multigrid.__new__(mgmod.Multigrid)  # no handle: validation comes first
    m._h, m.nx, m.ny = None, n, n
    with pytest.raises(_lib.ArgumentError):
        m.solve(f, np.zeros((n, n), order="F"))
    with pytest.raises(_lib.ArgumentError):
        m.solve(f, np.zeros((n + 1, n + 2))[:, :n + 1])  # C-ordered view
    with pytest.raises(_lib.ArgumentError):
        m.residual(np.zeros((n, n + 1), order="F"))


def test_julia_shim_ccalls_match_the_header():
    """julia/CFDJ.jl cannot run here (no julia): check statically that every ccall names an
    exported symbol and passes as many arguments, of the matching C kind, as the binding."""
    import ctypes as C
    import re

    src = open(os.path.join(ROOT, "julia", "CFDJ.jl"), encoding="utf-8").read()
    calls = re.findall(r"ccall\(\(:(\w+),\s*libcfdj\),\s*(\w+),\s*\(([^)]*)\)", src)
    assert len(calls) >= 20
    kind = {"Cint": C.c_int, "Clong": C.c_long, "Cdouble": C.c_double}
    seen = set()
    for name, ret, types in calls:
        assert name in _lib.SIGNATURES, name
        res, args = _lib.SIGNATURES[name]
        jl = [t.strip() for t in types.split(",") if t.strip()]
        assert len(jl) == len(args), (name, jl, args)
        for t, a in zip(jl, args):
            if t in kind:
                assert a is kind[t], (name, t, a)
            else:  # Ptr{...} / Ref{...} / Cstring: a pointer on the C side
                assert t.startswith(("Ptr{", "Ref{")) and a not in kind.values(), (name, t, a)
        assert {"Cint": C.c_int, "Cvoid": None, "Cstring": C.c_char_p}[ret] is res or \
            (ret == "Cstring" and res is C.c_char_p), (name, ret)
        seen.add(name)
    # the entry points the north star names as drop-in: vm.jl, lid_driven_cavity.jl, mg.jl
    for must in ("cfdj_vm_step", "cfdj_vm_rhs", "cfdj_fps_solve", "cfdj_cavity_step",
                 "cfdj_cavity_rhs", "cfdj_fps_sine", "cfdj_mg_solve", "cfdj_mg_residual"):
        assert must in seen, must
    assert "VM_CACHE" in src and "cached_vm(nx, ny" in src  # vm_rhs reuses its handle
