"""GPU parity of the FFT-fused stage kernel (vm_fused.hip): row c2r of the column-pass
output + Arakawa/Laplacian/RK3 stage + the next stage's row r2c in one kernel per stage,
psi never written to HBM.

Oracle: oracle/vm_oracle.py's restatement of vm.jl:12-90 / Common.jl:97-182.  Tolerances
as tests/test_gpu_parity.py: vorticity after K RK3 steps L-inf < 1e-10 (north star);
the fused and the five-pass GPU paths agree to FFT round-off (1e-12 absolute, |w| ~ 1).
Sizes cover the three row-group shapes of the kernel: nx = 1024 (8 rows per step),
2048 (4 rows), 4096 (2 rows), and rectangular grids (the mirrored symbol of ny < nx).
"""
import numpy as np
import pytest

from oracle import vm_oracle as vo

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cfdj():
    import cfd_julia_amd
    from cfd_julia_amd import _lib

    assert _lib.require_gpu() >= 1
    return cfd_julia_amd


def setup(nx, ny):
    dx, dy, x, y = vo.vm_grid(nx, ny)
    return dx, dy, vo.vm_ic(nx, ny, x, y), 5e-4 * (4096 / nx) ** 2


def run(cfdj, nx, ny, w0, dt, splits, fused=True):
    dx, dy, _, _ = vo.vm_grid(nx, ny)
    with cfdj.VortexMerger(nx, ny, dx, dy, 1000.0) as h:
        h.set_fused_stage(fused)
        assert h.fused_stage() == fused
        h.upload_interior(w0)
        for k in splits:
            h.step(dt, k)
        return h.download_interior()


@pytest.mark.parametrize("nx,ny,steps", [(1024, 1024, 8), (2048, 2048, 4), (4096, 4096, 2),
                                         (2048, 1024, 4), (4096, 1024, 3), (4096, 2048, 2),
                                         (1024, 2048, None)])
def test_gpu_fused_stage_vs_oracle(cfdj, nx, ny, steps):
    if steps is None:  # ny > nx: the reference's ky = kx aliasing raises (BoundsError)
        dx, dy, _, _ = vo.vm_grid(nx, ny)
        with pytest.raises(cfdj.ArgumentError):
            cfdj.VortexMerger(nx, ny, dx, dy, 1000.0)
        return
    dx, dy, w0, dt = setup(nx, ny)
    ref = vo.numerical(w0, steps, dt, dx, dy, 1000.0)
    w = run(cfdj, nx, ny, w0, dt, [steps])
    assert np.abs(w - ref).max() < 1e-10


@pytest.mark.parametrize("n", [1024, 4096])
def test_gpu_fused_stage_matches_five_pass(cfdj, n):
    _, _, w0, dt = setup(n, n)
    a = run(cfdj, n, n, w0, dt, [5], fused=True)
    b = run(cfdj, n, n, w0, dt, [5], fused=False)
    assert np.abs(a - b).max() < 1e-12


def test_gpu_fused_stage_call_splits(cfdj):
    """Each call starts with a row r2c of omega^n and skips the last stage's r2c: splitting
    K steps over several calls only moves FFT round-off."""
    n = 2048
    _, _, w0, dt = setup(n, n)
    a = run(cfdj, n, n, w0, dt, [6])
    b = run(cfdj, n, n, w0, dt, [1, 2, 3])
    assert np.abs(a - b).max() < 1e-13


def test_gpu_fused_stage_selection(cfdj):
    dx, dy, _, _ = vo.vm_grid(1024, 1024)
    with cfdj.VortexMerger(1024, 1024, dx, dy, 1000.0) as h:
        h.set_fused_stage(True)
        assert h.fused_stage()
        h.set_poisson("rocfft")  # needs the fused Poisson column pass
        assert not h.fused_stage()
        h.set_poisson("auto")
        assert h.fused_stage()
    with cfdj.VortexMerger(512, 512, dx, dy, 1000.0) as h:  # below the fused sizes
        h.set_fused_stage(True)
        assert not h.fused_stage()
    with cfdj.VortexMerger(8192, 1024, dx, dy, 1000.0) as h:  # rows beyond the LDS slots
        h.set_fused_stage(True)
        assert h.poisson() == "fused" and not h.fused_stage()
    with cfdj.VortexMerger(1024, 1024, dx, dy, 1000.0, kind="virtual", nranks=2) as h:
        h.set_fused_stage(True)
        assert not h.fused_stage()  # y-slabs keep the separate passes


def test_gpu_fused_stage_kernel_bench(cfdj):
    from cfd_julia_amd import _lib

    n = 4096
    _, _, w0, _ = setup(n, n)
    dx, dy, _, _ = vo.vm_grid(n, n)
    with cfdj.VortexMerger(n, n, dx, dy, 1000.0) as h:
        h.upload_interior(w0)
        for kid in (7, 8, 9, 10):
            assert h.kernel_bench(kid, 5e-4, 3) > 0
    with cfdj.VortexMerger(8192, 1024, dx, dy, 1000.0) as h:
        with pytest.raises(_lib.ArgumentError):
            h.kernel_bench(7, 1e-4, 1)
