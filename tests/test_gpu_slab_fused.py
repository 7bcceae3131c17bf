"""GPU parity of the generalised hand-written Poisson path (poisson_fft.hip):

  * rectangular grids ny < nx (Common.jl:112-123 with the ky = kx aliasing: the symbol is
    not even in ky, so the fused column pass applies the Hermitian projection that
    real(ifft(...)) performs) and the long-row / long-column kernels (nx up to 16384,
    ny up to 8192) that the multi-GPU weak-scaling grids need;
  * the y-slab path with the fused passes (row r2c -> all-to-all of column blocks ->
    segmented column pass -> all-to-all -> row c2r), run as P virtual ranks on one GPU,
    against the single-domain CPU oracle.

Tolerances as tests/test_gpu_parity.py: psi within 1e-12 * max|psi| (FFT round-off),
vorticity after K RK3 steps L-inf < 1e-10.
"""
import numpy as np
import pytest

from oracle import vm_oracle as vo
from tests.golden.make_golden import smooth_field, smooth_field_fast

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cfdj():
    import cfd_julia_amd
    from cfd_julia_amd import _lib

    assert _lib.require_gpu() >= 1
    return cfd_julia_amd


def field(nx, ny, seed):
    rng = np.random.default_rng(seed)
    smooth = smooth_field_fast if nx * ny >= 1 << 22 else smooth_field
    return np.asfortranarray(smooth(nx, ny, 3, seed) + 0.01 * rng.standard_normal((nx, ny)))


@pytest.mark.parametrize("nx,ny", [(2048, 1024), (4096, 2048), (8192, 1024), (16384, 1024),
                                   (2048, 2048)])
def test_gpu_fused_rect_fps_vs_oracle(cfdj, nx, ny):
    dx, dy, _, _ = vo.vm_grid(nx, ny)
    f = field(nx, ny, nx + ny)
    ref = vo.fps(f, dx, dy)
    with cfdj.PoissonFFT(nx, ny, dx, dy) as h:
        assert h.poisson() == "fused"
        s_f = h.solve(f)
        h.set_poisson("rocfft")
        s_r = h.solve(f)
    scale = np.abs(ref).max()
    assert np.abs(s_r - ref).max() <= 1e-12 * scale
    assert np.abs(s_f - ref).max() <= 1e-12 * scale, np.abs(s_f - ref).max() / scale


def test_gpu_fused_fps_8192_square(cfdj):
    # the 8192-point column kernel (one column per CU, 139 KB LDS) and 8192-point rows
    n = 8192
    dx, dy, _, _ = vo.vm_grid(n, n)
    f = field(n, n, 7)
    ref = vo.fps(f, dx, dy)
    with cfdj.PoissonFFT(n, n, dx, dy) as h:
        assert h.poisson() == "fused"
        s_f = h.solve(f)
    scale = np.abs(ref).max()
    assert np.abs(s_f - ref).max() <= 1e-12 * scale, np.abs(s_f - ref).max() / scale


@pytest.mark.parametrize("nx,ny,steps", [(2048, 1024, 4), (4096, 1024, 2)])
def test_gpu_fused_rect_vm_vs_oracle(cfdj, nx, ny, steps):
    dx, dy, x, y = vo.vm_grid(nx, ny)
    w0 = vo.vm_ic(nx, ny, x, y)
    dt = 5e-4 * (4096 / nx) ** 2
    ref = vo.numerical(w0, steps, dt, dx, dy, 1000.0)
    with cfdj.VortexMerger(nx, ny, dx, dy, 1000.0) as h:
        assert h.poisson() == "fused"
        h.upload_interior(w0)
        h.step(dt, steps)
        w = h.download_interior()
    assert np.abs(w - ref).max() < 1e-10


@pytest.mark.parametrize("P,nx,ny,steps", [(1, 1024, 1024, 3), (2, 1024, 1024, 3),
                                           (4, 1024, 1024, 3), (8, 1024, 1024, 3),
                                           (2, 2048, 1024, 2), (4, 2048, 1024, 2),
                                           (8, 2048, 2048, 2)])
def test_gpu_fused_virtual_slabs_vs_oracle(cfdj, P, nx, ny, steps):
    dx, dy, x, y = vo.vm_grid(nx, ny)
    w0 = vo.vm_ic(nx, ny, x, y)
    dt = 5e-4 * (4096 / nx) ** 2
    ref = vo.numerical(w0, steps, dt, dx, dy, 1000.0)
    with cfdj.VortexMerger(nx, ny, dx, dy, 1000.0, kind="virtual", nranks=P) as h:
        h.set_poisson("fused")  # the transpose path (AUTO prefers "schur" where it applies)
        assert h.poisson() == "fused"
        h.upload_interior(w0)
        h.step(dt, steps)
        w = h.download_interior()
    assert np.abs(w - ref).max() < 1e-10


def test_gpu_fused_virtual_matches_rocfft_slabs(cfdj):
    # the same slab decomposition through rocFFT + pack/unpack: identical up to FFT round-off
    nx, ny, P = 2048, 1024, 4
    dx, dy, x, y = vo.vm_grid(nx, ny)
    w0 = vo.vm_ic(nx, ny, x, y)
    out = {}
    for path in ("fused", "rocfft"):
        with cfdj.VortexMerger(nx, ny, dx, dy, 1000.0, kind="virtual", nranks=P) as h:
            h.set_poisson(path)
            h.upload_interior(w0)
            h.step(2e-3, 3)
            out[path] = h.download_interior()
    assert np.abs(out["fused"] - out["rocfft"]).max() < 1e-12


def test_gpu_fused_slab_path_selection(cfdj):
    dx, dy, _, _ = vo.vm_grid(1024, 1024)
    # 3 ranks do not split the 512 column blocks evenly: rocFFT slab path
    with cfdj.VortexMerger(1536, 768, dx, dy, 1000.0, kind="virtual", nranks=3) as h:
        assert h.poisson() == "rocfft"
        with pytest.raises(cfdj.ArgumentError):
            h.set_poisson("fused")
    with cfdj.VortexMerger(1024, 1024, dx, dy, 1000.0, kind="virtual", nranks=4) as h:
        assert h.poisson() == "fused"
        h.set_poisson("rocfft")
        assert h.poisson() == "rocfft"
        h.set_poisson("auto")
        assert h.poisson() == "fused"
