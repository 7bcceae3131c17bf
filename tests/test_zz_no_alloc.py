"""cfdj_fps_solve_device_noalloc (the entry point that allocates nothing: half spectrum in
the library's static device array) against cfdj_fps_solve_device, through the C ABI.

Both run the same three hand-written FFT passes with the same tables, so the results must be
bit-identical; two calls in a row, the second on a smaller grid (stale spectrum of the larger
solve left in the shared array)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cfdj():
    import cfd_julia_amd
    from cfd_julia_amd import _lib

    assert _lib.require_gpu() >= 1
    return cfd_julia_amd


class _Hip:
    """Device buffers through the HIP runtime the library itself is linked against (ctypes):
    the test must not depend on which of torch / libcfdj initialised the GPU first."""

    def __init__(self):
        import ctypes as C

        self.C = C
        self.rt = C.CDLL("libamdhip64.so.7")
        self.rt.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        self.rt.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        self.rt.hipFree.argtypes = [C.c_void_p]

    def ok(self, rc, what):
        assert rc == 0, f"{what}: hipError {rc}"

    def to_device(self, a):
        p = self.C.c_void_p()
        self.ok(self.rt.hipMalloc(self.C.byref(p), a.nbytes), "hipMalloc")
        self.ok(self.rt.hipMemcpy(p, a.ctypes.data, a.nbytes, 1), "hipMemcpy H2D")
        return p

    def to_host(self, p, shape):
        out = np.empty(shape)
        self.ok(self.rt.hipDeviceSynchronize(), "hipDeviceSynchronize")
        self.ok(self.rt.hipMemcpy(out.ctypes.data, p, out.nbytes, 2), "hipMemcpy D2H")
        return out

    def free(self, *ps):
        for p in ps:
            self.ok(self.rt.hipFree(p), "hipFree")


def _solve_both(hip, cfdj, nx, ny, seed):
    dx, dy = 2 * np.pi / nx, 2 * np.pi / ny
    f = np.random.default_rng(seed).standard_normal((ny, nx))  # rows = y, x contiguous
    nan = np.full((ny, nx), np.nan)
    with cfdj.PoissonFFT(nx, ny, dx, dy, device=0) as h:
        assert h.poisson() == "fused"
        fd, ad, bd = hip.to_device(f), hip.to_device(nan), hip.to_device(nan)
        h.solve_device(fd.value, ad.value)
        a = hip.to_host(ad, (ny, nx))
        h.solve_device_noalloc(fd.value, bd.value)
        b = hip.to_host(bd, (ny, nx))
        hip.free(fd, ad, bd)
    return f, a, b


def test_gpu_noalloc_matches_solve_device_twice(cfdj):
    from oracle import vm_oracle as vo

    hip = _Hip()
    for nx, ny, seed in [(2048, 1024, 1), (1024, 1024, 2)]:  # second call: smaller input
        print(f"noalloc case nx={nx} ny={ny} seed={seed}", flush=True)
        f, a, b = _solve_both(hip, cfdj, nx, ny, seed)
        assert np.isfinite(a).all() and np.isfinite(b).all()
        assert np.array_equal(a, b)
        # and the result itself against the oracle (device rows are y: transpose)
        if nx == ny:
            ref = vo.fps(np.asfortranarray(f.T), 2 * np.pi / nx, 2 * np.pi / ny)
            assert np.abs(b.T - ref).max() <= 1e-12 * np.abs(ref).max()


def test_gpu_noalloc_rejects_oversize_and_rocfft_plans(cfdj):
    hip = _Hip()
    z = hip.to_device(np.zeros(16))
    with cfdj.PoissonFFT(2048, 2048, 1.0, 1.0, device=0) as h:  # 2 Mi complex > 1 Mi
        with pytest.raises(cfdj.ArgumentError, match="exceed the static scratch"):
            h.solve_device_noalloc(z.value, z.value)
    with cfdj.PoissonFFT(64, 64, 1.0, 1.0, device=0) as h:  # rocFFT path
        with pytest.raises(cfdj.ArgumentError, match="hand-written FFT path"):
            h.solve_device_noalloc(z.value, z.value)
    hip.free(z)
