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
        import ctypes.util

        from cfd_julia_amd import _lib

        self.C = C
        _lib.load()  # libcfdj.so brings its own HIP runtime into the process
        name = ctypes.util.find_library("amdhip64") or "libamdhip64.so"
        self.rt = C.CDLL(name)
        self.rt.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        self.rt.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        self.rt.hipFree.argtypes = [C.c_void_p]
        self.rt.hipMemGetInfo.argtypes = [C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
        self.rt.hipStreamSynchronize.argtypes = [C.c_void_p]

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

    def free_bytes(self):
        free, total = self.C.c_size_t(), self.C.c_size_t()
        self.ok(self.rt.hipMemGetInfo(self.C.byref(free), self.C.byref(total)), "hipMemGetInfo")
        return free.value

    def sync(self, stream):
        self.ok(self.rt.hipStreamSynchronize(self.C.c_void_p(stream)), "hipStreamSynchronize")

    def free(self, *ps):
        for p in ps:
            self.ok(self.rt.hipFree(p), "hipFree")


def _solve_both(hip, cfdj, nx, ny, seed):
    """The no-alloc solve FIRST, on a plan whose own spectrum buffer has never been written
    (so nothing it produces can come from there), with the device's free memory read before
    and after it; then the allocating entry point on the same plan."""
    dx, dy = 2 * np.pi / nx, 2 * np.pi / ny
    f = np.random.default_rng(seed).standard_normal((ny, nx))  # rows = y, x contiguous
    nan = np.full((ny, nx), np.nan)
    bufs = []
    try:
        with cfdj.PoissonFFT(nx, ny, dx, dy, device=0) as h:
            assert h.poisson() == "fused"
            for a in (f, nan, nan):
                bufs.append(hip.to_device(a))
            fd, ad, bd = bufs
            hip.sync(h.stream())
            free0 = hip.free_bytes()
            h.solve_device_noalloc(fd.value, bd.value)
            hip.sync(h.stream())  # the accessor's stream is the one the kernels ran on
            free1 = hip.free_bytes()
            b = hip.to_host(bd, (ny, nx))
            h.solve_device(fd.value, ad.value)
            a = hip.to_host(ad, (ny, nx))
    finally:
        hip.free(*bufs)
    return f, a, b, free0 - free1


def test_gpu_noalloc_matches_solve_device_twice(cfdj):
    from oracle import vm_oracle as vo

    hip = _Hip()
    # load the library's kernels once (a first launch may make the runtime allocate for the
    # code object: not the entry point's doing)
    _solve_both(hip, cfdj, 1024, 1024, 0)
    for nx, ny, seed in [(2048, 1024, 1), (1024, 1024, 2)]:  # second call: smaller input
        print(f"noalloc case nx={nx} ny={ny} seed={seed}", flush=True)
        f, a, b, used = _solve_both(hip, cfdj, nx, ny, seed)
        assert used == 0, f"device free memory changed by {used} bytes across the call"
        assert np.isfinite(a).all() and np.isfinite(b).all()
        assert np.array_equal(a, b)
        # and the result itself against the oracle (device rows are y: transpose)
        if nx == ny:
            ref = vo.fps(np.asfortranarray(f.T), 2 * np.pi / nx, 2 * np.pi / ny)
            assert np.abs(b.T - ref).max() <= 1e-12 * np.abs(ref).max()


def test_gpu_noalloc_rejects_oversize_and_rocfft_plans(cfdj):
    hip = _Hip()
    z = hip.to_device(np.zeros(16))
    try:
        with cfdj.PoissonFFT(2048, 2048, 1.0, 1.0, device=0) as h:  # 2 Mi complex > 1 Mi
            with pytest.raises(cfdj.ArgumentError, match="exceed the static scratch"):
                h.solve_device_noalloc(z.value, z.value)
        with cfdj.PoissonFFT(64, 64, 1.0, 1.0, device=0) as h:  # rocFFT path
            with pytest.raises(cfdj.ArgumentError, match="hand-written FFT path"):
                h.solve_device_noalloc(z.value, z.value)
    finally:
        hip.free(z)
