"""GPU parity of the secondary paths: lid-driven cavity and multigrid.

Tolerances: cavity rhs bit-exact given (w, s); fps_sine within 1e-12 max|s| (DST via the
odd-extension FFT vs scipy's DST-I); cavity fields after K steps within 1e-10; multigrid:
red-black vs the reference's lexicographic smoother -> converged solutions compared at the
solver tolerance, and the ipr=1 MMS (exact for the 5-point Laplacian) to ~1e-8.
"""
import numpy as np
import pytest

from oracle import cavity_oracle as co
from tests.golden.make_golden import smooth_field

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from cfd_julia_amd import _lib

    assert _lib.require_gpu() >= 1
    return _lib


@pytest.mark.parametrize("n", [16, 64, 96])
def test_gpu_cavity_rhs_bit_exact(lib, n):
    from cfd_julia_amd.cavity import Cavity

    dx, dy, _, _ = co.cavity_grid(n, n)
    w = np.asfortranarray(np.pad(smooth_field(n - 1, n - 1, 3, 61), ((1, 1), (1, 1)))[:n + 1, :n + 1])
    s = np.asfortranarray(np.pad(smooth_field(n - 1, n - 1, 3, 62), ((1, 1), (1, 1)))[:n + 1, :n + 1])
    with Cavity(n, n, dx, dy, 100.0) as h:
        r = h.rhs(w, s)
    ref = co.cavity_rhs(w, s, dx, dy, 100.0)
    assert np.array_equal(r, ref)


@pytest.mark.parametrize("n", [16, 64, 512, 1024])
def test_gpu_fps_sine_vs_oracle(lib, n):
    from cfd_julia_amd.cavity import fps_sine

    dx, dy, _, _ = co.cavity_grid(n, n)
    f = np.zeros((n + 1, n + 1), order="F")
    f[1:n, 1:n] = smooth_field(n - 1, n - 1, 4, 63)
    s = fps_sine(n, n, dx, dy, f)
    ref = co.fps_sine(f, dx, dy)
    assert np.all(s[0, :] == 0) and np.all(s[:, 0] == 0) and np.all(s[n, :] == 0)
    assert np.abs(s - ref).max() <= 1e-12 * np.abs(ref).max()


@pytest.mark.parametrize("n,nt", [(32, 50), (64, 20), (512, 3)])
def test_gpu_cavity_steps_vs_oracle(lib, n, nt):
    from cfd_julia_amd import cavity

    dt = 0.001 * (64 / n) ** 2
    dx, dy, _, _ = co.cavity_grid(n, n)
    wn = np.zeros((n + 1, n + 1), order="F")
    sn = np.zeros((n + 1, n + 1), order="F")
    rms = np.zeros(nt)
    cavity.numerical(n, n, nt, dx, dy, dt, 100.0, wn, sn, rms)
    w_ref, s_ref, rms_ref = co.cavity_numerical(n, n, nt, dt, 100.0)
    assert np.abs(wn - w_ref).max() < 1e-10 * max(1.0, np.abs(w_ref).max())
    assert np.abs(sn - s_ref).max() < 1e-12
    assert np.allclose(rms, rms_ref, rtol=1e-8, atol=1e-16)


def test_gpu_cavity_reference_default_run_to_steady_state(lib):
    """lid_driven_cavity.jl:162-172 as shipped: 64^2, dt = .001, tf = 10 (10000 steps),
    re = 100.  Against the oracle's fields after the same steps, and against the primary
    vortex of the literature's Re = 100 cavity (Ghia, Ghia & Shin 1982: psi = -0.1034 at
    (0.6172, 0.7344)), which a 64^2 second-order solution meets within a percent."""
    from cfd_julia_amd import cavity

    n, nt, dt = 64, 10000, 0.001
    dx, dy, _, _ = co.cavity_grid(n, n)
    wn = np.zeros((n + 1, n + 1), order="F")
    sn = np.zeros((n + 1, n + 1), order="F")
    rms = np.zeros(nt)
    cavity.numerical(n, n, nt, dx, dy, dt, 100.0, wn, sn, rms)
    i, j = np.unravel_index(np.abs(sn).argmax(), sn.shape)
    assert abs(sn[i, j] + 0.1034) < 0.001, sn[i, j]
    assert abs(i * dx - 0.6172) <= dx and abs(j * dy - 0.7344) <= dy, (i, j)
    assert rms[-1] < 1e-6  # steady
    w_ref, s_ref, rms_ref = co.cavity_numerical(n, n, nt, dt, 100.0)
    assert np.abs(sn - s_ref).max() < 1e-11
    assert np.abs(wn - w_ref).max() < 1e-9 * np.abs(w_ref).max()
    assert np.allclose(rms, rms_ref, rtol=1e-6, atol=1e-14)


@pytest.mark.parametrize("nx,ny", [(512, 64), (1024, 256), (1536, 34), (4096, 16)])
def test_gpu_cavity_row_group_stage_matches_separate_kernels(lib, monkeypatch, nx, ny):
    """The fused row-group stage + wall-vorticity kernel (nx a multiple of 512, ny even) and
    the separate interior-stage and bc2 kernels give the same bits, walls and corners
    included, from a non-trivial state."""
    from cfd_julia_amd.cavity import Cavity

    dx, dy = 1.0 / nx, 1.0 / ny
    dt = 0.2 * min(dx, dy) ** 2 * 100.0 / 4
    rng = np.random.default_rng(nx + ny)
    w0 = np.asfortranarray(rng.standard_normal((nx + 1, ny + 1)))
    s0 = np.zeros((nx + 1, ny + 1), order="F")
    s0[1:nx, 1:ny] = 1e-3 * rng.standard_normal((nx - 1, ny - 1))
    outs = []
    for tile in ("1", "0"):
        monkeypatch.setenv("CFDJ_CAVITY_TILE", tile)
        with Cavity(nx, ny, dx, dy, 100.0, poisson="dst") as h:
            h.upload(w0, s0)
            rms = h.step(dt, 2)
            outs.append(h.download() + (rms,))
    for a, b in zip(outs[0], outs[1]):
        assert np.isfinite(a).all()
        assert np.array_equal(a, b)


def test_gpu_cavity_mg_matches_dst(lib):
    from cfd_julia_amd.cavity import Cavity

    n, nt, dt = 64, 20, 0.001
    dx, dy, _, _ = co.cavity_grid(n, n)
    out = {}
    for p in ("dst", "mg"):
        with Cavity(n, n, dx, dy, 100.0, poisson=p, tol=1e-12) as h:
            rms = h.step(dt, nt)
            out[p] = h.download() + (rms, h.mg_iterations() if p == "mg" else 0)
    (w1, s1, r1, _), (w2, s2, r2, its) = out["dst"], out["mg"]
    assert its > 0
    assert np.abs(s1 - s2).max() < 1e-9 * np.abs(s1).max()
    assert np.abs(w1 - w2).max() < 1e-6 * np.abs(w1).max()


@pytest.mark.parametrize("n,levels", [(64, 5), (512, 9)])
def test_gpu_mg_mms(lib, n, levels):
    from cfd_julia_amd import mg

    f, ue, un, dx, dy = mg.mms(n)
    it, hist = mg.mg_N(dx, dy, n, n, None, f, un, 2, 2, 2, 100000, 1e-9, n_level=levels)
    assert hist[-1] / hist[0] <= 1e-9 and it < 50
    # ipr = 1: (x^2-1)(y^2-1) is exact for the 5-point Laplacian -> solver error only
    assert np.abs(un - ue).max() < 1e-7
    # the red-black GPU V-cycle vs the oracle's red-black restatement: same iterations,
    # residual histories equal to round-off
    if n <= 64:
        u0 = mg.mms(n)[2]
        u_o, it_o, hist_o = co.mg_n(f, u0, dx, dy, levels)
        assert it == it_o
        np.testing.assert_allclose(hist, hist_o, rtol=1e-9)
        assert np.abs(un - u_o).max() < 1e-12


def test_gpu_mg_vs_reference_lexicographic(lib):
    """Reference smoother (lexicographic GS) vs the GPU's red-black: different iterates,
    same converged solution to the tolerance."""
    from cfd_julia_amd import mg

    n, levels = 32, 4
    f, ue, un, dx, dy = mg.mms(n, ipr=2)
    mg.mg_N(dx, dy, n, n, None, f, un, 2, 2, 2, 100000, 1e-10, n_level=levels)
    u_lex, it_lex, _ = co.mg_n(f, mg.mms(n, ipr=2)[2], dx, dy, levels, tol=1e-10,
                               smoother=co.gauss_seidel_lex)
    assert np.abs(un - u_lex).max() < 1e-9 * np.abs(u_lex).max()


# ---- 15_Poisson_Solver_Gauss_Seidel/gauss_seidel.jl (a Jacobi sweep) ---------------------
def test_gpu_jacobi_bit_exact_fixed_sweeps(lib):
    from cfd_julia_amd.gauss_seidel import gauss_seidel
    from oracle import misc_oracle as mo

    n = 64
    f, ue, un, dx, dy = co.mg_mms(n, ipr=2)
    u = np.asfortranarray(un.copy())
    it, _ = gauss_seidel(dx, dy, n, n, None, f, u, 60, 0.0, freq=1000)  # tol 0: 300 sweeps
    u_ref, it_ref, _ = mo.gauss_seidel(f, un.copy(), dx, dy, 60, 0.0, freq=1000)
    assert it == it_ref == 300
    assert np.array_equal(u, u_ref)


def test_gpu_jacobi_converges_mms(lib):
    from cfd_julia_amd.gauss_seidel import gauss_seidel

    n = 32
    f, ue, un, dx, dy = co.mg_mms(n, ipr=1)
    u = np.asfortranarray(un.copy())
    it, rms = gauss_seidel(dx, dy, n, n, None, f, u, 20000, 1e-9, freq=100)
    assert it < 5 * 20000 and np.abs(u - ue).max() < 1e-7


# ---- lid_driven_cavity.jl:161-216 main + its text output --------------------------------
def test_gpu_cavity_main_writes_reference_files(lib, tmp_path):
    from cfd_julia_amd import cavity
    from cfd_julia_amd.fieldio import read_field

    n = 32
    wn, sn, rms = cavity.main(nx=n, ny=n, dt=0.001, tf=0.02, re=100.0, outdir=str(tmp_path))
    res = np.loadtxt(tmp_path / "res_plot.txt", ndmin=2)
    assert res.shape == (20, 2) and np.array_equal(res[:, 0], np.arange(1, 21))
    assert np.array_equal(res[:, 1], rms)
    assert np.array_equal(read_field(tmp_path / "field_final.txt", n, n, 2), wn)
    assert np.array_equal(read_field(tmp_path / "field_final.txt", n, n, 3), sn)
    xy = np.loadtxt(tmp_path / "field_final.txt")[:, :2]
    assert xy[1, 0] == 1.0 / n and xy[n + 1, 1] == 1.0 / n


@pytest.mark.parametrize("n,levels,sweeps", [(512, 9, (2, 2, 2)), (512, 9, (2, 1, 3)),
                                             (256, 4, (1, 2, 1)), (1024, 10, (3, 2, 2)),
                                             (384, 3, (2, 2, 2))])
def test_gpu_mg_fused_kernels_are_bit_identical(lib, monkeypatch, n, levels, sweeps):
    """The V-cycle's fused kernels (several red-black sweeps per pass over a level in LDS
    tiles, with the descent's residual, norm partial sums and restriction taken from the
    same tile; all coarse levels in one workgroup; cycles replayed from a HIP graph) reorder
    no arithmetic of the iteration: iterates, final residual and iteration count equal the
    one-launch-per-half-sweep, level-by-level, eagerly launched V-cycle bit for bit.  The
    residual history is bit-equal too while the norm's partial sums come from the separate
    residual kernel; the fused descent sums the same squares per tile instead of per 64x4
    block, so there the history agrees to round-off of the sum."""
    from cfd_julia_amd import mg

    v1, v2, v3 = sweeps
    keys = ("CFDJ_MG_FUSED_SMOOTH", "CFDJ_MG_FUSED_DESC", "CFDJ_MG_COARSE", "CFDJ_MG_GRAPH",
            "CFDJ_MG_WIDE_TILES")
    out = {}
    for name, env in (("fused", {}),
                      ("narrow", {"CFDJ_MG_WIDE_TILES": "0"}),
                      ("nodesc", {"CFDJ_MG_FUSED_DESC": "0"}),
                      ("plain", {"CFDJ_MG_FUSED_SMOOTH": "0", "CFDJ_MG_COARSE": "0",
                                 "CFDJ_MG_GRAPH": "0"})):
        for k in keys:
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        f, ue, un, dx, dy = mg.mms(n, ipr=2)
        r = np.zeros((n + 1, n + 1), order="F")
        it, hist = mg.mg_N(dx, dy, n, n, r, f, un, v1, v2, v3, 100000, 1e-9, n_level=levels)
        out[name] = (it, hist, un, r)
    assert out["plain"][0] > 2
    for name in ("fused", "narrow", "nodesc"):
        assert out[name][0] == out["plain"][0], name
        assert np.array_equal(out[name][2], out["plain"][2]), name
        assert np.array_equal(out[name][3], out["plain"][3]), name
    assert np.array_equal(out["nodesc"][1], out["plain"][1])
    np.testing.assert_allclose(out["fused"][1], out["plain"][1], rtol=1e-13)
    np.testing.assert_allclose(out["narrow"][1], out["plain"][1], rtol=1e-13)


@pytest.mark.parametrize("i", range(5))
def test_gpu_fft_d_matches_order_jl(lib, i):
    """14_Poisson_Solver_FST/fft_d.jl:47-75 on the GPU DST-I (cfd_julia_amd.fft_d over
    cfdj_fps_sine) at N = 32 ... 512 against the reference-held L2 errors of order.jl:11.
    Those are the errors of 12/fft_p.jl; they pin fft_d.jl as well because the manufactured
    right-hand side is odd about every wall of the unit box: the zero-mean periodic 5-point
    solution is then odd, vanishes on the walls and solves fft_d.jl's Dirichlet system too
    -- one discrete field, one norm (compute_l2norm_bnds).  Tolerance 1e-9 relative up to
    N = 128; at 256 and 512 the rounding of the two scripts' own symbols (cancellation from
    O(nx^2) to 8 pi^2) bounds the agreement at 1e-8 / 1.6e-7 (vo.fft_d_order_tolerance; the
    CPU oracle differs from order.jl:11 by 1.8e-9 / 2.9e-8 there)."""
    from cfd_julia_amd import fft_d
    from oracle import vm_oracle as vo

    n = vo.ORDER_JL_GRID[i]
    l2, linf = fft_d.main(grids=(n,))[n]
    ref = vo.ORDER_JL_FFT_FDM[i]
    assert abs(l2 - ref) / ref < vo.fft_d_order_tolerance(n, ref), (n, l2, ref)
    assert linf < 4 * ref  # two modes: the maximum norm stays within a few L2 norms


def test_gpu_fft_d_default_run_matches_oracle(lib):
    """fft_d.jl's shipped run (nx = ny = 128): the interior solution against the oracle's
    restatement (division by the symbol, fft_d.jl:15-20), 1e-12 of max|u|."""
    from cfd_julia_amd import fft_d

    f, ue, dx, dy = fft_d.mms(128)
    u = fft_d.ps_fst(128, 128, dx, dy, f)
    ref = co.ps_fst(f, dx, dy)
    assert u.shape == (127, 127)
    assert np.abs(u - ref).max() < 1e-12 * np.abs(ref).max()


def test_gpu_cavity_rhs_call_leaves_the_state_alone(lib):
    """cfdj_cavity_rhs (lid_driven_cavity.jl:124-159 as a function of the caller's w, s) between
    an upload and a step: the step continues from the uploaded fields -- the psi the caller
    hands to rhs, here with non-zero wall values, must not leak into either of the handle's
    two psi buffers."""
    from cfd_julia_amd.cavity import Cavity

    n, nt = 64, 2
    dx, dy, _, _ = co.cavity_grid(n, n)
    dt = 1e-3
    rng = np.random.default_rng(18)
    w0 = np.asfortranarray(np.pad(smooth_field(n - 1, n - 1, 3, 71), ((1, 1), (1, 1))))
    s0 = np.asfortranarray(np.pad(1e-2 * smooth_field(n - 1, n - 1, 3, 72), ((1, 1), (1, 1))))
    wx = np.asfortranarray(rng.standard_normal((n + 1, n + 1)))
    sx = np.asfortranarray(rng.standard_normal((n + 1, n + 1)))  # walls != 0
    with Cavity(n, n, dx, dy, 100.0) as h:
        h.upload(w0, s0)
        r = h.rhs(wx, sx)
        rms = h.step(dt, nt)
        wn, sn = h.download()
    assert np.array_equal(r, co.cavity_rhs(wx, sx, dx, dy, 100.0))
    w_ref, s_ref, rms_ref = co.cavity_numerical(n, n, nt, dt, 100.0, wn=w0, sn=s0)
    assert np.abs(wn - w_ref).max() < 1e-10 * max(1.0, np.abs(w_ref).max())
    assert np.abs(sn - s_ref).max() < 1e-12
    assert np.allclose(rms, rms_ref, rtol=1e-8, atol=1e-16)


@pytest.mark.parametrize("half", ["0", "1"])
@pytest.mark.parametrize("n", [512, 2048, 4096])
def test_gpu_fps_sine_both_transform_routes(lib, monkeypatch, n, half):
    """lid_driven_cavity.jl:11-21 by both routes to FFTW's RODFT00: the odd extension of a row
    pair (a complex FFT of 2n points; CFDJ_DST_HALF=0) and the half-length transform (n points,
    the odd coefficients as a running sum; CFDJ_DST_HALF=1).  The default picks per pass and
    size; each alone must meet the oracle (scipy's DST-I) to 1e-12 of max|psi|."""
    from cfd_julia_amd.cavity import fps_sine

    monkeypatch.setenv("CFDJ_DST_HALF", half)
    dx, dy, _, _ = co.cavity_grid(n, n)
    f = np.zeros((n + 1, n + 1), order="F")
    rng = np.random.default_rng(n)
    f[1:n, 1:n] = smooth_field(n - 1, n - 1, 4, 65) + 0.01 * rng.standard_normal((n - 1, n - 1))
    s = fps_sine(n, n, dx, dy, f)
    ref = co.fps_sine(f, dx, dy)
    assert np.all(s[0, :] == 0) and np.all(s[:, 0] == 0) and np.all(s[n, :] == 0)
    assert np.abs(s - ref).max() <= 1e-12 * np.abs(ref).max()


def test_gpu_cavity_steps_half_length_transform(lib, monkeypatch):
    """Cavity steps (512^2 x 3, the RMS partial sums of the inverse row pass included) on the
    half-length DST kernels alone against the oracle, as test_gpu_cavity_steps_vs_oracle does
    for the default mix."""
    from cfd_julia_amd import cavity

    monkeypatch.setenv("CFDJ_DST_HALF", "1")
    n, nt = 512, 3
    dt = 0.001 * (64 / n) ** 2
    dx, dy, _, _ = co.cavity_grid(n, n)
    wn = np.zeros((n + 1, n + 1), order="F")
    sn = np.zeros((n + 1, n + 1), order="F")
    rms = np.zeros(nt)
    cavity.numerical(n, n, nt, dx, dy, dt, 100.0, wn, sn, rms)
    w_ref, s_ref, rms_ref = co.cavity_numerical(n, n, nt, dt, 100.0)
    assert np.abs(wn - w_ref).max() < 1e-10 * max(1.0, np.abs(w_ref).max())
    assert np.abs(sn - s_ref).max() < 1e-12
    assert np.allclose(rms, rms_ref, rtol=1e-8, atol=1e-16)
