"""GPU parity at the sizes BASELINE.json's configs name (the smaller cases live in the other
test_gpu_* files): C3 4096^2 vortex merger for 20 RK3 steps, C4 2048^2 lid-driven cavity with
the DST-I and with the V-cycle multigrid Poisson solve, C5 8192^2 vortex merger as 8 y-slabs
(virtual ranks: the slab code of the 8-GPU run on one GPU) and through the RCCL slab code with
a one-rank communicator.  Everything goes through the C ABI; the oracle is the checker.

Tolerances: vorticity L-inf < 1e-10 (the north-star criterion) for the vortex merger and the
DST cavity; the multigrid cavity is compared at its own solver tolerance (the reference's
cavity uses the DST, lid_driven_cavity.jl:84; multigrid is BASELINE config 4's variant)."""
import numpy as np
import pytest

from oracle import cavity_oracle as co
from oracle import vm_oracle as vo

pytestmark = pytest.mark.gpu

_cache = {}


@pytest.fixture(scope="module")
def cfdj():
    import cfd_julia_amd
    from cfd_julia_amd import _lib

    assert _lib.require_gpu() >= 1
    return cfd_julia_amd


def _vm_reference(n, steps, dt):
    key = (n, steps, dt)
    if key not in _cache:
        dx, dy, x, y = vo.vm_grid(n, n)
        w0 = vo.vm_ic(n, n, x, y)
        _cache.clear()  # one 8192^2 reference at a time (0.5 GB each)
        _cache[key] = (dx, dy, w0, vo.numerical(w0, steps, dt, dx, dy, 1000.0))
    return _cache[key]


# ---- C3: vm.jl at 4096^2, 20 steps ---------------------------------------------------------
def test_gpu_c3_4096_20_steps_vs_oracle(cfdj):
    n, steps, dt = 4096, 20, 5e-4
    dx, dy, w0, ref = _vm_reference(n, steps, dt)
    with cfdj.VortexMerger(n, n, dx, dy, 1000.0) as h:
        h.upload_interior(w0)
        h.step(dt, steps)
        w = h.download_interior()
    err = np.abs(w - ref).max()
    print(f"C3 4096^2 {steps} steps: Linf = {err:.3e}", flush=True)
    assert err < 1e-10


# ---- C5: vm.jl at 8192^2 as 8 y-slabs --------------------------------------------------------
C5 = (8192, 2, 1e-4)


def test_gpu_c5_8192_eight_virtual_slabs_vs_oracle(cfdj):
    n, steps, dt = C5
    dx, dy, w0, ref = _vm_reference(n, steps, dt)
    with cfdj.VortexMerger(n, n, dx, dy, 1000.0, kind="virtual", nranks=8) as h:
        assert h.poisson() == "schur"  # 1024 rows per rank: the substructured y-solve
        h.upload_interior(w0)
        h.step(dt, steps)
        w = h.download_interior()
    err = np.abs(w - ref).max()
    print(f"C5 8192^2 P=8 virtual, {steps} steps: Linf = {err:.3e}", flush=True)
    assert err < 1e-10


def test_gpu_c5_8192_rccl_one_rank_slab_vs_oracle(cfdj, monkeypatch):
    n, steps, dt = C5
    dx, dy, w0, ref = _vm_reference(n, steps, dt)
    monkeypatch.setenv("CFDJ_FORCE_SLAB", "1")
    uid = cfdj.VortexMerger.unique_id()
    with cfdj.VortexMerger(n, n, dx, dy, 1000.0, device=0, kind="dist", nranks=1, rank=0,
                           nccl_id=uid) as h:
        assert h.slab() == (0, n)
        path = h.poisson()
        h.upload_interior(w0)
        h.step(dt, steps)
        w = h.download_interior()
    err = np.abs(w - ref).max()
    print(f"C5 8192^2 RCCL one-rank slab ({path}), {steps} steps: Linf = {err:.3e}", flush=True)
    assert err < 1e-10


def test_gpu_c5_8192_single_gpu_vs_oracle(cfdj):
    n, steps, dt = C5
    dx, dy, w0, ref = _vm_reference(n, steps, dt)
    with cfdj.VortexMerger(n, n, dx, dy, 1000.0) as h:
        h.upload_interior(w0)
        h.step(dt, steps)
        w = h.download_interior()
    assert np.abs(w - ref).max() < 1e-10


# ---- C4: lid-driven cavity at 2048^2 -----------------------------------------------------------
C4_N, C4_NT, C4_DT = 2048, 3, 5e-6


def _cavity_reference():
    if "c4" not in _cache:
        _cache["c4"] = co.cavity_numerical(C4_N, C4_N, C4_NT, C4_DT, 100.0)
    return _cache["c4"]


def test_gpu_c4_fps_sine_2048_vs_oracle(cfdj):
    from cfd_julia_amd.cavity import fps_sine
    from tests.golden.make_golden import smooth_field

    n = C4_N
    dx, dy, _, _ = co.cavity_grid(n, n)
    f = np.zeros((n + 1, n + 1), order="F")
    f[1:n, 1:n] = smooth_field(n - 1, n - 1, 4, 63)
    s = fps_sine(n, n, dx, dy, f)
    ref = co.fps_sine(f, dx, dy)
    assert np.all(s[0, :] == 0) and np.all(s[:, 0] == 0) and np.all(s[n, :] == 0)
    assert np.abs(s - ref).max() <= 1e-12 * np.abs(ref).max()


def test_gpu_c4_cavity_2048_dst_vs_oracle(cfdj):
    from cfd_julia_amd import cavity

    n, nt, dt = C4_N, C4_NT, C4_DT
    dx, dy, _, _ = co.cavity_grid(n, n)
    wn = np.zeros((n + 1, n + 1), order="F")
    sn = np.zeros((n + 1, n + 1), order="F")
    rms = np.zeros(nt)
    cavity.numerical(n, n, nt, dx, dy, dt, 100.0, wn, sn, rms)
    w_ref, s_ref, rms_ref = _cavity_reference()
    ew = np.abs(wn - w_ref).max() / max(1.0, np.abs(w_ref).max())
    es = np.abs(sn - s_ref).max()
    print(f"C4 cavity 2048^2 DST: rel Linf(w) = {ew:.3e}, Linf(psi) = {es:.3e}", flush=True)
    assert ew < 1e-10
    assert es < 1e-12
    assert np.allclose(rms, rms_ref, rtol=1e-8, atol=1e-16)


def test_gpu_c4_cavity_2048_multigrid_vs_oracle(cfdj):
    """BASELINE config 4: the cavity step with the V-cycle multigrid Poisson (mg_N.jl) in
    place of fps_sine, against the DST oracle at the multigrid tolerance."""
    from cfd_julia_amd.cavity import Cavity

    n, nt, dt = C4_N, C4_NT, C4_DT
    dx, dy, _, _ = co.cavity_grid(n, n)
    with Cavity(n, n, dx, dy, 100.0, poisson="mg", tol=1e-11) as h:
        rms = h.step(dt, nt)
        wn, sn = h.download()
        its = h.mg_iterations()
    w_ref, s_ref, rms_ref = _cavity_reference()
    ew = np.abs(wn - w_ref).max() / np.abs(w_ref).max()
    es = np.abs(sn - s_ref).max() / np.abs(s_ref).max()
    print(f"C4 cavity 2048^2 MG: V-cycles = {its}, rel Linf(w) = {ew:.3e}, "
          f"rel Linf(psi) = {es:.3e}", flush=True)
    assert its >= 3 * nt
    assert es < 1e-8
    assert ew < 1e-6
    assert np.allclose(rms, rms_ref, rtol=1e-5)


def test_gpu_c4_mg_mms_2048(cfdj):
    from cfd_julia_amd import mg

    n = C4_N
    f, ue, un, dx, dy = mg.mms(n)
    it, hist = mg.mg_N(dx, dy, n, n, None, f, un, 2, 2, 2, 100000, 1e-9, n_level=11)
    print(f"C4 MG MMS 2048^2: {it} V-cycles, rms/rms0 = {hist[-1] / hist[0]:.3e}", flush=True)
    assert hist[-1] / hist[0] <= 1e-9 and it < 50
    assert np.abs(un - ue).max() < 1e-6


# ---- mg.jl: the two-level cycle (coarse grid v3 sweeps, post-smoothing v2 sweeps) -----------
def test_gpu_mg_two_level_vs_oracle(cfdj, tmp_path):
    import io

    from cfd_julia_amd import mg

    n = 64
    f, ue, un, dx, dy = mg.mms(n, ipr=2)
    u0 = un.copy(order="F")
    r = np.zeros((n + 1, n + 1), order="F")
    out = io.StringIO()
    it, hist = mg.mg(dx, dy, n, n, r, f, un, 2, 1, 3, 100000, 1e-8, out=out, freq=10,
                     outdir=str(tmp_path))
    u_o, it_o, hist_o, r_o = co.mg_2level(f, u0, dx, dy, v1=2, v2=1, v3=3, tol=1e-8)
    assert it == it_o
    np.testing.assert_allclose(hist, hist_o, rtol=1e-9)
    assert np.abs(un - u_o).max() < 1e-12
    assert np.abs(r - r_o).max() <= 1e-9 * np.abs(r_o).max() + 1e-12
    # un-exchanged sweep roles (mg_N with n_level = 2 and the same v2, v3) iterate differently
    uN = u0.copy(order="F")
    itN, histN = mg.mg_N(dx, dy, n, n, None, f, uN, 2, 1, 3, 100000, 1e-8, n_level=2)
    assert not np.allclose(histN[:min(len(histN), len(hist))], hist[:min(len(histN), len(hist))],
                           rtol=1e-6)
    lines = out.getvalue().splitlines()
    assert lines[0].startswith("L-2 Norm=") and lines[1].startswith("Maximum Norm=")
    assert lines[2] == f"Iterations={it}"
    assert float(lines[1].split("=")[1]) == np.abs(r).max()
    res = np.loadtxt(tmp_path / "residual.txt", ndmin=2)
    assert res.shape == (it // 10, 3) and res[0, 0] == 10 and res[0, 1] == hist[10]


def test_gpu_mg_n_outputs(cfdj, tmp_path):
    """mg_N.jl:8,59,64-67,109-111: r holds the final fine residual, the three output lines,
    and mg_residual.txt with one "it rms rms/rms0" line per iteration (freq = 1)."""
    import io

    from cfd_julia_amd import mg

    n = 64
    f, ue, un, dx, dy = mg.mms(n)
    r = np.zeros((n + 1, n + 1), order="F")
    out = io.StringIO()
    it, hist = mg.mg_N(dx, dy, n, n, r, f, un, 2, 2, 2, 100000, 1e-9, out=out, n_level=5,
                       outdir=str(tmp_path))
    ref_r = co.compute_residual(f, un, dx, dy)
    # r is the residual at the last convergence check == residual of the returned u_n
    assert np.abs(r - ref_r).max() <= 1e-9 * max(np.abs(ref_r).max(), 1e-300) + 1e-12
    assert np.all(r[0, :] == 0) and np.all(r[:, 0] == 0)
    assert abs(co.compute_l2norm(r) - hist[-1]) <= 1e-12 * hist[0]
    lines = out.getvalue().splitlines()
    assert [l.split("=")[0] for l in lines] == ["L-2 Norm", "Maximum Norm", "Iterations"]
    res = np.loadtxt(tmp_path / "mg_residual.txt", ndmin=2)
    assert res.shape == (it, 3) and np.array_equal(res[:, 0], np.arange(1, it + 1))
    assert np.array_equal(res[:, 1], hist[1:])
