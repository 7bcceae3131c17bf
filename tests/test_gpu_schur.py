"""GPU parity of the substructured y-slab Poisson path (schur.hip, CFDJ_POISSON_SCHUR):
row FFTs + per-x-mode periodic y-tridiagonal split at one separator row per slab (interiors
solved directly in 32-row Thomas chunks + an interface system on the GPU, by DST-I in the
CPU restatement; P x P circulant separator system), run as P virtual ranks on one GPU and
as a one-rank RCCL communicator (tests/test_gpu_rccl.py).

Tolerances.  The reference (vm_oracle.fps, Common.jl:97-125) divides by D = (aa + bb cos kx)
+ cc cos ky evaluated in double; with |cc| = 2/dy^2 ~ n^2 that rounding perturbs its low
modes by ~eps * cc / |D|.  The decomposition inverts the same operator through sums of the
same magnitude (separator system, interior pivots / DST eigenvalues), so two correct implementations agree to
~eps * n^2 relative, not to a fixed 1e-12: psi within tol = 2e-12 * (n/1024)^2 * max|psi|
of the CPU restatement (oracle/schur_oracle.py) and 2 tol of the reference (the CPU
restatement itself is 1.2e-12 / 6e-12 from the reference at 1024^2 / 4096^2).  The north-star criterion -- vorticity
after K RK3 steps within 1e-10 (L-inf) of the reference -- is tested directly.
"""
import numpy as np
import pytest

from oracle import schur_oracle as so
from oracle import vm_oracle as vo

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cfdj():
    import cfd_julia_amd
    from cfd_julia_amd import _lib

    assert _lib.require_gpu() >= 1
    return cfd_julia_amd


@pytest.mark.parametrize("n,P", [(1024, 1), (1024, 2), (2048, 1), (2048, 2), (2048, 4),
                                 (4096, 1), (4096, 2), (4096, 4), (4096, 8)])
def test_gpu_schur_psi_vs_oracles(cfdj, n, P):
    dx, dy, x, y = vo.vm_grid(n, n)
    w = vo.vm_ic(n, n, x, y) + 0.01 * np.random.default_rng(n + P).standard_normal((n, n))
    ref = vo.fps(-w, dx, dy)
    dec = so.schur_fps(-w, dx, dy, P)
    with cfdj.VortexMerger(n, n, dx, dy, 1000.0, kind="virtual", nranks=P) as h:
        assert h.poisson() == "schur"
        _, s = h.rhs(vo.to_ghosted(w))
    s = vo.from_ghosted(s)
    scale = np.abs(ref).max()
    tol = 2e-12 * (n / 1024) ** 2 * scale
    assert np.abs(s - dec).max() <= tol, np.abs(s - dec).max() / scale
    assert np.abs(s - ref).max() <= 2 * tol, np.abs(s - ref).max() / scale


@pytest.mark.parametrize("n,P,steps", [(1024, 2, 4), (2048, 2, 3), (2048, 4, 3), (4096, 8, 2)])
def test_gpu_schur_vm_steps_vs_reference(cfdj, n, P, steps):
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.vm_ic(n, n, x, y)
    dt = 5e-4 * (4096 / n) ** 2
    ref = vo.numerical(w0, steps, dt, dx, dy, 1000.0)
    with cfdj.VortexMerger(n, n, dx, dy, 1000.0, kind="virtual", nranks=P) as h:
        assert h.poisson() == "schur"
        h.upload_interior(w0)
        h.step(dt, steps)
        w = h.download_interior()
    assert np.abs(w - ref).max() < 1e-10


def test_gpu_schur_matches_transpose_path(cfdj):
    n, P = 2048, 4
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.vm_ic(n, n, x, y)
    out = {}
    for path in ("schur", "fused"):
        with cfdj.VortexMerger(n, n, dx, dy, 1000.0, kind="virtual", nranks=P) as h:
            h.set_poisson(path)
            h.upload_interior(w0)
            h.step(2e-3, 5)
            out[path] = h.download_interior()
    assert np.abs(out["schur"] - out["fused"]).max() < 1e-11


def test_gpu_schur_16384_long_rows_vs_library_path(cfdj):
    """Rows of 16384 reals are beyond the small-item row kernels: the persistent row kernels
    run, and the packed column travels through strided copies.  psi of one right-hand side
    against the library transposes' path on the same 8 slabs (no oracle at this size: the
    NumPy solve would need minutes)."""
    n, P = 16384, 8
    dx, dy, x, y = vo.vm_grid(n, n)
    w = vo.to_ghosted(vo.vm_ic(n, n, x, y))
    out = {}
    for path in ("schur", "rocfft"):
        with cfdj.VortexMerger(n, n, dx, dy, 1000.0, kind="virtual", nranks=P) as h:
            h.set_poisson(path)
            assert h.poisson() == path
            _, s = h.rhs(w)
            out[path] = vo.from_ghosted(s)
            del s
    scale = np.abs(out["rocfft"]).max()
    err = np.abs(out["schur"] - out["rocfft"]).max()
    assert err <= 2e-12 * (n / 1024) ** 2 * scale, err / scale


def test_gpu_schur_path_selection(cfdj):
    dx, dy, _, _ = vo.vm_grid(2048, 2048)
    with cfdj.VortexMerger(2048, 2048, dx, dy, 1000.0) as h:  # single GPU: no slabs
        assert h.poisson() == "fused"
        with pytest.raises(cfdj.ArgumentError):
            h.set_poisson("schur")
    with cfdj.VortexMerger(2048, 1024, dx, dy, 1000.0, kind="virtual", nranks=2) as h:
        assert h.poisson() == "fused"  # ny < nx: the aliased ky symbol is not a y-stencil
        with pytest.raises(cfdj.ArgumentError):
            h.set_poisson("schur")
    with cfdj.VortexMerger(2048, 2048, dx, dy, 1000.0, kind="virtual", nranks=2) as h:
        assert h.poisson() == "schur"
        h.set_poisson("fused")
        assert h.poisson() == "fused"
        h.set_poisson("auto")
        assert h.poisson() == "schur"


@pytest.mark.parametrize("n,P,path", [(2048, 4, "schur"), (4096, 8, "schur"), (4096, 2, "schur"),
                                      (1024, 2, "fused"), (256, 2, "rocfft")])
def test_gpu_virtual_slabs_side_stream_schedule_is_bit_identical(cfdj, monkeypatch, n, P, path):
    """The multi-GPU step's event schedule on one GPU: virtual slabs created with
    CFDJ_VIRTUAL_OVERLAP=1 run what the RCCL ranks run -- halo exchanges on the side stream
    (omega during the Poisson passes, psi during the interior rows of the stage kernel) and the
    substructured solve's two gathers on the side stream behind their four events -- with
    device copies in place of the collectives.  What a slab contributes to a gather goes to a
    staging buffer and reaches the shared arrays only through the side stream's copy, so a
    consumer that did not wait for its event would read the previous solve's values.  Several
    steps over several calls must equal the single-stream order bit for bit, and the oracle
    to the north-star tolerance.  (The substructured path exchanges no halo rows by default:
    the switches below put it back on the exchanging schedule this test is about.)"""
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.vm_ic(n, n, x, y)
    dt = min(0.01, 5e-4 * (4096 / n) ** 2)
    monkeypatch.setenv("CFDJ_SLAB_PSI_HALO", "exchange")
    monkeypatch.setenv("CFDJ_SLAB_W_HALO", "exchange")
    out = {}
    for ov in ("0", "1"):
        monkeypatch.setenv("CFDJ_VIRTUAL_OVERLAP", ov)
        with cfdj.VortexMerger(n, n, dx, dy, 1000.0, kind="virtual", nranks=P) as h:
            h.set_poisson(path)
            assert h.poisson() == path
            h.upload_interior(w0)
            h.step(dt, 2)
            h.step(dt, 1)
            out[ov] = h.download_interior()
    assert np.array_equal(out["0"], out["1"])
    if n <= 2048:
        ref = vo.numerical(w0, 3, dt, dx, dy, 1000.0)
        assert np.abs(out["1"] - ref).max() < 1e-10


@pytest.mark.parametrize("n,P", [(2048, 4), (4096, 8), (4096, 2), (1024, 2)])
def test_gpu_virtual_slabs_without_halo_exchange(cfdj, monkeypatch, n, P):
    """The substructured y-slab step needs no halo exchange of its own: psi's two halo rows come
    out of the slab's solve (the next slab's separator value; the previous slab's last row from
    the operator's equation at this slab's separator row), omega's ride in the solve's
    all-gather.  Against the exchanging schedules -- psi computed and omega exchanged
    (CFDJ_SLAB_W_HALO=exchange), both exchanged (+ CFDJ_SLAB_PSI_HALO=exchange) -- after 3
    steps: equal to round-off (1e-12 of max|w|; the computed psi rows differ from the
    neighbour's own in the last bits), and the oracle to the north-star tolerance."""
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.vm_ic(n, n, x, y)
    dt = min(0.01, 5e-4 * (4096 / n) ** 2)
    out = {}
    for name, env in (("none", {}), ("omega", {"CFDJ_SLAB_W_HALO": "exchange"}),
                      ("both", {"CFDJ_SLAB_W_HALO": "exchange", "CFDJ_SLAB_PSI_HALO": "exchange"})):
        for k in ("CFDJ_SLAB_W_HALO", "CFDJ_SLAB_PSI_HALO"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        with cfdj.VortexMerger(n, n, dx, dy, 1000.0, kind="virtual", nranks=P) as h:
            assert h.poisson() == "schur"
            h.upload_interior(w0)
            h.step(dt, 2)
            h.step(dt, 1)
            out[name] = h.download_interior()
    scale = np.abs(out["both"]).max()
    assert np.array_equal(out["none"], out["omega"])  # the same rows, by another route
    assert np.abs(out["none"] - out["both"]).max() <= 1e-12 * scale
    if n <= 2048:
        ref = vo.numerical(w0, 3, dt, dx, dy, 1000.0)
        assert np.abs(out["none"] - ref).max() < 1e-10


@pytest.mark.parametrize("n,P", [(1024, 2), (2048, 4), (4096, 8), (4096, 2)])
def test_gpu_virtual_slabs_tall_tile_stage_kernel_matches_marching(cfdj, monkeypatch, n, P):
    """Slabs of the substructured path whose column sums come in 16-row blocks (the default
    from 8 M cells per slab on; here by CFDJ_SLAB_ROWS_PER_WAVE=16 at every size) run the
    tall-tile stage kernel: 128 x 16-row workgroups in row-major order, a block's column sums
    added up in LDS in the marching kernel's order.  Against the marching kernel with the same
    blocks (set_rows_per_wave(16) selects it) the field after 3 steps -- 9 stage launches
    whose column sums feed the next Poisson solve -- must be the same bits."""
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.vm_ic(n, n, x, y)
    dt = min(0.01, 5e-4 * (4096 / n) ** 2)
    monkeypatch.setenv("CFDJ_SLAB_ROWS_PER_WAVE", "16")
    out = {}
    for name in ("tall", "marching"):
        with cfdj.VortexMerger(n, n, dx, dy, 1000.0, kind="virtual", nranks=P) as h:
            assert h.poisson() == "schur"
            if name == "marching":
                h.set_rows_per_wave(16)
            h.upload_interior(w0)
            h.step(dt, 2)
            h.step(dt, 1)
            out[name] = h.download_interior()
    assert np.array_equal(out["tall"], out["marching"])
    if n <= 2048:
        ref = vo.numerical(w0, 3, dt, dx, dy, 1000.0)
        assert np.abs(out["tall"] - ref).max() < 1e-10


@pytest.mark.parametrize("n,P", [(1024, 2), (2048, 4), (4096, 8), (4096, 1)])
def test_gpu_schur_column_sums_transformed_after_the_gather(cfdj, monkeypatch, n, P):
    """The constant-mode correction needs the spectrum of the field's column sum over ALL rows.
    Default: every slab's untransformed sums ride in the all-gather (added up from the stage
    kernel's partial rows by extra workgroups of the forward row pass) and one more workgroup
    of the packed column's solve adds the ranks' rows and transforms the total.
    CFDJ_SLAB_LATE_CS=0: a summing launch and a transform per slab before the gather, the
    solve adding the spectra.  The correction is ~1e-8 of psi, so psi must agree far below the
    oracle tolerance (1e-14 of max|psi|), and both routes stay within it."""
    dx, dy, x, y = vo.vm_grid(n, n)
    w = vo.vm_ic(n, n, x, y) + 0.01 * np.random.default_rng(7 * n + P).standard_normal((n, n))
    ref = vo.fps(-w, dx, dy)
    out = {}
    for late in ("1", "0"):
        monkeypatch.setenv("CFDJ_SLAB_LATE_CS", late)
        with cfdj.VortexMerger(n, n, dx, dy, 1000.0, kind="virtual", nranks=P) as h:
            assert h.poisson() == "schur"
            _, s = h.rhs(vo.to_ghosted(w))
        out[late] = vo.from_ghosted(s)
    scale = np.abs(ref).max()
    assert np.abs(out["1"] - out["0"]).max() <= 1e-14 * scale
    tol = 4e-12 * (n / 1024) ** 2 * scale
    assert np.abs(out["1"] - ref).max() <= tol
    # a correction left out would be visible: the y-constant part of psi differs from the
    # circulant's by ~1e-8 relative


def test_gpu_schur_16384_steps_exchange_free_vs_exchanging_schedule(cfdj, monkeypatch):
    """16384^2 on 8 slabs (rows and columns of 16384: the longest the small-item row kernels
    and the split packed-column solve take): 2 steps of the default schedule -- one all-gather
    per stage, psi's halo rows out of the solve, column sums transformed after the gather --
    against the exchanging one with the per-slab column-sum transforms.  No oracle at this size;
    the two schedules share the interior solve but not the halo rows' route, the packed
    column's partner lookup or the correction's input, and must agree to round-off."""
    n, P = 16384, 8
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.vm_ic(n, n, x, y)
    dt = 5e-4 * (4096 / n) ** 2
    out = {}
    for name, env in (("default", {}), ("exchange", {"CFDJ_SLAB_W_HALO": "exchange",
                                                     "CFDJ_SLAB_PSI_HALO": "exchange",
                                                     "CFDJ_SLAB_LATE_CS": "0"})):
        for k in ("CFDJ_SLAB_W_HALO", "CFDJ_SLAB_PSI_HALO", "CFDJ_SLAB_LATE_CS"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        with cfdj.VortexMerger(n, n, dx, dy, 1000.0, kind="virtual", nranks=P) as h:
            assert h.poisson() == "schur"
            h.upload_interior(w0)
            h.step(dt, 2)
            out[name] = h.download_interior()
    scale = np.abs(out["exchange"]).max()
    assert np.isfinite(out["default"]).all()
    assert np.abs(out["default"] - out["exchange"]).max() <= 1e-12 * scale
    assert np.abs(out["default"] - w0).max() > 1e-6 * scale  # (the field moved)
