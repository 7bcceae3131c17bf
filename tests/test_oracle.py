"""CPU tests: pin the oracle to the reference's published numbers and known answers.

order.jl:10-11 hold the only numbers the reference publishes (FD-FFT and spectral Poisson
L2 errors of fft_p.jl / fft_s.jl at N = 32..512).  tgv.jl:82-90 gives the analytic
Taylor-Green decay; the vortex-merger figure (Python_Vectorized/field_fdm.png) shows a peak
vorticity of about 0.74 at 128^2, t = 20.
"""
import math

import numpy as np
import pytest

from oracle import vm_oracle as vo
from tests.golden.make_golden import smooth_field


@pytest.mark.parametrize("i", range(5))
def test_fft_p_matches_order_jl(i):
    n = vo.ORDER_JL_GRID[i]
    l2, _ = vo.fft_p_mms_error(n)
    ref = vo.ORDER_JL_FFT_FDM[i]
    assert abs(l2 - ref) / ref < 1e-10, (n, l2, ref)


@pytest.mark.parametrize("i", range(5))
def test_fft_s_spectral_is_roundoff(i):
    # order.jl:10: the spectral solver's errors are round-off (~1.3e-16..1.5e-16)
    n = vo.ORDER_JL_GRID[i]
    f, ue, dx, dy = vo.fft_p_mms(n)
    un = np.zeros_like(f)
    un[:n, :n] = vo.ps_spectral(np.ascontiguousarray(f[:n, :n]), dx, dy)
    un[n, :] = un[0, :]
    un[:, n] = un[:, 0]
    l2 = vo.compute_l2norm_bnds(un - ue)
    # same MMS as fft_p.jl; the spectral solver is exact, so the error is pure round-off
    # and only its magnitude is comparable (FFTW vs pocketfft rounding differs)
    ref = vo.ORDER_JL_FFT_SPECTRAL[i]
    assert 0.5 * ref < l2 < 2.0 * ref, (n, l2, ref)


@pytest.mark.parametrize("solver", ["ps_fst", "fps_sine"])
@pytest.mark.parametrize("i", range(5))
def test_fft_d_matches_order_jl(i, solver):
    """14_Poisson_Solver_FST/fft_d.jl:47-75 runs the manufactured solution of 12/fft_p.jl
    (order.jl:11 holds that script's L2 errors) through the DST-I solver.  The right-hand
    side is odd about every wall of the unit box, so the zero-mean periodic 5-point solution
    of fft_p.jl is odd too, vanishes on the walls, and therefore IS the solution of the
    Dirichlet 5-point system fft_d.jl solves: same discrete field, same norm
    (compute_l2norm_bnds over all (nx+1)(ny+1) nodes), hence order.jl:11's numbers pin the
    sine-transform solver (the cavity's fps_sine, lid_driven_cavity.jl:11-21, is the same
    solve with the reciprocal symbol tabulated).
    Tolerance: 1e-9 relative up to N = 128.  Beyond, the two scripts' own symbols limit the
    agreement: (2/dx^2)(cos(pi i/nx) - 1) here and aa + bb cos kx + cc cos ky there both
    cancel from O(nx^2) terms to 8 pi^2 for the dominant mode, each with its own rounding,
    so the mode's amplitude carries a relative error of about 4 nx^2 eps / (8 pi^2) and the
    (much smaller) L2 error norm that amount divided by itself: 1e-8 at 256, 1.6e-7 at 512
    (measured differences: 1.8e-9 and 2.9e-8)."""
    from oracle import cavity_oracle as co

    n = vo.ORDER_JL_GRID[i]
    l2, _ = co.fft_d_mms_error(n, solver)
    ref = vo.ORDER_JL_FFT_FDM[i]
    assert abs(l2 - ref) / ref < vo.fft_d_order_tolerance(n, ref), (n, solver, l2, ref)


def test_kx_table_reference_layout():
    kx = vo.kx_table(8, 1e-6)
    hx = 2 * math.pi / 8
    assert kx[0] == 1e-6
    assert list(kx[1:4]) == [hx * 1, hx * 2, hx * 3]
    assert list(kx[4:]) == [hx * -4, hx * -3, hx * -2, hx * -1]
    with pytest.raises(ValueError):
        vo.kx_table(7)


def test_fps_ny_gt_nx_is_bounds_error():
    with pytest.raises(IndexError):
        vo.fps_denominator(8, 16, 0.1, 0.1)


def test_fps_inverts_fd_laplacian():
    nx = ny = 64
    dx, dy, _, _ = vo.vm_grid(nx, ny)
    w = smooth_field(nx, ny, 5, 3)
    f = w - w.mean()
    s = vo.fps(f, dx, dy)
    lap = ((np.roll(s, -1, 0) - 2 * s + np.roll(s, 1, 0)) / dx ** 2
           + (np.roll(s, -1, 1) - 2 * s + np.roll(s, 1, 1)) / dy ** 2)
    assert np.abs(lap - f).max() < 1e-9


def test_arakawa_conservation_properties():
    # Arakawa's J conserves Σ J, Σ ω J (enstrophy) and Σ ψ J (energy) on a periodic grid
    nx = ny = 48
    dx, dy, _, _ = vo.vm_grid(nx, ny)
    w = smooth_field(nx, ny, 6, 4)
    s = smooth_field(nx, ny, 6, 5)
    J = vo.arakawa_rhs(w, s, dx, dy, 1e300)  # viscous term vanishes
    scale = np.abs(J).max()
    assert abs(J.sum()) < 1e-12 * scale * J.size
    assert abs((w * J).sum()) < 1e-12 * scale * np.abs(w).max() * J.size
    assert abs((s * J).sum()) < 1e-12 * scale * np.abs(s).max() * J.size


def test_ghost_layout_roundtrip():
    w = smooth_field(16, 16, 3, 7)
    g = vo.to_ghosted(w)
    assert g.flags.f_contiguous and g.shape == (18, 18)
    assert np.array_equal(vo.from_ghosted(g), w)
    assert np.array_equal(g[0, 1:-1], w[-1, :]) and np.array_equal(g[-1, 1:-1], w[0, :])
    assert np.array_equal(g[1:-1, 0], w[:, -1]) and np.array_equal(g[1:-1, -1], w[:, 0])


def test_golden_fixtures_reproduce(golden):
    for n in (32, 64):
        z = golden(f"fps_mms_{n}")
        np.testing.assert_allclose(vo.ps_fft(z["f"], float(z["dx"]), float(z["dy"])), z["s"],
                                   rtol=0, atol=1e-13)
    for name in ("vm_rhs_64x64", "vm_rhs_96x64"):
        z = golden(name)
        r, s = vo.vm_rhs(z["w"], float(z["dx"]), float(z["dy"]), float(z["re"]))
        np.testing.assert_allclose(r, z["r"], rtol=0, atol=1e-11)
        np.testing.assert_allclose(s, z["s"], rtol=0, atol=1e-13)
    z = golden("vm_64_10steps")
    w = vo.numerical(z["w0"], int(z["nt"]), float(z["dt"]), float(z["dx"]), float(z["dy"]),
                     float(z["re"]))
    np.testing.assert_allclose(w, z["w10"], rtol=0, atol=1e-13)


def test_tgv_known_answer(golden):
    # tgv.jl: RK3 + Arakawa + FD Poisson vs the analytic decay 8cos4x cos4y e^{-32t/re}
    l2, linf = vo.tgv_error(64, 10.0, 0.01, 1.0)
    z = golden("tgv_64")
    assert abs(l2 - float(z["l2"])) < 1e-14 and abs(linf - float(z["linf"])) < 1e-14
    # second-order FD in space: amplitude 8e^{-3.2} ~ 0.33, error ~2% of it at 64^2
    assert 5e-3 < l2 < 8e-3
    l2_32, _ = vo.tgv_error(32, 10.0, 0.01, 1.0)
    assert 3.0 < l2_32 / l2 < 5.0  # O(dx^2) convergence


@pytest.mark.slow
def test_vortex_merger_peak_matches_reference_figure():
    # Python_Vectorized/field_fdm.png: 128^2, re = 1000, dt = .01, t = 20 -> peak ω ≈ 0.74
    nx = ny = 128
    dx, dy, x, y = vo.vm_grid(nx, ny)
    w = vo.numerical(vo.vm_ic(nx, ny, x, y), 2000, 0.01, dx, dy, 1000.0, workers=1)
    assert 0.72 < w.max() < 0.76


def test_cavity_oracle_default_run_matches_literature_vortex():
    # lid_driven_cavity.jl:162-172 as shipped (64^2, dt = .001, 10000 steps, re = 100); the
    # reference holds no number for it, the literature does: Ghia, Ghia & Shin (1982), Re = 100,
    # primary vortex psi = -0.1034 at (0.6172, 0.7344)
    from oracle import cavity_oracle as co

    n = 64
    w, s, rms = co.cavity_numerical(n, n, 10000, 0.001, 100.0)
    i, j = np.unravel_index(np.abs(s).argmax(), s.shape)
    assert abs(s[i, j] + 0.1034) < 0.001
    assert abs(i / n - 0.6172) <= 1 / n and abs(j / n - 0.7344) <= 1 / n
    assert rms[-1] < 1e-6


def test_cpu_mirror_modules_import():
    # the host mirrors import without a GPU (compute raises CfdjError, never a CPU path)
    from cfd_julia_amd import common, fft_p, fft_s, vm  # noqa: F401

    assert callable(fft_s.ps_spectral) and callable(vm.numerical)


# ---- spectral-space solvers (hybrid.jl, pseudospectral_23/32_rule.jl) ------------------------
@pytest.mark.parametrize("kind", [0, 1, 2])
def test_spectral_oracle_tgv_scheme_decay(kind):
    """Taylor-Green has J(w, psi) = 0: each solver reproduces the CN-RK3 decay exactly."""
    from oracle import spectral_oracle as so

    n, re, dt, nt = 32, 10.0, 0.01, 20
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.exact_tgv(x, y, 0.0, re)[:n, :n].copy()
    w = so.numerical(w0, nt, dt, dx, dy, re, kind)
    assert np.abs(w - so.cn_decay(n, dx, dt, re, nt, 4, 4) * w0).max() < 1e-12


def test_spectral_oracle_jacobians_agree():
    """Band-limited input: the 2/3- and 3/2-rule products are exact (equal to round-off);
    the hybrid's FD Arakawa Jacobian converges to them at second order."""
    from oracle import spectral_oracle as so
    from tests.golden.make_golden import smooth_field

    errs = []
    for n in (32, 64):
        dx, dy, _, _ = vo.vm_grid(n, n)
        wf = so.to_spectral(smooth_field(n, n, 3, 5))
        k2 = so.wavespace(n, n, dx, dy)
        j = [so.to_physical(so.JACOBIANS[k](wf, k2, dx, dy)) for k in (0, 1, 2)]
        assert np.abs(j[1] - j[2]).max() < 1e-12 * np.abs(j[1]).max()
        errs.append(np.abs(j[0] - j[1]).max())
    assert 3.0 < errs[0] / errs[1] < 5.0  # O(dx^2)


# ---- mg.jl (two-level) vs mg_N.jl with n_level = 2 ------------------------------------------
def test_mg_two_level_is_mg_n_with_v2_v3_exchanged():
    """mg.jl:66,77 relax the coarse grid v3 times and the corrected fine grid v2 times;
    mg_N.jl:91,103 the other way round.  With v2 != v3 the two differ unless exchanged."""
    from oracle import cavity_oracle as co

    n = 32
    f, ue, un, dx, dy = co.mg_mms(n, ipr=2)
    u2, it2, h2, r2 = co.mg_2level(f, un, dx, dy, v1=2, v2=1, v3=3, tol=1e-8)
    uN, itN, hN = co.mg_n(f, un, dx, dy, 2, v1=2, v2=3, v3=1, tol=1e-8)
    assert it2 == itN and np.array_equal(u2, uN) and h2 == hN
    uX, itX, hX = co.mg_n(f, un, dx, dy, 2, v1=2, v2=1, v3=3, tol=1e-8)
    assert not np.array_equal(u2, uX)  # same arguments, un-exchanged: a different iteration
    assert np.array_equal(r2, co.compute_residual(f, u2, dx, dy)) or it2 > 0
    assert np.abs(u2 - ue).max() < 5e-3  # converged to the discrete solution (O(h^2) from ue)
