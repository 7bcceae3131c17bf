"""GPU parity of the spectral-space NS2D solvers (libcfdj.so `cfdj_spec_*`, spectral.hip)
against oracle/spectral_oracle.py -- the CPU restatement of
20_NS2D_Hybrid_Solver/hybrid.jl and the 2/3- and 3/2-rule pseudospectral scripts.

Tolerances: one Jacobian evaluation 1e-12 relative to max|jf| (FFT round-off: rocFFT vs
pocketfft); vorticity after K steps L-inf < 1e-10 (north-star bound, |w| ~ 1); the
Taylor-Green known answer (zero Jacobian, exact scheme decay) to 1e-12.
"""
import functools
import math

import numpy as np
import pytest

from oracle import spectral_oracle as so
from oracle import vm_oracle as vo
from tests.golden.make_golden import smooth_field

pytestmark = pytest.mark.gpu
KINDS = ["hybrid", "2/3", "3/2"]
KIND_ID = {"hybrid": so.HYBRID, "2/3": so.PS23, "3/2": so.PS32}


@pytest.fixture(scope="module")
def spec():
    from cfd_julia_amd import _lib, spectral

    assert _lib.require_gpu() >= 1
    return spectral


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("n", [64, 96, 256, 1024])
def test_gpu_spectral_jacobian_vs_oracle(spec, kind, n):
    dx, dy, _, _ = vo.vm_grid(n, n)
    wf = _noisy_spectrum(n)
    k2 = so.wavespace(n, n, dx, dy)
    ref = so.JACOBIANS[KIND_ID[kind]](wf, k2, dx, dy)
    with spec.SpectralNS2D(n, n, dx, dy, 1000.0, kind) as h:
        got = h.jacobian(wf)
    assert np.abs(got - ref).max() <= 1e-12 * np.abs(ref).max()


@functools.lru_cache(maxsize=1)
def _noisy_spectrum(n):
    """Spectrum of a smooth field plus white noise: content in every mode, Nyquist included.
    From 2048 on the smooth part is set mode by mode in spectral space (smooth_field's 169
    full-grid cos/sin passes take most of a minute at 4096^2)."""
    rng = np.random.default_rng(n)
    noise = 0.01 * rng.standard_normal((n, n))
    if n < 2048:
        return so.to_spectral(smooth_field(n, n, 6, n) + noise)
    wf = np.fft.fft2(noise)
    for kx in range(-6, 7):
        for ky in range(-6, 7):
            if (kx, ky) > (0, 0):  # one of each conjugate pair, its mirror set with it
                c = complex(*rng.standard_normal(2)) * n * n / (1.0 + kx * kx + ky * ky)
                wf[kx % n, ky % n] += c
                wf[-kx % n, -ky % n] += np.conj(c)
    return so.to_spectral(np.real(np.fft.ifft2(wf)))


@pytest.mark.parametrize("kind", ["hybrid", "2/3"])
@pytest.mark.parametrize("n", [2048, 4096])
def test_gpu_spectral_jacobian_vs_oracle_large(spec, kind, n):
    """The half-spectrum transforms (n = 2048 and the benchmarked 4096) against the oracle's
    full complex ones, on a field with content in every mode up to the Nyquist row and
    column: 1e-12 of max|jf| like the small grids."""
    dx, dy, _, _ = vo.vm_grid(n, n)
    wf = _noisy_spectrum(n)
    ref = so.JACOBIANS[KIND_ID[kind]](wf, so.wavespace(n, n, dx, dy), dx, dy)
    with spec.SpectralNS2D(n, n, dx, dy, 1000.0, kind) as h:
        got = h.jacobian(wf)
    assert np.abs(got - ref).max() <= 1e-12 * np.abs(ref).max()


@pytest.mark.parametrize("kind", ["hybrid", "2/3"])
def test_gpu_spectral_jacobian_4096_half_vs_full_spectrum(spec, monkeypatch, kind):
    """The benchmarked grid: the half-spectrum path against the full-spectrum complex
    transforms (CFDJ_SPEC_HALF=0, itself checked against the oracle on the smaller grids) on
    the same noisy field, 1e-12 of max|jf|."""
    n = 4096
    dx, dy, _, _ = vo.vm_grid(n, n)
    wf = _noisy_spectrum(n)
    out = {}
    for name, env in (("half", None), ("full", "0")):
        monkeypatch.delenv("CFDJ_SPEC_HALF", raising=False)
        if env is not None:
            monkeypatch.setenv("CFDJ_SPEC_HALF", env)
        with spec.SpectralNS2D(n, n, dx, dy, 1000.0, kind) as h:
            out[name] = h.jacobian(wf)
    assert np.abs(out["half"] - out["full"]).max() <= 1e-12 * np.abs(out["full"]).max()


@pytest.mark.parametrize("kind", ["hybrid", "2/3"])
def test_gpu_spectral_8192_half_vs_library(spec, monkeypatch, kind):
    """The largest grid of the half-spectrum path (8192^2: 4096-point half rows, 8192-point
    columns, the inverse row pass without its band limit) against the library's complex
    transforms: vortex-merger fields after 2 steps, 1e-12 of max|w|."""
    n = 8192
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.vm_ic(n, n, x, y)
    out = {}
    for name, env in (("half", None), ("rocfft", "rocfft")):
        monkeypatch.delenv("CFDJ_SPEC_FFT", raising=False)
        if env is not None:
            monkeypatch.setenv("CFDJ_SPEC_FFT", env)
        with spec.SpectralNS2D(n, n, dx, dy, 1000.0, kind) as h:
            h.upload_interior(w0)
            h.step(2.5e-4, 2)
            out[name] = h.download()
    assert np.isfinite(out["half"]).all()
    assert np.abs(out["half"] - out["rocfft"]).max() <= 1e-12 * np.abs(out["rocfft"]).max()


@pytest.mark.parametrize("kind", ["hybrid", "2/3"])
def test_gpu_spectral_vm_steps_vs_oracle_1024(spec, kind):
    """Vortex-merger steps on the half-spectrum path (n = 1024) against the oracle."""
    n, steps, dt = 1024, 5, 1e-3
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.vm_ic(n, n, x, y)
    ref = so.numerical(w0, steps, dt, dx, dy, 1000.0, KIND_ID[kind])
    with spec.SpectralNS2D(n, n, dx, dy, 1000.0, kind) as h:
        h.upload_interior(w0)
        h.step(dt, steps)
        ut = h.download()
    assert np.abs(ut[:n, :n] - ref).max() < 1e-10
    assert np.array_equal(ut[n, :], ut[0, :]) and np.array_equal(ut[:, n], ut[:, 0])


@pytest.mark.parametrize("kind", KINDS)
def test_gpu_spectral_reference_default_run_to_t20(spec, kind):
    """hybrid.jl:160-165 / pseudospectral_*_rule.jl as shipped: 128^2, dt = .01, tf = 20 (2000
    substep triples), re = 1000, against the oracle after the same steps; the merged vortex
    stands as high as the finite-difference solver's (the reference figures' 0.74)."""
    n, nt = 128, 2000
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.vm_ic(n, n, x, y)
    ref = so.numerical(w0, nt, 0.01, dx, dy, 1000.0, KIND_ID[kind])
    with spec.SpectralNS2D(n, n, dx, dy, 1000.0, kind) as h:
        h.upload_interior(w0)
        h.step(0.01, nt)
        ut = h.download()
    # w_f[1,1] = 0 (hybrid.jl:28) removes the mean: the peak stands 0.74 above the background
    assert 0.72 < ut.max() - ut.min() < 0.76, (ut.max(), ut.min())
    assert np.abs(ut[:n, :n] - ref).max() < 1e-12, np.abs(ut[:n, :n] - ref).max()  # ~1e-15


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("n,steps,dt", [(128, 20, 0.01), (256, 10, 0.005)])
def test_gpu_spectral_vm_steps_vs_oracle(spec, kind, n, steps, dt):
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.vm_ic(n, n, x, y)
    ref = so.numerical(w0, steps, dt, dx, dy, 1000.0, KIND_ID[kind])
    with spec.SpectralNS2D(n, n, dx, dy, 1000.0, kind) as h:
        h.upload_interior(w0)
        h.step(dt, steps)
        ut = h.download()
        wf = h.spectrum()
    assert np.abs(ut[:n, :n] - ref).max() < 1e-10
    assert np.array_equal(ut[n, :], ut[0, :]) and np.array_equal(ut[:, n], ut[:, 0])
    assert wf[0, 0] == 0 or abs(wf[0, 0]) < 1e-9  # hybrid.jl:59 zeroes stages 1-2 only


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("n", [512, 2048])
def test_gpu_spectral_hand_fft_matches_library(spec, monkeypatch, kind, n):
    """Power-of-two grids run hand-written transforms: from 1024 on (hybrid, 2/3 rule) the
    real transforms on the half spectrum (fft2d_r2c.hip), below that -- or with
    CFDJ_SPEC_HALF=0 -- the two-pass complex transform (fft2d_c2c.hip) with real
    physical-space fields; CFDJ_SPEC_REAL=0 keeps those fields complex, CFDJ_SPEC_FFT=rocfft
    keeps the library plans.  All give the same fields to FFT round-off (1e-12 of max|w| after
    3 steps) and the same full spectrum through the C interface."""
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.vm_ic(n, n, x, y)
    out, spc = {}, {}
    envs = ("CFDJ_SPEC_HALF", "CFDJ_SPEC_REAL", "CFDJ_SPEC_FFT")
    for name, env in (("half", {}), ("real", {"CFDJ_SPEC_HALF": "0"}),
                      ("complex", {"CFDJ_SPEC_REAL": "0"}), ("rocfft", {"CFDJ_SPEC_FFT": "rocfft"})):
        for k in envs:
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        with spec.SpectralNS2D(n, n, dx, dy, 1000.0, kind) as h:
            h.upload_interior(w0)
            h.step(1e-3, 3)
            out[name] = h.download()
            spc[name] = h.spectrum()
    scale = np.abs(out["rocfft"]).max()
    sscale = np.abs(spc["rocfft"]).max()
    for name in ("half", "real", "complex"):
        assert np.isfinite(out[name]).all()
        assert np.abs(out[name] - out["rocfft"]).max() <= 1e-12 * scale, name
        assert np.abs(spc[name] - spc["rocfft"]).max() <= 1e-12 * sscale, name


@pytest.mark.parametrize("kind", KINDS)
def test_gpu_spectral_half_spectrum_round_trip(spec, kind):
    """set_spectrum / spectrum through the half-spectrum state (n = 1024), Nyquist row and
    column included, bit for bit: the hybrid solver returns the Hermitian part (w_f(k) +
    conj(w_f(-k))) / 2 of what went in -- for the spectrum of a real field the spectrum itself,
    up to the last-bit asymmetries of the CPU FFT that produced it -- the 2/3 rule the kx
    columns 0..n/2 as given and their conjugate mirror.  The 3/2 rule's state also carries the
    row ky index n/2 of the other half as given: its unpadding (pseudospectral_32_rule.jl:
    171-178) fills that row with the padded grid's mode -n/2, which is not the conjugate of
    the row's first half, so the test makes the two halves of that row differ."""
    n = 1024
    dx, dy, _, _ = vo.vm_grid(n, n)
    f = smooth_field(n, n, 5, n) + 0.01 * np.random.default_rng(7).standard_normal((n, n))
    wf = so.to_spectral(f)
    if kind == "3/2":
        rng = np.random.default_rng(11)
        wf[n // 2 + 1:, n // 2] += rng.standard_normal(n // 2 - 1) + 1j * rng.standard_normal(n // 2 - 1)
    with spec.SpectralNS2D(n, n, dx, dy, 1000.0, kind) as h:
        h.set_spectrum(wf)
        back = h.spectrum()
    mirror = np.conj(wf[(-np.arange(n)) % n][:, (-np.arange(n)) % n])
    herm = 0.5 * (wf + mirror) if kind == "hybrid" else wf
    if kind != "3/2":
        assert np.abs(herm - wf).max() <= 1e-15 * np.abs(wf).max()
    i = np.arange(n // 2 + 1)
    assert np.array_equal(back[i, :], herm[i, :])
    hm = np.conj(herm[(-np.arange(n)) % n][:, (-np.arange(n)) % n])
    if kind == "3/2":
        hm[n // 2 + 1:, n // 2] = wf[n // 2 + 1:, n // 2]
    assert np.array_equal(back[n // 2 + 1:, :], hm[n // 2 + 1:, :])


def _noisy_start(n):
    """The vortex pair plus white noise: content in every mode, the Nyquist row and column
    included, which the 3/2 rule's padding treats unsymmetrically."""
    dx, dy, x, y = vo.vm_grid(n, n)
    return vo.vm_ic(n, n, x, y) + 0.05 * np.random.default_rng(3 * n).standard_normal((n, n))


def test_gpu_spectral_32_rule_noisy_steps_vs_oracle_1024(spec):
    """pseudospectral_32_rule.jl on the half-spectrum state (n = 1024: padded grid 1536 = 3 *
    2^9) against the oracle over 3 steps from a field with content in every mode: the state's
    Nyquist row stops being Hermitian after the first Jacobian (the unpadding takes the padded
    grid's mode -n/2 for it), which the half spectrum carries as an extra row.  Fields to
    1e-10, the full spectrum through the C interface to 1e-12 of its maximum."""
    n, steps, dt = 1024, 3, 1e-3
    dx, dy, _, _ = vo.vm_grid(n, n)
    w0 = _noisy_start(n)
    k2 = so.wavespace(n, n, dx, dy)
    wf = so.to_spectral(w0)
    for _ in range(steps):
        wf = so.step(wf, k2, dt, 1000.0, dx, dy, so.PS32)
    ref = so.to_physical(wf)
    with spec.SpectralNS2D(n, n, dx, dy, 1000.0, "3/2") as h:
        h.upload_interior(w0)
        h.step(dt, steps)
        ut = h.download()
        got = h.spectrum()
    # the oracle's state is not Hermitian on the Nyquist row: the test would not see a
    # symmetrised state otherwise
    hy = n // 2
    asym = np.abs(wf[hy + 1:, hy] - np.conj(wf[1:hy, hy][::-1])).max()
    assert asym > 1e-6 * np.abs(wf[:, hy]).max()
    assert np.abs(ut[:n, :n] - ref).max() < 1e-10
    assert np.abs(got - wf).max() <= 1e-12 * np.abs(wf).max()


@pytest.mark.parametrize("n", [1024, 4096])
def test_gpu_spectral_32_rule_variants_agree(spec, monkeypatch, n):
    """The 3/2 rule's paths on the hand-written 3 * 2^k transforms give the same fields and
    spectra to FFT round-off (1e-12 of the maximum, 2 steps from the noisy start): the
    half-spectrum state with the product fused into the row passes (default), the product as
    a kernel of its own (CFDJ_SPEC_PS32_FUSE=0), and the full-spectrum state with separate
    derivative / unpadding kernels (CFDJ_SPEC_HALF=0)."""
    dx, dy, _, _ = vo.vm_grid(n, n)
    w0 = _noisy_start(n)
    out, spc = {}, {}
    envs = ("CFDJ_SPEC_PS32_FUSE", "CFDJ_SPEC_HALF")
    for name, env in (("fused", {}), ("unfused", {"CFDJ_SPEC_PS32_FUSE": "0"}),
                      ("full", {"CFDJ_SPEC_HALF": "0"})):
        for k in envs:
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        with spec.SpectralNS2D(n, n, dx, dy, 1000.0, "3/2") as h:
            h.upload_interior(w0)
            h.step(2.5e-4, 2)
            out[name] = h.download()
            spc[name] = h.spectrum()
    scale, sscale = np.abs(out["full"]).max(), np.abs(spc["full"]).max()
    for name in ("fused", "unfused"):
        assert np.isfinite(out[name]).all()
        assert np.abs(out[name] - out["full"]).max() <= 1e-12 * scale, name
        assert np.abs(spc[name] - spc["full"]).max() <= 1e-12 * sscale, name


@pytest.mark.parametrize("kind", KINDS)
def test_gpu_spectral_tgv_known_answer(spec, kind):
    """Taylor-Green: J(w, psi) = 0, so the field decays by the scheme's exact factor."""
    n, re, dt, nt = 64, 10.0, 0.01, 50
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.exact_tgv(x, y, 0.0, re)[:n, :n].copy()
    g = so.cn_decay(n, dx, dt, re, nt, 4, 4)
    with spec.SpectralNS2D(n, n, dx, dy, re, kind) as h:
        h.upload_interior(w0)
        h.step(dt, nt)
        ut = h.download()
    assert np.abs(ut[:n, :n] - g * w0).max() < 1e-12
    assert abs(g - math.exp(-2 * 16 * nt * dt / re)) < 1e-5  # CN-RK3 vs exact decay


def test_gpu_spectral_reference_signature(spec, tmp_path):
    c = spec.setup(nx=64, ny=64, dt=0.01, tf=0.2, ns=2)
    ref = so.numerical(c["wn"][1:-1, 1:-1], c["nt"], c["dt"], c["dx"], c["dy"], c["re"],
                       so.HYBRID)
    un = spec.numerical(c["nx"], c["ny"], c["nt"], c["dx"], c["dy"], c["dt"], c["re"], c["x"],
                        c["y"], c["wn"], c["ns"], "hybrid", snapshot_dir=str(tmp_path))
    assert un.shape == (65, 65) and np.abs(un[:64, :64] - ref).max() < 1e-10
    assert (tmp_path / "vm1.txt").exists() and (tmp_path / "vm2.txt").exists()


def test_gpu_spectral_argument_errors(spec):
    from cfd_julia_amd import _lib

    dx = 2 * math.pi / 64
    with pytest.raises(_lib.ArgumentError):
        spec.SpectralNS2D(64, 32, dx, dx, 1000.0)  # ky = kx aliasing: square only
    with pytest.raises(_lib.ArgumentError):
        spec.SpectralNS2D(63, 63, dx, dx, 1000.0)  # odd nx


def test_gpu_spectral_jacobian_of_a_non_hermitian_spectrum(spec):
    """hybrid.jl:92-152 takes real(ifft(.)) of w_f and of w_f / k2 (k2 even), i.e. it sees the
    Hermitian part of w_f only.  A w_f that is NOT the spectrum of a real field must therefore
    give the oracle's Jacobian on the half-spectrum path (n = 1024) as on the full-spectrum
    ones (n = 96: library transforms, n = 256: hand-written).  (The pseudospectral rules'
    i k and band-filter multipliers are not Hermitian at index 1 and on the filter's edge:
    they are defined here for spectra of real fields, like the reference's loop produces.)"""
    for n in (96, 256, 1024):
        dx, dy, _, _ = vo.vm_grid(n, n)
        rng = np.random.default_rng(7 * n)
        wf = _noisy_spectrum(n) + n * (rng.standard_normal((n, n))
                                       + 1j * rng.standard_normal((n, n)))
        wf[0, 0] = 0.0  # as every spectrum of the loop (hybrid.jl:28): k2[1,1] = 2 eps^2
        ref = so.jacobian_hybrid(wf, so.wavespace(n, n, dx, dy), dx, dy)
        with spec.SpectralNS2D(n, n, dx, dy, 1000.0, "hybrid") as h:
            got = h.jacobian(wf)
        assert np.abs(got - ref).max() <= 1e-12 * np.abs(ref).max(), n


@pytest.mark.parametrize("n", [1024, 2048, 4096])
def test_gpu_spectral_32_rule_hand_transforms_vs_library(spec, monkeypatch, n):
    """pseudospectral_32_rule.jl:94-186 on product grids of 3 * 2^k points (1536, 3072, 6144 = 1.5
    x the benchmarked 4096): the hand-written radix-3 + power-of-two transforms on the columns
    0..nx/2 of the padded half spectrum (fft2d_r2c3.hip) against the library's real transforms
    (CFDJ_SPEC_PS32_HAND=0) on a field with content in every mode: one Jacobian to 1e-12 of
    max|jf|, and at 1024 also against the oracle."""
    dx, dy, _, _ = vo.vm_grid(n, n)
    wf = _noisy_spectrum(n)
    out = {}
    for name, env in (("hand", None), ("library", "0")):
        monkeypatch.delenv("CFDJ_SPEC_PS32_HAND", raising=False)
        if env is not None:
            monkeypatch.setenv("CFDJ_SPEC_PS32_HAND", env)
        with spec.SpectralNS2D(n, n, dx, dy, 1000.0, "3/2") as h:
            out[name] = h.jacobian(wf)
    scale = np.abs(out["library"]).max()
    assert np.isfinite(out["hand"]).all()
    assert np.abs(out["hand"] - out["library"]).max() <= 1e-12 * scale
    if n == 1024:
        ref = so.jacobian_ps32(wf, so.wavespace(n, n, dx, dy), dx, dy)
        assert np.abs(out["hand"] - ref).max() <= 1e-12 * np.abs(ref).max()


@pytest.mark.parametrize("n", [1024, 2048, 4096])
def test_gpu_spectral_23_rule_fused_product_matches_unfused(spec, monkeypatch, n):
    """pseudospectral_23_rule.jl:134-140 on the half-spectrum path: the fourth field's inverse
    row pass, the product and its forward row pass as one kernel (default, grids of up to
    4096^2) against the separate kernels (CFDJ_SPEC_PS23_FUSE=0): one Jacobian of the noisy
    spectrum to 1e-12 of max|jf|, fields and spectra after 2 steps to 1e-12 of their maxima."""
    dx, dy, _, _ = vo.vm_grid(n, n)
    wf = _noisy_spectrum(n)
    w0 = _noisy_start(n)
    jac, out, spc = {}, {}, {}
    for name, env in (("fused", None), ("unfused", "0")):
        monkeypatch.delenv("CFDJ_SPEC_PS23_FUSE", raising=False)
        if env is not None:
            monkeypatch.setenv("CFDJ_SPEC_PS23_FUSE", env)
        with spec.SpectralNS2D(n, n, dx, dy, 1000.0, "2/3") as h:
            jac[name] = h.jacobian(wf)
            h.upload_interior(w0)
            h.step(2.5e-4, 2)
            out[name] = h.download()
            spc[name] = h.spectrum()
    assert np.isfinite(out["fused"]).all()
    assert np.abs(jac["fused"] - jac["unfused"]).max() <= 1e-12 * np.abs(jac["unfused"]).max()
    assert np.abs(out["fused"] - out["unfused"]).max() <= 1e-12 * np.abs(out["unfused"]).max()
    assert np.abs(spc["fused"] - spc["unfused"]).max() <= 1e-12 * np.abs(spc["unfused"]).max()
