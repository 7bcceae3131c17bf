"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

The reference (Julia) cannot run in this image (no julia binary,
unregistered Unroll/Utils deps), so the fixtures are produced by oracle/vm_oracle.py,
which is itself pinned to the reference's published numbers (order.jl:10-11) and the
analytic TGV decay (tgv.jl:82-90) -- see tests/test_oracle.py.  Re-run with
    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import vm_oracle as vo  # noqa: E402


def smooth_field(nx, ny, kmax, seed):
    """Random smooth periodic field: Fourier modes |k| <= kmax, seeded."""
    rng = np.random.default_rng(seed)
    dx, dy, x, y = vo.vm_grid(nx, ny)
    X, Y = x[:nx, None], y[None, :ny]
    w = np.zeros((nx, ny))
    for kx in range(-kmax, kmax + 1):
        for ky in range(-kmax, kmax + 1):
            a, b = rng.standard_normal(2) / (1.0 + kx * kx + ky * ky)
            w += a * np.cos(kx * X + ky * Y) + b * np.sin(kx * X + ky * Y)
    return w


def smooth_field_fast(nx, ny, kmax, seed):
    """The same field as smooth_field (same draws, same modes) assembled from products of
    1-D cos / sin tables -- cos(kx x + ky y) = cos kx x cos ky y - sin kx x sin ky y -- as four
    matrix products instead of (2 kmax + 1)^2 full-grid passes; equal to smooth_field up to
    rounding.  For the large GPU test grids (not for the committed fixtures)."""
    rng = np.random.default_rng(seed)
    dx, dy, x, y = vo.vm_grid(nx, ny)
    k = np.arange(-kmax, kmax + 1)
    ab = rng.standard_normal((k.size, k.size, 2)) / (1.0 + k[:, None] ** 2 + k[None, :] ** 2)[..., None]
    A, B = ab[..., 0], ab[..., 1]
    cx, sx = np.cos(np.outer(x[:nx], k)), np.sin(np.outer(x[:nx], k))
    cy, sy = np.cos(np.outer(k, y[:ny])), np.sin(np.outer(k, y[:ny]))
    return cx @ (A @ cy + B @ sy) + sx @ (B @ cy - A @ sy)


def main():
    out = {}
    # FD-FFT Poisson on the fft_p.jl MMS (12_Poisson_Solver_FFT/fft_p.jl:67-92)
    for n in (32, 64):
        f, ue, dx, dy = vo.fft_p_mms(n)
        s = vo.ps_fft(np.ascontiguousarray(f[:n, :n]), dx, dy)
        np.savez_compressed(os.path.join(HERE, f"fps_mms_{n}.npz"), f=f[:n, :n], s=s,
                            dx=dx, dy=dy)
        out[f"fps_mms_{n}"] = float(np.abs(s).max())
    # vm_rhs on a random smooth vorticity (Common.jl:132-182), 64x64 and 96x64 (ny < nx)
    for nx, ny, seed in ((64, 64, 1), (96, 64, 2)):
        w = smooth_field(nx, ny, 6, seed)
        dx, dy, _, _ = vo.vm_grid(nx, ny)
        r, s = vo.vm_rhs(w, dx, dy, 1000.0)
        np.savez_compressed(os.path.join(HERE, f"vm_rhs_{nx}x{ny}.npz"), w=w, r=r, s=s,
                            dx=dx, dy=dy, re=1000.0)
        out[f"vm_rhs_{nx}x{ny}"] = float(np.abs(r).max())
    # vortex merger, vm.jl setup at 64^2, re = 1000, dt = 0.01, 10 RK3 steps
    nx = ny = 64
    dx, dy, x, y = vo.vm_grid(nx, ny)
    w0 = vo.vm_ic(nx, ny, x, y)
    w10 = vo.numerical(w0, 10, 0.01, dx, dy, 1000.0)
    np.savez_compressed(os.path.join(HERE, "vm_64_10steps.npz"), w0=w0, w10=w10, dx=dx,
                        dy=dy, re=1000.0, dt=0.01, nt=10)
    out["vm_64_10steps"] = float(np.abs(w10).max())
    # Taylor-Green (tgv.jl:92-139): 64^2, re = 10, dt = 0.01, t = 1
    l2, linf = vo.tgv_error(64, 10.0, 0.01, 1.0)
    np.savez_compressed(os.path.join(HERE, "tgv_64.npz"), l2=l2, linf=linf)
    out["tgv_64"] = (l2, linf)
    for k, v in out.items():
        print(k, v)


if __name__ == "__main__":
    main()
