"""CPU oracle of the two small solvers beside the Navier-Stokes paths (TEST INFRASTRUCTURE ONLY):

  * 15_Poisson_Solver_Gauss_Seidel/gauss_seidel.jl:8-54 -- the reference's "Gauss-Seidel"
    is a Jacobi sweep (r = f - lap(u_old) everywhere, then u += r / dd), so a vectorised
    NumPy restatement reproduces it exactly;
  * 01_Heat_Equation_FTCS/ftcs.jl:9-64 -- 1D heat FTCS with the analytic decay check.
"""
from __future__ import annotations

import math

import numpy as np

from .cavity_oracle import compute_l2norm, compute_residual


def jacobi_sweep(f, u, dx, dy):
    C, E, W = slice(1, -1), slice(2, None), slice(0, -2)
    r = np.zeros_like(u)
    r[C, C] = f[C, C] - ((u[E, C] - 2 * u[C, C] + u[W, C]) / (dx * dx)
                         + (u[C, E] - 2 * u[C, C] + u[C, W]) / (dy * dy))
    un = u.copy()
    un[C, C] += r[C, C] / (-2 / (dx * dx) - 2 / (dy * dy))
    return un, r


def gauss_seidel(f, u, dx, dy, max_iter, tol, freq=10000):
    """gauss_seidel.jl:8-54: returns (u, iterations, last rms)."""
    r = compute_residual(f, u, dx, dy)
    init_rms = rms = compute_l2norm(r)
    it = 0
    while it < 5 * max_iter:
        it += 1
        u, r = jacobi_sweep(f, u, dx, dy)
        if it % freq == 0:
            r = compute_residual(f, u, dx, dy)
            rms = compute_l2norm(r)
            if rms / init_rms <= tol:
                break
    return u, it, rms


def ftcs_setup(dx=0.025, dt=0.0025, t=1.0, x_l=-1.0, x_r=1.0):
    """ftcs.jl:10-32."""
    nx = int(round((x_r - x_l) / dx))
    nt = int(round(t / dt))
    alpha = 1.0 / math.pi ** 2
    x = x_l + dx * np.arange(nx + 1)
    u0 = -np.sin(math.pi * x)
    u0[0] = 0.0
    u0[-1] = 0.0
    ue = -math.exp(-t) * np.sin(math.pi * x)
    beta = alpha * dt / (dx * dx)
    return nx, nt, beta, x, u0, ue


def ftcs(u0, nt, beta):
    """ftcs.jl:34-41: history (nx+1, nt+1)."""
    nx = u0.size - 1
    un = np.zeros((nx + 1, nt + 1), order="F")
    un[:, 0] = u0
    for k in range(1, nt + 1):
        a = un[:, k - 1]
        un[1:nx, k] = a[1:nx] + beta * (a[2:nx + 1] - 2 * a[1:nx] + a[0:nx - 1])
        un[0, k] = 0.0
        un[nx, k] = 0.0
    return un


def compute_l2norm_1d(nx, r):
    """Common.jl:224-227: sqrt(sum r[2:nx]^2 / (nx - 1))."""
    a = r[1:nx]
    return math.sqrt(float(np.sum(a * a)) / (nx - 1))
