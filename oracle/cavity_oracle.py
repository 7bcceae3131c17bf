"""CPU oracle for the secondary paths (TEST INFRASTRUCTURE ONLY, like vm_oracle.py):

  * lid-driven cavity, 18_NS2D_Lid_Driven_Cavity/lid_driven_cavity.jl:11-159
    (fps_sine DST-I Poisson, bc2 Jensen wall vorticity, rhs, RK3 + RMS monitor);
  * n-level V-cycle multigrid, 17_Poisson_Solver_Multigrid/mg_N.jl:7-114 with
    Common.jl:21-92 (restriction, prolongation, lexicographic Gauss-Seidel) and
    Common.jl:229-246 (compute_l2norm, compute_residual).

Arrays are (nx+1, ny+1) node fields indexed [i, j] (0-based; the reference's [i+1, j+1]),
expression order copied from the reference source.  FFTW's RODFT00 is scipy.fft.dst
type 1 (same unnormalised definition y_k = 2 sum x_n sin(pi (n+1)(k+1)/(N+1))).
Parity pinning: the cavity has no stored reference output (parity unpinned by the
reference's own tests beyond physics: zero-mean divergence, lid-driven circulation); the
multigrid MMS (mg_N.jl:152-161, ipr = 1) has a quadratic exact solution which the 5-point
Laplacian reproduces exactly, so the converged solver error is the solver tolerance.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.fft as sfft


# ---- lid-driven cavity -----------------------------------------------------------------
def cavity_grid(nx, ny):
    """lid_driven_cavity.jl:162-186: unit box, x[i] = Δx(i-1)."""
    dx = (1.0 - 0.0) / nx
    dy = (1.0 - 0.0) / ny
    return dx, dy, dx * np.arange(nx + 1), dy * np.arange(ny + 1)


def iden_table(nx, ny, dx, dy):
    """lid_driven_cavity.jl:64-69 for i, j = 1..nx-1 (the part fps_sine uses)."""
    i = np.arange(1, nx)
    j = np.arange(1, ny)
    tx = (2 / (dx * dx)) * (np.array([math.cos(math.pi * k / nx) for k in i]) - 1.0)
    ty = (2 / (dy * dy)) * (np.array([math.cos(math.pi * k / ny) for k in j]) - 1.0)
    return 1.0 / (tx[:, None] + ty[None, :])


def fps_sine(f, dx, dy, iden=None):
    """lid_driven_cavity.jl:11-21: DST-I Poisson; f is (nx+1, ny+1), returns s with
    s[1:nx, 1:ny] solved (Julia s[2:nx, 2:ny]) and a zero boundary."""
    nx, ny = f.shape[0] - 1, f.shape[1] - 1
    if iden is None:
        iden = iden_table(nx, ny, dx, dy)
    e = sfft.dstn(np.array(f[1:nx, 1:ny]), type=1)
    data1 = e * iden
    s = np.zeros_like(f)
    s[1:nx, 1:ny] = sfft.dstn(data1, type=1) / ((2 * nx) * (2 * ny))
    return s


def ps_fst(f, dx, dy):
    """14_Poisson_Solver_FST/fft_d.jl:7-23: the same solve with the symbol DIVIDED into the
    sine coefficients (fft_d.jl:15-20) instead of multiplied by a tabulated reciprocal;
    f is (nx+1, ny+1), returns the (nx-1, ny-1) interior solution."""
    nx, ny = f.shape[0] - 1, f.shape[1] - 1
    e = sfft.dstn(np.array(f[1:nx, 1:ny]), type=1)
    cx = np.array([math.cos(math.pi * k / nx) for k in range(1, nx)])
    cy = np.array([math.cos(math.pi * k / ny) for k in range(1, ny)])
    data1 = e / ((2.0 / dx ** 2) * (cx[:, None] - 1.0) + (2.0 / dy ** 2) * (cy[None, :] - 1.0))
    return sfft.dstn(data1, type=1) / (2 * nx * 2 * ny)


def fft_d_mms(nx, km=16):
    """fft_d.jl:26-62: the manufactured solution of 12/fft_p.jl on the unit box (its
    right-hand side is odd about every wall, so it is also a Dirichlet problem)."""
    dx = dy = (1.0 - 0.0) / nx
    x = 0.0 + dx * np.arange(nx + 1)
    X, Y = x[:, None], x[None, :]
    tp = 2 * math.pi
    c1, c2 = (1.0 / km) ** 2, -8 * math.pi ** 2
    ue = np.sin(tp * X) * np.sin(tp * Y) + c1 * np.sin(km * tp * X) * np.sin(km * tp * Y)
    f = c2 * np.sin(tp * X) * np.sin(tp * Y) + c2 * np.sin(km * tp * X) * np.sin(km * tp * Y)
    return f, ue, dx, dy


def fft_d_mms_error(nx, solver="ps_fst"):
    """fft_d.jl:64-75: (L2 over all (nx+1)(ny+1) nodes, Linf) of un - ue."""
    f, ue, dx, dy = fft_d_mms(nx)
    un = np.zeros_like(f)
    if solver == "ps_fst":
        un[1:nx, 1:nx] = ps_fst(f, dx, dy)
    else:
        un = fps_sine(f, dx, dy)
    err = un - ue
    return float(np.sqrt(np.sum(err ** 2) / ((nx + 1) * (nx + 1)))), float(np.abs(err).max())


def bc2(w, s, dx, dy):
    """lid_driven_cavity.jl:39-51 (Jensen, 2nd order), in place; the i-loop (bottom/top)
    runs second and overwrites the corners."""
    nx, ny = w.shape[0] - 1, w.shape[1] - 1
    w[0, :] = (-4 * s[1, :] + 0.5 * s[2, :]) / (dx * dx)
    w[nx, :] = (-4 * s[nx - 1, :] + 0.5 * s[nx - 2, :]) / (dx * dx)
    w[:, 0] = (-4 * s[:, 1] + 0.5 * s[:, 2]) / (dy * dy)
    w[:, ny] = (-4 * s[:, ny - 1] + 0.5 * s[:, ny - 2]) / (dy * dy) - 3.0 / dy
    return w


def cavity_rhs(w, s, dx, dy, re):
    """lid_driven_cavity.jl:124-159 on the interior (gg applied per term)."""
    aa = 1 / (re * (dx * dx))
    bb = 1 / (re * (dy * dy))
    gg = 1 / ((4 * dx) * dy)
    hh = 1 / 3
    C = slice(1, -1)
    E, W = slice(2, None), slice(0, -2)
    wc = w[C, C]
    wE, wW, wN, wS = w[E, C], w[W, C], w[C, E], w[C, W]
    wNE, wSW, wNW, wSE = w[E, E], w[W, W], w[W, E], w[E, W]
    sE, sW, sN, sS = s[E, C], s[W, C], s[C, E], s[C, W]
    sNE, sSW, sNW, sSE = s[E, E], s[W, W], s[W, E], s[E, W]
    j1 = gg * ((wE - wW) * (sN - sS) - (wN - wS) * (sE - sW))
    j2 = gg * (wE * (sNE - sSE) - wW * (sNW - sSW) - wN * (sNE - sNW) + wS * (sSE - sSW))
    j3 = gg * (wNE * (sN - sE) - wSW * (sW - sS) - wNW * (sN - sW) + wSE * (sE - sS))
    jac = (j1 + j2 + j3) * hh
    r = np.zeros_like(w)
    r[C, C] = -jac + (aa * (wE - 2 * wc + wW) + bb * (wN - 2 * wc + wS))
    return r


def cavity_step(wn, sn, dt, dx, dy, re, iden):
    """One RK3 step, lid_driven_cavity.jl:75-114; returns (wn, sn, rms)."""
    I = (slice(1, -1), slice(1, -1))
    sp = sn.copy()
    r = cavity_rhs(wn, sn, dx, dy, re)
    wt = np.zeros_like(wn)
    wt[I] = wn[I] + dt * r[I]
    bc2(wt, sn, dx, dy)
    sn = fps_sine(-wt, dx, dy, iden)
    r = cavity_rhs(wt, sn, dx, dy, re)
    wt[I] = (0.75 * wn[I] + 0.25 * wt[I]) + (0.25 * dt) * r[I]
    bc2(wt, sn, dx, dy)
    sn = fps_sine(-wt, dx, dy, iden)
    r = cavity_rhs(wt, sn, dx, dy, re)
    wn = wn.copy()
    wn[I] = ((1 / 3) * wn[I] + (2 / 3) * wt[I]) + ((2 / 3) * dt) * r[I]
    bc2(wn, sn, dx, dy)
    sn = fps_sine(-wn, dx, dy, iden)
    d = sn - sp
    rms = math.sqrt(float(np.sum(d * d)) / ((wn.shape[0]) * (wn.shape[1])))
    return wn, sn, rms


def cavity_numerical(nx, ny, nt, dt, re, wn=None, sn=None):
    """lid_driven_cavity.jl:58-118 from rest (wn = sn = 0, :188-191); returns (wn, sn, rms)."""
    dx, dy, _, _ = cavity_grid(nx, ny)
    wn = np.zeros((nx + 1, ny + 1)) if wn is None else wn.copy()
    sn = np.zeros((nx + 1, ny + 1)) if sn is None else sn.copy()
    iden = iden_table(nx, ny, dx, dy)
    rms = np.empty(nt)
    for k in range(nt):
        wn, sn, rms[k] = cavity_step(wn, sn, dt, dx, dy, re, iden)
    return wn, sn, rms


# ---- multigrid (Common.jl:21-92, 229-246; mg_N.jl:7-114) --------------------------------
def compute_residual(f, u, dx, dy):
    """Common.jl:239-246 on the interior."""
    r = np.zeros_like(u)
    C, E, W = slice(1, -1), slice(2, None), slice(0, -2)
    r[C, C] = f[C, C] - ((u[E, C] - 2 * u[C, C] + u[W, C]) / (dx * dx)
                         + (u[C, E] - 2 * u[C, C] + u[C, W]) / (dy * dy))
    return r


def compute_l2norm(r):
    """Common.jl:229-232: sqrt(sum r[2:nx,2:ny]^2 / ((nx-1)(ny-1)))."""
    a = r[1:-1, 1:-1]
    return math.sqrt(float(np.sum(a * a)) / a.size)


def gauss_seidel_lex(f, u, dx, dy, sweeps):
    """Common.jl:78-92: in-place LEXICOGRAPHIC Gauss-Seidel (j outer, i inner).  Pure
    Python loops: small grids only."""
    nx, ny = u.shape[0] - 1, u.shape[1] - 1
    dd = -2 / (dx * dx) - 2 / (dy * dy)
    for _ in range(sweeps):
        for j in range(1, ny):
            for i in range(1, nx):
                rt = f[i, j] - ((u[i + 1, j] - 2 * u[i, j] + u[i - 1, j]) / (dx * dx)
                                + (u[i, j + 1] - 2 * u[i, j] + u[i, j - 1]) / (dy * dy))
                u[i, j] += rt / dd
    return u


def gauss_seidel_rb(f, u, dx, dy, sweeps):
    """Red-black ordering of the same update (what libcfdj runs on the GPU): each sweep
    updates the (i+j) even points, then the odd points, with the reference's formula."""
    C, E, W = slice(1, -1), slice(2, None), slice(0, -2)
    dd = -2 / (dx * dx) - 2 / (dy * dy)
    nx, ny = u.shape[0] - 1, u.shape[1] - 1
    I, J = np.meshgrid(np.arange(1, nx), np.arange(1, ny), indexing="ij")
    for _ in range(sweeps):
        for parity in (0, 1):
            mask = ((I + J) % 2) == parity
            rt = f[C, C] - ((u[E, C] - 2 * u[C, C] + u[W, C]) / (dx * dx)
                            + (u[C, E] - 2 * u[C, C] + u[C, W]) / (dy * dy))
            upd = u[C, C] + rt / dd
            u[C, C] = np.where(mask, upd, u[C, C])
    return u


def restriction(r, nxc, nyc):
    """Common.jl:21-48: full weighting on the interior, injection on the boundary."""
    ec = np.zeros((nxc + 1, nyc + 1))
    F = r
    i = np.arange(1, nxc)[:, None]
    j = np.arange(1, nyc)[None, :]
    fi, fj = 2 * i, 2 * j
    center = 4 * F[fi, fj]
    grid = 2 * (F[fi, fj + 1] + F[fi, fj - 1] + F[fi + 1, fj] + F[fi - 1, fj])
    corner = F[fi + 1, fj + 1] + F[fi + 1, fj - 1] + F[fi - 1, fj + 1] + F[fi - 1, fj - 1]
    ec[1:nxc, 1:nyc] = (center + grid + corner) / 16
    nxf, nyf = r.shape[0] - 1, r.shape[1] - 1
    jj = np.arange(nyc + 1)
    ec[0, :] = r[0, 2 * jj]
    ec[nxc, :] = r[nxf, 2 * jj]
    ii = np.arange(nxc + 1)
    ec[:, 0] = r[2 * ii, 0]
    ec[:, nyc] = r[2 * ii, nyf]
    return ec


def prolongation(unc, nxf, nyf):
    """Common.jl:50-76: bilinear interpolation + boundary copy."""
    nxc, nyc = unc.shape[0] - 1, unc.shape[1] - 1
    ef = np.zeros((nxf + 1, nyf + 1))
    u = unc
    ef[0:2 * nxc:2, 0:2 * nyc:2] = u[:nxc, :nyc]
    ef[0:2 * nxc:2, 1:2 * nyc:2] = 0.5 * (u[:nxc, :nyc] + u[:nxc, 1:nyc + 1])
    ef[1:2 * nxc:2, 0:2 * nyc:2] = 0.5 * (u[:nxc, :nyc] + u[1:nxc + 1, :nyc])
    ef[1:2 * nxc:2, 1:2 * nyc:2] = 0.25 * (u[:nxc, :nyc] + u[:nxc, 1:nyc + 1]
                                           + u[1:nxc + 1, :nyc] + u[1:nxc + 1, 1:nyc + 1])
    ii = np.arange(nxc + 1)
    ef[2 * ii, 0] = u[:, 0]
    ef[2 * ii, nyf] = u[:, nyc]
    jj = np.arange(nyc + 1)
    ef[0, 2 * jj] = u[0, :]
    ef[nxf, 2 * jj] = u[nxc, :]
    return ef


def mg_n(f, u, dx, dy, n_level, v1=2, v2=2, v3=2, tol=1e-9, max_iter=100000,
         smoother=gauss_seidel_rb):
    """mg_N.jl:7-114 (V-cycle with the reference's level/sweep structure).  Returns
    (u, iterations, [rms history incl. iteration 0])."""
    nx, ny = u.shape[0] - 1, u.shape[1] - 1
    u = u.copy()
    r = compute_residual(f, u, dx, dy)
    init_rms = rms = compute_l2norm(r)
    hist = [rms]
    lnx, lny, ldx, ldy = [nx], [ny], [dx], [dy]
    for _ in range(1, n_level):
        lnx.append(lnx[-1] // 2)
        lny.append(lny[-1] // 2)
        ldx.append(2 * ldx[-1])
        ldy.append(2 * ldy[-1])
    u_mg = [u] + [np.zeros((lnx[k] + 1, lny[k] + 1)) for k in range(1, n_level)]
    f_mg = [f] + [np.zeros((lnx[k] + 1, lny[k] + 1)) for k in range(1, n_level)]
    it = 0
    while it < max_iter:
        it += 1
        smoother(f_mg[0], u_mg[0], ldx[0], ldy[0], v1)
        r = compute_residual(f_mg[0], u_mg[0], ldx[0], ldy[0])
        rms = compute_l2norm(r)
        hist.append(rms)
        if rms / init_rms <= tol:
            break
        for k in range(1, n_level):
            tmp = r if k == 1 else compute_residual(f_mg[k - 1], u_mg[k - 1], ldx[k - 1],
                                                   ldy[k - 1])
            f_mg[k] = restriction(tmp, lnx[k], lny[k])
            u_mg[k][...] = 0.0
            smoother(f_mg[k], u_mg[k], ldx[k], ldy[k], v1 if k < n_level - 1 else v2)
        for k in range(n_level - 1, 0, -1):
            p = prolongation(u_mg[k], lnx[k - 1], lny[k - 1])
            u_mg[k - 1][1:-1, 1:-1] += p[1:-1, 1:-1]
            smoother(f_mg[k - 1], u_mg[k - 1], ldx[k - 1], ldy[k - 1], v3)
    return u_mg[0], it, hist


def mg_2level(f, u, dx, dy, v1=2, v2=2, v3=2, tol=1e-9, max_iter=100000,
              smoother=gauss_seidel_rb):
    """17_Poisson_Solver_Multigrid/mg.jl:7-85, the two-level cycle: v1 sweeps on the fine
    grid (mg.jl:44), convergence check (:47-58), restriction (:61), v3 sweeps on the coarse
    grid from zero (:63-66), prolongation + correction (:70-75), v2 sweeps on the fine grid
    (:77).  Returns (u, iterations, [rms history incl. iteration 0], final residual r)."""
    nx, ny = u.shape[0] - 1, u.shape[1] - 1
    u = u.copy()
    r = compute_residual(f, u, dx, dy)
    init_rms = rms = compute_l2norm(r)
    hist = [rms]
    nxc, nyc = nx // 2, ny // 2
    dxc, dyc = dx * 2, dy * 2
    it = 0
    while it < max_iter:
        it += 1
        smoother(f, u, dx, dy, v1)
        r = compute_residual(f, u, dx, dy)
        rms = compute_l2norm(r)
        hist.append(rms)
        if rms / init_rms <= tol:
            break
        fc = restriction(r, nxc, nyc)
        unc = np.zeros_like(fc)
        smoother(fc, unc, dxc, dyc, v3)
        p = prolongation(unc, nx, ny)
        u[1:-1, 1:-1] += p[1:-1, 1:-1]
        smoother(f, u, dx, dy, v2)
    return u, it, hist, r


def mg_mms(nx, ny=None, ipr=1):
    """mg_N.jl:127-169: unit box MMS, Dirichlet boundary from the exact solution."""
    ny = nx if ny is None else ny
    dx = 1.0 / nx
    dy = 1.0 / ny
    x = dx * np.arange(nx + 1)
    y = dy * np.arange(ny + 1)
    X, Y = x[:, None], y[None, :]
    if ipr == 1:
        ue = (X ** 2 - 1) * (Y ** 2 - 1)
        f = -2 * (2 - X ** 2 - Y ** 2)
    else:
        c1 = (1.0 / 16) ** 2
        c2 = -2 * math.pi ** 2
        ue = (np.sin(2 * math.pi * X) * np.sin(2 * math.pi * Y)
              + c1 * np.sin(16 * math.pi * X) * np.sin(16 * math.pi * Y))
        f = (4 * c2 * np.sin(2 * math.pi * X) * np.sin(2 * math.pi * Y)
             + c2 * np.sin(16 * math.pi * X) * np.sin(16 * math.pi * Y))
    un = np.zeros_like(ue)
    un[:, 0] = ue[:, 0]
    un[:, ny] = ue[:, ny]
    un[0, :] = ue[0, :]
    un[nx, :] = ue[nx, :]
    return f, ue, un, dx, dy
