"""Host-side mirror of `01_Heat_Equation_FTCS/ftcs.jl` (BASELINE config 1: CPU plumbing
only).  The update runs in libcfdj.so's host code (cfdj_ftcs); no GPU is involved."""
from __future__ import annotations

import math

import numpy as np

from . import _lib
from ._lib import check, dptr


def ftcs(u0, nt, beta):
    """ftcs.jl:34-41: returns the (nx+1, nt+1) history."""
    u0 = np.ascontiguousarray(u0, dtype=np.float64)
    nx = u0.size - 1
    un = np.zeros((nx + 1, nt + 1), order="F")
    check(_lib.load().cfdj_ftcs(int(nx), int(nt), float(beta), dptr(u0), dptr(un),
                                un.shape[0]), "cfdj_ftcs")
    return un


def main(dx=0.025, dt=0.0025, t=1.0):
    """ftcs.jl:9-64 without files: returns (L2, Linf) of the error at t vs -e^{-t} sin(pi x)."""
    x_l, x_r = -1.0, 1.0
    nx = int(round((x_r - x_l) / dx))
    nt = int(round(t / dt))
    alpha = 1.0 / math.pi ** 2
    x = x_l + dx * np.arange(nx + 1)
    u0 = -np.sin(math.pi * x)
    u0[0] = u0[-1] = 0.0
    ue = -math.exp(-t) * np.sin(math.pi * x)
    un = ftcs(u0, nt, alpha * dt / (dx * dx))
    err = un[:, nt] - ue
    a = err[1:nx]
    return math.sqrt(float(np.sum(a * a)) / (nx - 1)), float(np.max(np.abs(err)))
