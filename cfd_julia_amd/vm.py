"""Host-side mirror of `19_NS2D_Vortex_Merger/vm.jl` (and the RK3 loop of `tgv.jl`).

`numerical` keeps the reference signature (vm.jl:12) and semantics: wn is the ghosted
(nx+2, ny+2) Julia-layout array, mutated in place to the final state; the return value is
the (nx+1, ny+1) array wn[2:nx+2, 2:ny+2] including the duplicated periodic node.  The
whole time loop runs on the GPU (libcfdj.so); between snapshots nothing returns to the
host.
"""
from __future__ import annotations

import math
import os

import numpy as np

from .common import periodic_ghosts, vm_ic
from .fieldio import write_field
from .solver import VortexMerger


def _write_field(path, x, y, ut):
    """vm.jl:81-85 format: "x y ω" per line, j outer / i inner over (nx+1)(ny+1) nodes,
    numbers as Julia prints them (fieldio.julia_str)."""
    write_field(path, x, y, ut)


def numerical(nx, ny, nt, dx, dy, dt, re, x, y, wn, ns, *, snapshots=True, outdir=".",
              fix_snapshot_index=False, eps=1e-6, device=-1):
    """vm.jl:12-90.  Every nt÷ns steps the reference prints k and writes vm$m.txt; its
    m is never incremented (vm.jl:21,81), so every snapshot overwrites vm1.txt --
    reproduced unless fix_snapshot_index=True.  snapshots=False skips the text output
    (benchmarks).  nt < ns raises ZeroDivisionError like Julia's mod(k, 0)."""
    freq = nt // ns
    m = 1
    with VortexMerger(nx, ny, dx, dy, re, eps, device) as h:
        h.upload(wn)
        k = 0
        while k < nt:
            if snapshots:
                if freq == 0:
                    raise ZeroDivisionError("mod(k, nt ÷ ns) with nt < ns (vm.jl:22,78)")
                chunk = freq - (k % freq)
            else:
                chunk = nt - k
            chunk = min(chunk, nt - k)
            h.step(dt, chunk)
            k += chunk
            if snapshots and k % freq == 0:
                print(f"k = {k}")
                w = h.download()
                _write_field(os.path.join(outdir, f"vm{m}.txt"), x, y, w[1:nx + 2, 1:ny + 2])
                if fix_snapshot_index:
                    m += 1
        if wn.flags.f_contiguous:
            h.download(wn)
        else:
            wn[...] = h.download()
    return np.array(wn[1:nx + 2, 1:ny + 2], order="F")


def setup(nx=128, ny=128, dt=0.01, tf=20.0, re=1000.0, ns=10):
    """vm.jl:93-128: grid on [0, 2π]², x[i] = Δx(i-1), IC + ghost fill."""
    x_l, x_r = 0.0, 2 * math.pi
    y_b, y_t = 0.0, 2 * math.pi
    dx = (x_r - x_l) / nx
    dy = (y_t - y_b) / ny
    nt = int(tf / dt)
    x = dx * np.arange(nx + 1, dtype=np.float64)
    y = dy * np.arange(ny + 1, dtype=np.float64)
    wn = np.empty((nx + 2, ny + 2), dtype=np.float64, order="F")
    vm_ic(nx, ny, x, y, wn)
    # vm.jl:121-128 (this order: rows/cols 1 first, then nx+2/ny+2)
    wn[0, :] = wn[nx, :]
    wn[:, 0] = wn[:, ny]
    wn[nx + 1, :] = wn[1, :]
    wn[:, ny + 1] = wn[:, 1]
    return dict(nx=nx, ny=ny, nt=nt, dx=dx, dy=dy, dt=dt, re=re, x=x, y=y, wn=wn, ns=ns)


def main(nx=128, ny=128, dt=0.01, tf=20.0, re=1000.0, ns=10, outdir=".", snapshots=True):
    """vm.jl:93-148: writes vm0.txt, runs `numerical`, writes field_final.txt."""
    c = setup(nx, ny, dt, tf, re, ns)
    _write_field(os.path.join(outdir, "vm0.txt"), c["x"], c["y"], c["wn"][1:nx + 2, 1:ny + 2])
    un = numerical(c["nx"], c["ny"], c["nt"], c["dx"], c["dy"], c["dt"], c["re"], c["x"],
                   c["y"], c["wn"], c["ns"], snapshots=snapshots, outdir=outdir)
    _write_field(os.path.join(outdir, "field_final.txt"), c["x"], c["y"], un)
    return un


__all__ = ["numerical", "setup", "main", "periodic_ghosts"]
