"""Sweep the stage kernel's rows-per-wavefront at a grid size, interleaved rounds in one
process (per-kernel HIP-event timing through cfdj_vm_timing).

  python tools/tune_stage.py [--nx 4096] [--rounds 3] [--steps 10] [--rpw 4,8,16,32,64]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from cfd_julia_amd import VortexMerger  # noqa: E402
from cfd_julia_amd.common import vm_ic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rpw", default="4,8,16,32,64")
    a = ap.parse_args()
    nx = a.nx
    dx = 2 * math.pi / nx
    h = VortexMerger(nx, nx, dx, dx, 1000.0)
    x = dx * np.arange(nx + 1)
    wn = np.empty((nx + 2, nx + 2), order="F")
    vm_ic(nx, nx, x, x, wn)
    h.upload(wn)
    dt = 5e-4 * (4096.0 / nx) ** 2
    h.step(dt, 2)
    res = {}
    for _ in range(a.rounds):
        for rpw in [int(v) for v in a.rpw.split(",")]:
            h.set_rows_per_wave(rpw)
            h.set_timing(True)
            h.step(dt, a.steps)
            t = h.timing()
            h.set_timing(False)
            ms, n = t["stage"]
            res.setdefault(rpw, []).append(ms * 1e3 / n)
    cells = nx * nx
    out = {}
    for rpw, us in res.items():
        best = min(us)
        out[rpw] = {"us_min": round(best, 2), "us_med": round(float(np.median(us)), 2),
                    "GBs_88B": round(88 / 3 * cells / (best * 1e-6) / 1e9, 1)}
    print(json.dumps({"nx": nx, "stage_kernel": out}))
    h.close()


if __name__ == "__main__":
    main()
