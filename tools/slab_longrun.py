#!/usr/bin/env python3
"""Many steps of the y-slab path (P virtual slabs, default schedule) against the single-GPU
path of the same grid: max |difference| relative to max |w| every `--every` steps.
  python3 tools/slab_longrun.py --nx 2048 --ranks 4 --steps 400"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=2048)
    ap.add_argument("--ranks", type=int, default=4)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--every", type=int, default=100)
    a = ap.parse_args()
    from cfd_julia_amd import VortexMerger
    from cfd_julia_amd.common import vm_ic

    n = a.nx
    dx = 2 * math.pi / n
    x = dx * np.arange(n + 1)
    wn = np.zeros((n + 2, n + 2), order="F")
    vm_ic(n, n, x, x, wn)
    dt = 5e-4 * (4096 / n) ** 2
    with VortexMerger(n, n, dx, dx, 1000.0) as h1, \
            VortexMerger(n, n, dx, dx, 1000.0, kind="virtual", nranks=a.ranks) as hp:
        h1.upload(wn)
        hp.upload(wn)
        done = 0
        while done < a.steps:
            k = min(a.every, a.steps - done)
            h1.step(dt, k)
            hp.step(dt, k)
            done += k
            w1, wp = h1.download(), hp.download()
            print(f"step {done:5d} t = {done * dt:.4f}  max|w| = {np.abs(w1).max():.6f}  "
                  f"rel diff = {np.abs(w1 - wp).max() / np.abs(w1).max():.3e}", flush=True)


if __name__ == "__main__":
    main()
