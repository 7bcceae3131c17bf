#!/usr/bin/env python3
"""One rank's share of a P-rank y-slab step alone on this GPU (timing rehearsal; see
tools/bench_secondary.py bench_rank_rehearsal), for profiling:

  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d OUT -o t -- \
      python3 tools/solo_run.py --nx 8192 --ranks 8 --steps 3
  python3 tools/timeline.py OUT/t_kernel_trace.csv [OUT/t_memory_copy_trace.csv]
"""
import argparse
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=8192)
    ap.add_argument("--ny", type=int, default=None)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--rpw", type=int, default=0, help="rows per wavefront of the stage kernel")
    ap.add_argument("--all-slabs", action="store_true", help="every slab, not rank 0 alone")
    a = ap.parse_args()
    if not a.all_slabs:
        os.environ["CFDJ_VIRTUAL_SOLO_RANK"] = "0"
    if not a.no_overlap:
        os.environ["CFDJ_VIRTUAL_OVERLAP"] = "1"
    from cfd_julia_amd import VortexMerger
    from cfd_julia_amd.common import vm_ic

    nx, ny = a.nx, a.ny or a.nx
    dx, dy = 2 * math.pi / nx, 2 * math.pi / ny
    dt = 5e-4 * 2.0 * 4096.0 ** 2 / (nx * nx + ny * ny)
    with VortexMerger(nx, ny, dx, dy, 1000.0, kind="virtual", nranks=a.ranks) as h:
        row0, rows = h.slab()
        if a.rpw:
            h.set_rows_per_wave(a.rpw)
        x, y = dx * np.arange(nx + 1), dy * np.arange(ny + 1)
        wn = np.zeros((nx + 2, ny + 2), order="F")
        vm_ic(nx, rows - 1, x, y[row0:], wn[:, row0:])
        h.upload(wn)
        del wn
        h.step(dt, 2)
        t0 = time.perf_counter()
        h.step(dt, a.steps)
        t = time.perf_counter() - t0
        print(f"{nx}x{ny} rank 0 of {a.ranks} ({h.poisson()}) rpw {a.rpw or 'default'}: "
              f"{t * 1e3 / a.steps:.4f} ms/step")


if __name__ == "__main__":
    main()
