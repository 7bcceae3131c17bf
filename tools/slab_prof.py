"""One short virtual-slab run for rocprofv3: python tools/slab_prof.py [n] [P]."""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from cfd_julia_amd import VortexMerger  # noqa: E402
from cfd_julia_amd.common import vm_ic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
P = int(sys.argv[2]) if len(sys.argv) > 2 else 8
dx = 2 * math.pi / n
dt = 5e-4 * 2.0 * 4096.0 ** 2 / (2 * n * n)
with VortexMerger(n, n, dx, dx, 1000.0, kind="virtual", nranks=P) as h:
    x = dx * np.arange(n + 1)
    wn = np.zeros((n + 2, n + 2), order="F")
    vm_ic(n, n, x, x, wn)
    h.upload(wn)
    del wn
    h.step(dt, 1)
    t0 = time.perf_counter()
    h.step(dt, 3)
    t = (time.perf_counter() - t0) / 3
    print(f"{n}^2 / {P} slabs ({h.poisson()}): {t * 1e3:.3f} ms per step, "
          f"{t * 1e3 / P:.3f} per rank")
