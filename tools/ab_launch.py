"""A/B of launch modes at 4096^2 in one process: eager vs HIP graph, timing events on/off.
  python tools/ab_launch.py [--nx 4096] [--steps 20] [--rounds 3]"""
import argparse, json, math, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from cfd_julia_amd import VortexMerger
from cfd_julia_amd.common import vm_ic

ap = argparse.ArgumentParser()
ap.add_argument("--nx", type=int, default=4096)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
nx = a.nx; dx = 2 * math.pi / nx; dt = 5e-4 * (4096 / nx) ** 2
h = VortexMerger(nx, nx, dx, dx, 1000.0)
x = dx * np.arange(nx + 1); wn = np.empty((nx + 2, nx + 2), order="F"); vm_ic(nx, nx, x, x, wn)
h.upload(wn)
res = {}
for _ in range(a.rounds):
    for graph in (False, True):
        for timing in (False, True):
            h.set_graph(graph); h.set_timing(timing)
            h.step(dt, a.steps)  # capture / warm
            h.set_timing(timing)
            t0 = time.perf_counter(); h.step(dt, a.steps); t = time.perf_counter() - t0
            k = f"graph={graph},timing={timing}"
            res.setdefault(k, []).append(t * 1e3 / a.steps)
            if timing:
                tm = h.timing()
                res.setdefault(k + ",kernel_sum", []).append(sum(v[0] for v in tm.values()) / a.steps)
print(json.dumps({k: round(min(v), 4) for k, v in res.items()}))
