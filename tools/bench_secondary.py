"""Secondary BASELINE configs (not the headline bench line):

  C2  2D FFT Poisson (12/fft_p.jl) 2048^2 periodic: GPU solve time (device-resident, fused
      3-pass path) vs the CPU oracle (scipy.fft, all host cores), with the MMS L2 error.
  C4  lid-driven cavity (18/lid_driven_cavity.jl) 2048^2, re = 100, dt = 5e-6: ms per RK3
      step with the DST-I (fused FFT on the 4096^2 odd extension) and the V-cycle MG solver.
  S   spectral solvers (20/hybrid.jl, 21/22 pseudospectral) at 1024^2 and 4096^2: ms per
      RK3-CN step, MLUPS.
  Y   the multi-GPU y-slab code on one GPU (--virtual P): per-rank ms per step at the
      weak-scaling grids, i.e. the compute of one rank of an N-GPU run without the RCCL
      latency (8192^2 / P = 2, 4, 8 -- P = 8 is BASELINE config 5; 16384^2 / P = 8).

  python tools/bench_secondary.py [--steps 20]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def bench_poisson(n=2048, reps=20):
    import torch

    from cfd_julia_amd import PoissonFFT, fft_p
    from oracle import vm_oracle as vo

    f, ue, dx, dy = fft_p.mms(n)
    out = {"config": f"C2 fft_p {n}^2"}
    with PoissonFFT(n, n, dx, dy) as h:
        fd = torch.tensor(np.ascontiguousarray(f[:n, :n].T), dtype=torch.float64, device="cuda")
        sd = torch.empty_like(fd)
        for path in ("fused", "rocfft"):
            h.set_poisson(path)
            h.solve_device(fd.data_ptr(), sd.data_ptr())
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                h.solve_device(fd.data_ptr(), sd.data_ptr())
            torch.cuda.synchronize()
            out[f"gpu_{path}_ms"] = round((time.perf_counter() - t0) * 1e3 / reps, 4)
        un = np.zeros_like(f)
        un[:n, :n] = sd.cpu().numpy().T
    un[n, :] = un[0, :]
    un[:, n] = un[:, 0]
    out["l2_error"] = float(np.sqrt(np.mean((un - ue) ** 2)))
    workers = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    t0 = time.perf_counter()
    vo.ps_fft(np.ascontiguousarray(f[:n, :n]), dx, dy, workers=workers)
    out["cpu_oracle_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    out["cpu_workers"] = workers
    return out


def bench_cavity(n=2048, steps=20, dt=5e-6):
    from cfd_julia_amd.cavity import Cavity

    out = {"config": f"C4 cavity {n}^2 re=100 dt={dt}"}
    dx = 1.0 / n
    for p in ("dst", "mg"):
        with Cavity(n, n, dx, dx, 100.0, poisson=p, tol=1e-6) as h:
            h.step(dt, 2)
            k = steps if p == "mg" else max(steps, 100)  # a DST step is 0.3 ms: time 30 ms
            t0 = time.perf_counter()
            rms = h.step(dt, k)
            t = time.perf_counter() - t0
            out[f"{p}_steps"] = k
            out[f"{p}_ms_per_step"] = round(t * 1e3 / k, 3)
            out[f"{p}_MLUPS"] = round(n * n * k / t / 1e6, 1)
            out[f"{p}_final_rms"] = float(rms[-1])
            if p == "mg":
                out["mg_vcycles_total"] = int(h.mg_iterations())
    return out


def bench_spectral(steps=5):
    import math

    from cfd_julia_amd.spectral import SpectralNS2D
    from cfd_julia_amd.common import vm_ic

    out = []
    for n in (1024, 4096):
        dx = 2 * math.pi / n
        x = dx * np.arange(n + 1)
        wn = np.zeros((n + 2, n + 2), order="F")
        vm_ic(n, n, x, x, wn)
        for kind in ("hybrid", "2/3", "3/2"):
            k = steps if n > 1024 else 8 * steps
            with SpectralNS2D(n, n, dx, dx, 1000.0, kind) as h:
                h.upload(wn)
                h.step(1e-4, 2)  # also captures the step's graph where it has one
                t0 = time.perf_counter()
                h.step(1e-4, k)
                t = time.perf_counter() - t0
            out.append({"config": f"S {kind} {n}^2", "steps": k,
                        "ms_per_step": round(t * 1e3 / k, 3),
                        "MLUPS": round(n * n * k / t / 1e6, 1)})
    return out


def bench_slabs(steps=3):
    import math

    from cfd_julia_amd import VortexMerger
    from cfd_julia_amd.common import vm_ic

    out = []
    for n, P in ((8192, 2), (8192, 4), (8192, 8), (16384, 8)):
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
            h.step(dt, steps)
            t = time.perf_counter() - t0
            out.append({"config": f"Y {n}^2 virtual {P} slabs ({h.poisson()})",
                        "ms_per_step_all_slabs": round(t * 1e3 / steps, 3),
                        "ms_per_step_per_rank": round(t * 1e3 / steps / P, 3),
                        "cells_per_rank": n * n // P})
    return out


def bench_rank_rehearsal(steps=20, single_ms=None):
    """One rank's compute of an N-rank y-slab step, alone on this GPU (CFDJ_VIRTUAL_SOLO_RANK:
    rank 0's slab only, every exchange a device copy from itself), launched in the RCCL ranks'
    own schedule (CFDJ_VIRTUAL_OVERLAP=1: exchanges and the packed column's solve on side
    streams).  The field is not the global solution -- a timing rehearsal.  `rate_vs_single` =
    the single-GPU path's time per cell (4096^2, measured here) / this rank's time per cell."""
    import math

    from cfd_julia_amd import VortexMerger
    from cfd_julia_amd.common import vm_ic

    def run(nx, ny, P, solo, overlap):
        dx, dy = 2 * math.pi / nx, 2 * math.pi / ny
        dt = 5e-4 * 2.0 * 4096.0 ** 2 / (nx * nx + ny * ny)
        os.environ.pop("CFDJ_VIRTUAL_SOLO_RANK", None)
        os.environ.pop("CFDJ_VIRTUAL_OVERLAP", None)
        if solo:
            os.environ["CFDJ_VIRTUAL_SOLO_RANK"] = "0"
        if overlap:
            os.environ["CFDJ_VIRTUAL_OVERLAP"] = "1"
        kw = dict(kind="virtual", nranks=P) if P else {}
        with VortexMerger(nx, ny, dx, dy, 1000.0, **kw) as h:
            row0, rows = h.slab()
            x, y = dx * np.arange(nx + 1), dy * np.arange(ny + 1)
            wn = np.zeros((nx + 2, ny + 2), order="F")
            vm_ic(nx, rows - 1, x, y[row0:], wn[:, row0:])
            h.upload(wn)
            del wn
            h.step(dt, 3)
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                h.step(dt, steps)
                ts.append((time.perf_counter() - t0) / steps)
            path = h.poisson()
        os.environ.pop("CFDJ_VIRTUAL_SOLO_RANK", None)
        os.environ.pop("CFDJ_VIRTUAL_OVERLAP", None)
        return sorted(ts)[len(ts) // 2] * 1e3, path

    out = []
    if single_ms is None:
        single_ms, _ = run(4096, 4096, 0, False, False)
    per_cell = single_ms / (4096 * 4096)
    out.append({"config": "R single-GPU path 4096^2", "ms_per_step": round(single_ms, 4)})
    for ladder, nx, ny, P in (("strong 4096^2", 4096, 4096, 2), ("strong 4096^2", 4096, 4096, 4),
                              ("strong 4096^2", 4096, 4096, 8),
                              ("config 5 8192^2", 8192, 8192, 2), ("config 5 8192^2", 8192, 8192, 4),
                              ("config 5 8192^2", 8192, 8192, 8),
                              ("weak", 8192, 4096, 2), ("weak", 16384, 8192, 8),
                              ("square 16384^2", 16384, 16384, 8),
                              ("square 16384^2", 16384, 16384, 4)):
        ms, path = run(nx, ny, P, True, True)
        cells = nx * ny // P
        out.append({"config": f"R {ladder}: rank 0 of {P}, {nx}x{ny} ({path})",
                    "cells_per_rank": cells, "ms_per_step": round(ms, 4),
                    "rate_vs_single": round(per_cell * cells / ms, 3)})
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--only", default="poisson,cavity,spectral,slabs,ranks",
                    help="comma-separated sections: poisson, cavity, spectral, slabs, ranks")
    a = ap.parse_args()
    only = set(a.only.split(","))
    if "poisson" in only:
        print(json.dumps(bench_poisson()), flush=True)
    if "cavity" in only:
        print(json.dumps(bench_cavity(steps=a.steps)), flush=True)
    if "spectral" in only:
        for r in bench_spectral():
            print(json.dumps(r), flush=True)
    if "slabs" in only:
        for r in bench_slabs():
            print(json.dumps(r), flush=True)
    if "ranks" in only:
        for r in bench_rank_rehearsal(steps=a.steps):
            print(json.dumps(r), flush=True)
