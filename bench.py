#!/usr/bin/env python3
"""Benchmark of the reference hot path: the vortex-merger SSP-RK3 step
(19_NS2D_Vortex_Merger/vm.jl:12-90 + Common.jl:97-182) on MI355X through libcfdj.so.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

One "step" = one full RK3 step (3 RHS evaluations = 3 FFT Poisson solves + 3 fused
Arakawa/Laplacian/RK stage kernels) over the whole grid, all data resident in HBM.
N = 1 runs BASELINE.json config 3 (4096^2, re = 1000, dt = 5e-4: the reference's dt = .01
is unstable at this size).  N > 1 runs, by default, BASELINE.json config 5: the 8192^2 grid
as N y-slabs (total work fixed for N = 2, 4, 8: "scaling": "strong"; 1024 rows per rank at
N = 8).  Other ladders:
  --strong NX   fixed NX^2 grid at any N (the north star's 4096^2 at 1/2/4/8 GPUs);
  --weak        16.8 M cells per GPU at every N on power-of-two grids (hand-written FFT
                passes): 4096^2, 8192x4096, 8192^2, 16384x8192 at N = 1, 2, 4, 8;
  --weak-square 4096^2 / 5760^2 / 8192^2 / 11520^2 (16.6-16.8 M cells per GPU; the
                non-power-of-two grids run rocFFT rows/columns + all-to-all transposes).
Each RK3 stage on square power-of-two slabs: RCCL halo rows + the substructured Poisson
solve (two all-gathers of O(nx) numbers) -- no spectrum transpose; rectangular and other
grids transpose the half spectrum with ncclAllToAll.

Rehearsals on one GPU (not the headline): --virtual P runs the y-slab code with P virtual
ranks (device copies for the transposes); --dist runs the RCCL slab code with a one-rank
communicator (CFDJ_FORCE_SLAB=1).

Rank 0 prints ONE JSON line (metric / value = whole-job MLUPS, roofline of the fused stage
kernel from live HIP-event timing, cpu_baseline = the NumPy oracle on this host).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MLUPS (cell-updates/s) + achieved HBM GB/s, 4096² vortex-merger RK3 step"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# Algorithmic HBM bytes per cell: stage kernels 24 + 32 + 32 per step,
# Poisson 32 per solve (D2Z read 8 + write ~8, Z2D read ~8 + write 8; divide fused).
STAGE_BYTES_PER_CELL_STEP = 24 + 32 + 32
STEP_BYTES_PER_CELL = 184
# per-kernel algorithmic bytes per cell for cfdj_vm_kernel_bench ids:
# stages read w (+ wn) and psi and write the stage output; each fused Poisson pass reads
# and writes 8 B per cell (real field or half spectrum)
KB_BYTES_PER_CELL = {1: 24, 2: 32, 3: 32, 4: 16, 5: 16, 6: 16}
KB_LAUNCHES = 20
# Grid ladders (nx, ny) per GPU count; the second field of each value is the `scaling` label
# of the runs at N > 1.  "c5" (default): BASELINE config 3 at N = 1, config 5 (8192^2) on
# N = 2, 4, 8 slabs -- total work fixed over N > 1.  "weak": 16.8 M cells per GPU on
# power-of-two grids (ny <= nx: the reference aliases ky = kx).  "weak-square": constant
# cells on square grids, 5760^2 and 11520^2 not being powers of two.
LADDERS = {
    "c5": ({1: (4096, 4096), 2: (8192, 8192), 4: (8192, 8192), 8: (8192, 8192)}, "strong"),
    "weak": ({1: (4096, 4096), 2: (8192, 4096), 4: (8192, 8192), 8: (16384, 8192)}, "weak"),
    "weak-square": ({1: (4096, 4096), 2: (5760, 5760), 4: (8192, 8192), 8: (11520, 11520)},
                    "weak"),
}


def grid_for(n_gpus, ladder="c5", nx=None, ny=None, strong=None):
    """-> (nx, ny, scaling label, workload note)."""
    if strong:
        return strong, strong, "strong", f"strong scaling of the {strong}^2 grid"
    if nx:
        return nx, ny or nx, "strong", "grid fixed on the command line"
    table, label = LADDERS[ladder]
    if n_gpus in table:
        g = table[n_gpus]
        note = {"c5": "BASELINE config 3" if n_gpus == 1 else
                      "BASELINE config 5 (8192^2 y-slabs; total work fixed for N > 1)",
                "weak": "weak ladder, 16.8 M cells per GPU, power-of-two grids",
                "weak-square": "weak ladder 4096^2/5760^2/8192^2/11520^2"}[ladder]
        return g[0], g[1], label if n_gpus > 1 else "weak", note
    step = 128 * n_gpus // math.gcd(128, n_gpus)
    n = max(step, int(round(4096 * math.sqrt(n_gpus) / step)) * step)
    return n, n, "weak", "constant cells per GPU (square grid rounded to 128 N)"


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def stable_dt(nx, ny=None):
    # 5e-4 at 4096^2 (RK3 viscous limit 7.39e-4), scaled with 1/(1/dx^2 + 1/dy^2)
    ny = ny or nx
    return 5e-4 * 2.0 * 4096.0 ** 2 / (nx ** 2 + ny ** 2)


def load_pmc(nx):
    """PMC traffic of the stage kernel from the committed rocprofv3 summary
    (tools/pmc_summary.py output, separate --pmc passes, FETCH_SIZE doubled for gfx950)."""
    path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("nx") != nx:
        return None
    return d


def cpu_baseline(nx, ny, steps, workers, warmup=1):
    """The CPU oracle (NumPy + scipy.fft restatement of vm.jl/Common.jl) on this host:
    `warmup` untimed RK3 steps, then `steps` timed ones."""
    from oracle import vm_oracle as vo

    dx, dy, x, y = vo.vm_grid(nx, ny)
    w = vo.vm_ic(nx, ny, x, y)
    dt = stable_dt(nx, ny)
    for _ in range(warmup):
        w = vo.rk3_step(w, dt, dx, dy, 1000.0, workers=workers)
    t0 = time.perf_counter()
    for _ in range(steps):
        w = vo.rk3_step(w, dt, dx, dy, 1000.0, workers=workers)
    t = time.perf_counter() - t0
    return {"value": round(nx * ny * steps / t / 1e6, 4), "unit": "MLUPS", "cores": workers,
            "kind": "port", "s_per_step": round(t / steps, 3),
            "host_cpus": os.cpu_count(), "cpu_model": cpu_model(),
            "sample": f"{warmup} warm-up + {steps} timed RK3 steps of the {nx}x{ny} vortex "
                      f"merger, NumPy oracle (oracle/vm_oracle.py; scipy.fft workers="
                      f"{workers} = this job's CPU share of the host's {os.cpu_count()} "
                      f"logical CPUs, stencil single-threaded NumPy), {t:.1f} s; Julia "
                      f"reference not runnable here"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--nx", type=int, default=None, help="override the grid size")
    ap.add_argument("--ny", type=int, default=None)
    ap.add_argument("--virtual", type=int, default=0,
                    help="one-GPU rehearsal: y-slab code with this many virtual ranks")
    ap.add_argument("--dist", action="store_true",
                    help="one-GPU rehearsal: RCCL slab code with a one-rank communicator")
    ap.add_argument("--poisson", default="auto", choices=["auto", "fused", "rocfft", "schur"])
    ap.add_argument("--rows-per-wave", type=int, default=None)
    ap.add_argument("--ladder", default="c5", choices=sorted(LADDERS),
                    help="grid per GPU count (default: config 3 at N=1, config 5 at N>1)")
    ap.add_argument("--weak", action="store_const", const="weak", dest="ladder")
    ap.add_argument("--weak-square", action="store_const", const="weak-square", dest="ladder")
    ap.add_argument("--strong", type=int, default=None, metavar="NX",
                    help="fixed NX^2 grid at any GPU count (e.g. 4096: the north-star report)")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true",
                    help="do not record per-kernel HIP events in the timed region")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n_gpus = max(world, 1)
    if args.gpus != n_gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # RCCL prints its version banner on stdout at communicator init: send everything the
    # libraries write to fd 1 to stderr, so stdout carries only the one JSON line
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)

    import numpy as np
    import torch
    import torch.distributed as dist

    from cfd_julia_amd import VortexMerger, _lib
    from cfd_julia_amd.common import vm_ic

    _lib.require_gpu()
    torch.cuda.set_device(local_rank)
    if world > 1:
        # host-side coordination only (unique-id broadcast, barriers, max-reduce);
        # the data path (halos, FFT all-to-all) is RCCL inside libcfdj.so
        dist.init_process_group("gloo")

    def barrier():
        if world > 1:
            dist.barrier()

    nx, ny, scaling, ladder_note = grid_for(n_gpus, args.ladder, args.nx, args.ny, args.strong)
    dx, dy = 2 * math.pi / nx, 2 * math.pi / ny
    dt = stable_dt(nx, ny)
    re = 1000.0

    if args.dist:
        os.environ["CFDJ_FORCE_SLAB"] = "1"
    if world > 1 or args.dist:
        uid = VortexMerger.unique_id() if rank == 0 else bytes(128)
        t = torch.frombuffer(bytearray(uid), dtype=torch.uint8)
        if world > 1:
            dist.broadcast(t, src=0)
        h = VortexMerger(nx, ny, dx, dy, re, device=local_rank, kind="dist", nranks=world,
                         rank=rank, nccl_id=bytes(t.numpy().tobytes()))
    elif args.virtual:
        h = VortexMerger(nx, ny, dx, dy, re, device=local_rank, kind="virtual",
                         nranks=args.virtual)
    else:
        h = VortexMerger(nx, ny, dx, dy, re, device=local_rank)
    h.set_poisson(args.poisson)
    if args.rows_per_wave:
        h.set_rows_per_wave(args.rows_per_wave)

    # vm.jl:107-128 IC on the global ghosted grid; each rank evaluates (and uploads) only
    # its own rows -- np.zeros pages stay untouched elsewhere, so host memory is one slab
    x = dx * np.arange(nx + 1)
    y = dy * np.arange(ny + 1)
    row0, rows = h.slab()
    wn = np.zeros((nx + 2, ny + 2), order="F")
    vm_ic(nx, rows - 1, x, y[row0:], wn[:, row0:])  # fills wn[1:nx+2, row0+1:row0+rows+1]
    h.upload(wn)
    del wn

    def timed(instrumented):
        """One timed region of exactly K steps, barrier + device sync on both sides."""
        h.set_timing(instrumented)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h.step_async(dt, args.steps)
        h.sync()
        torch.cuda.synchronize()
        barrier()
        el = time.perf_counter() - t0
        kern = (h.timing(), h.stage_timing()) if instrumented else None
        h.set_timing(False)
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt[0])
        return el, kern

    # warm-up: also captures the HIP graph of K steps that the headline region replays
    h.step(dt, args.warmup)
    h.step_async(dt, args.steps)
    h.sync()
    # (1) headline: graph replay (single-GPU fused path), no instrumentation
    elapsed, _ = timed(False)
    # (2) the same K steps again with HIP events around every kernel on the handle's
    # stream (eager launches: event nodes cannot be captured into graphs on this ROCm)
    if args.no_timing:
        elapsed_i, kern, kern_stage = None, {k: (0.0, 0) for k in _lib.K_NAMES}, [(0.0, 0)] * 3
    else:
        elapsed_i, (kern, kern_stage) = timed(True)

    # sanity: the state stays finite and bounded (conservative scheme)
    h.set_check_finite(True)
    h.sync()
    h.set_check_finite(False)

    # (3) per-kernel roofline: each kernel of the step launched KB_LAUNCHES times back to
    # back between two HIP events on the handle's stream (runs after (1)/(2): it clobbers
    # the stage buffers).  Single-GPU fused path only; slab runs use (2)'s events.
    kb = {}
    if n_gpus == 1 and not args.virtual and not args.dist and h.poisson() == "fused":
        for kid, name in _lib.KB_NAMES.items():
            us = h.kernel_bench(kid, dt, KB_LAUNCHES) * 1e3
            alg = KB_BYTES_PER_CELL[kid] * nx * ny
            kb[name] = {"us_per_launch": round(us, 2), "alg_bytes": alg,
                        "alg_gbs": round(alg / (us * 1e-6) / 1e9, 1),
                        "frac": round(alg / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}

    parallelism = "single" if n_gpus == 1 else f"yslab{n_gpus}"
    if args.virtual:
        parallelism = f"virtual-yslab{args.virtual} (1 GPU rehearsal)"
    elif args.dist and world == 1:
        parallelism = "rccl-yslab1 (1 GPU rehearsal)"
    cells = nx * ny
    value = cells * args.steps / elapsed / 1e6
    ms_step = elapsed * 1e3 / max(args.steps, 1)
    local_cells = cells / n_gpus
    kname = "vm_stage"
    # the row-group form runs where the row length is a multiple of 512, the slab's row count
    # even and no column partial sums are wanted (the substructured y-slab Poisson wants them)
    rows_local = ny // max(n_gpus, args.virtual or 1)
    tile = (nx % 512 == 0 and rows_local % 2 == 0 and h.poisson() != "schur"
            and not args.rows_per_wave)
    stage_kernel = "vm_stage_tile_kernel<1..3>" if tile else "vm_stage_kernel<1..3>"
    # Roofline of the stage kernels from their IN-STEP launch times: HIP events around every
    # stage-kernel launch of the instrumented timed region (the kernels run in the step's
    # own sequence, between the Poisson passes), algorithmic bytes 24 / 32 / 32 per cell
    # The back-to-back microbenchmark figure is kept beside it as frac_isolated.
    alg_cell = (24, 32, 32)
    per_stage = []
    for i, (ms_i, n_i) in enumerate(kern_stage):
        if n_i:
            us_i = ms_i * 1e3 / n_i
            gbs_i = alg_cell[i] * local_cells / (us_i * 1e-6) / 1e9
            per_stage.append({"stage": i + 1, "avg_launch_us": round(us_i, 2),
                              "alg_bytes": int(alg_cell[i] * local_cells),
                              "achieved": round(gbs_i, 1),
                              "frac": round(gbs_i / HBM_PEAK_GBS, 4), "launches": n_i})
    stage_ms, stage_n = kern["stage"]
    stage_us = stage_ms * 1e3 / max(stage_n, 1)
    stage_alg = sum(alg_cell) / 3.0 * local_cells
    source = ("HIP events around every stage-kernel launch on the handle stream, in the "
              "step's own kernel sequence, over a second timed region of the same K steps "
              "(eager launches); mean over the three RK3 stages")
    stage_gbs = stage_alg / (stage_us * 1e-6) / 1e9 if stage_us > 0 else None
    iso = None
    if kb:
        st = [kb[f"{kname}<{i}>"] for i in (1, 2, 3)]
        iso_us = sum(k["us_per_launch"] for k in st) / 3.0
        iso_alg = sum(k["alg_bytes"] for k in st) / 3.0
        iso = iso_alg / (iso_us * 1e-6) / 1e9
    roofline = {
        "kernel": stage_kernel + " (fused Arakawa J + 5-pt Laplacian + RK3 stage)",
        "bound": "hbm",
        "achieved": round(stage_gbs, 1) if stage_gbs else None,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(stage_gbs / HBM_PEAK_GBS, 4) if stage_gbs else None,
        "traffic": None,
        "alg_bytes_per_launch": int(round(stage_alg)),
        "avg_launch_us": round(stage_us, 2),
        "launches": stage_n,
        "per_stage": per_stage,
        "frac_isolated": round(iso / HBM_PEAK_GBS, 4) if iso else None,
        "frac_isolated_source": (f"{KB_LAUNCHES} back-to-back launches of each stage kernel "
                                 f"on identical inputs (cfdj_vm_kernel_bench)") if iso else None,
        "source": source,
    }
    pmc = load_pmc(nx)
    if pmc:
        roofline["traffic"] = pmc["stage_bytes_per_launch"]
        roofline["traffic_source"] = pmc["source"]
    step_gbs = STEP_BYTES_PER_CELL * local_cells * args.steps / elapsed / 1e9
    breakdown = {k: {"ms_per_step": round(v[0] / max(args.steps, 1), 4), "launches": v[1]}
                 for k, v in kern.items() if v[1]}

    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "MLUPS",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: vm_ic two-Gaussian vortex-merger IC (Common.jl:208-219)",
        "config": {"workload": f"NS2D vortex merger {nx}x{ny} periodic, Arakawa + FD-FFT "
                               f"Poisson + SSP-RK3 (vm.jl): {ladder_note}",
                   "nx": nx, "ny": ny, "dt": dt,
                   "re": re, "parallelism": parallelism, "poisson": h.poisson(),
                   "cells_per_gpu": cells // n_gpus},
        "ms_per_step_instrumented": round(elapsed_i * 1e3 / args.steps, 4) if elapsed_i else None,
        "achieved_hbm_gbs_step": round(step_gbs, 1),
        "step_roofline_frac": round(step_gbs / HBM_PEAK_GBS, 4),
        "kernels": breakdown,
        "kernel_bench": kb or None,
        "roofline": roofline,
    }
    if rank == 0 and n_gpus == 1 and not args.no_cpu_baseline and not args.virtual:
        workers = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
                      or os.cpu_count() or 1)
        line["cpu_baseline"] = cpu_baseline(nx, ny, args.cpu_steps, workers, warmup=1)
    if rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    h.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
