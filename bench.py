#!/usr/bin/env python3
"""Benchmark of the reference hot path: the vortex-merger SSP-RK3 step
(19_NS2D_Vortex_Merger/vm.jl:12-90 + Common.jl:97-182) on MI355X through libcfdj.so.

  python bench.py [--gpus N] [--steps K] [--warmup W]

`--gpus N` with N > 1 and no WORLD_SIZE in the environment starts the N ranks itself: the
parent process (which never touches a GPU) runs
`python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
--master-port P bench.py --gpus N ...` as a child process, relays the child's one JSON line
and exits with its status; it refuses (non-zero, with the reason) when fewer than N GPUs
are visible.  Started under torch.distributed.run (WORLD_SIZE set) it is one rank of that
job.

One "step" = one full RK3 step (3 RHS evaluations = 3 FFT Poisson solves + 3 fused
Arakawa/Laplacian/RK stage kernels) over the whole grid, all data resident in HBM.
N = 1 runs BASELINE.json config 3 (4096^2, re = 1000, dt = 5e-4: the reference's dt = .01
is unstable at this size).  N > 1 runs, by default, BASELINE.json config 5: the 8192^2 grid
as N y-slabs (total work fixed for N = 2, 4, 8: "scaling": "strong"; 1024 rows per rank at
N = 8) as the headline `value`, and -- in the same process group, each with its own warm-up
and timed regions -- the other two ladders of the north star as the `ladders` object: the
4096^2 grid on N GPUs (strong) and 16.8 M cells per GPU (weak), each with its time per step,
MLUPS, communication time per step and its efficiency against the single-GPU 4096^2 run
measured on rank 0's GPU in the same invocation.  Other headline grids:
  --strong NX   fixed NX^2 grid at any N (the north star's 4096^2 at 1/2/4/8 GPUs);
  --weak        16.8 M cells per GPU at every N on power-of-two grids (hand-written FFT
                passes): 4096^2, 8192x4096, 8192^2, 16384x8192 at N = 1, 2, 4, 8;
  --weak-square 4096^2 / 5760^2 / 8192^2 / 11520^2 (16.6-16.8 M cells per GPU; the
                non-power-of-two grids run rocFFT rows/columns + all-to-all transposes).
Each RK3 stage on square power-of-two slabs: RCCL halo rows + the substructured Poisson
solve (two all-gathers of O(nx) numbers) -- no spectrum transpose; rectangular and other
grids transpose the half spectrum with ncclAllToAll.

Every timed region is exactly K steps between barrier + device sync on both sides, max
over ranks; it is repeated `--repeats` times (default 5) and the MEDIAN region gives
`value` / `ms_per_step` (all repeats are listed in `repeat_ms_per_step`).

Rehearsals on one GPU (not the headline): --virtual P runs the y-slab code with P virtual
ranks (device copies for the transposes); --dist runs the RCCL slab code with a one-rank
communicator (CFDJ_FORCE_SLAB=1) and prints the multi-GPU schema (ladders, rccl_ranks).

Rank 0 prints ONE JSON line (metric / value = whole-job MLUPS, roofline of the fused stage
kernel from live HIP-event timing, cpu_baseline = the NumPy oracle on this host).
"""
import argparse
import json
import math
import os
import socket
import statistics
import subprocess
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
RE = 1000.0


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


# ---- launcher: `python bench.py --gpus N` starts its own N ranks ---------------------------
def visible_gpu_count():
    """GPUs this process may use, counted without initialising the HIP runtime."""
    import torch

    return int(torch.cuda.device_count())


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(n_gpus, argv, port):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={n_gpus}", "--master-addr", "127.0.0.1", "--master-port",
            str(port), os.path.abspath(__file__)] + list(argv)


def launch_ranks(n_gpus, argv, device_count=visible_gpu_count, run=subprocess.run,
                 out=None, err=None):
    """Parent side of `bench.py --gpus N` (N > 1, not under torch.distributed.run): start
    the N ranks as a child process, relay the one JSON line, return the exit status.  The
    parent makes no GPU call (a process that has initialised the GPU must not be replaced,
    and the ranks must find the devices untouched)."""
    out = out or sys.stdout
    err = err or sys.stderr
    have = device_count()
    if have < n_gpus:
        err.write(f"bench.py: --gpus {n_gpus} needs {n_gpus} visible GPUs, this node shows "
                  f"{have}: refusing to run a smaller job under that label\n")
        return 2
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = launch_command(n_gpus, argv, free_port())
    err.write("bench.py: starting " + " ".join(cmd) + "\n")
    err.flush()
    r = run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, text=True)
    lines = [ln for ln in (r.stdout or "").splitlines() if ln.strip()]
    json_lines = [ln for ln in lines if ln.lstrip().startswith("{")]
    for ln in lines:
        if ln not in json_lines[-1:]:
            err.write(ln + "\n")
    if r.returncode == 0 and not json_lines:
        err.write("bench.py: the ranks exited 0 without a JSON line\n")
        return 3
    if json_lines:
        out.write(json_lines[-1] + "\n")
        out.flush()
    return r.returncode


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
        w = vo.rk3_step(w, dt, dx, dy, RE, workers=workers)
    t0 = time.perf_counter()
    for _ in range(steps):
        w = vo.rk3_step(w, dt, dx, dy, RE, workers=workers)
    t = time.perf_counter() - t0
    return {"value": round(nx * ny * steps / t / 1e6, 4), "unit": "MLUPS", "cores": workers,
            "kind": "port", "s_per_step": round(t / steps, 3),
            "host_cpus": os.cpu_count(), "cpu_model": cpu_model(),
            "sample": f"{warmup} warm-up + {steps} timed RK3 steps of the {nx}x{ny} vortex "
                      f"merger, NumPy oracle (oracle/vm_oracle.py; scipy.fft workers="
                      f"{workers} = this job's CPU share of the host's {os.cpu_count()} "
                      f"logical CPUs, stencil single-threaded NumPy), {t:.1f} s; Julia "
                      f"reference not runnable here"}


class Job:
    """One rank's view of the run: process group, handle factory, timed regions."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist

        self.args = args
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.n_gpus = max(self.world, 1)
        torch.cuda.set_device(self.local_rank)
        if self.world > 1:
            # host-side coordination only (unique-id broadcast, barriers, max-reduce), on
            # CPU tensors; the data path (halos, all-gathers, all-to-all) is RCCL inside
            # libcfdj.so
            dist.init_process_group("gloo")

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max_over_ranks(self, v):
        if self.world > 1:
            t = self.torch.tensor([v], dtype=self.torch.float64)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
            return float(t[0])
        return v

    def handle(self, nx, ny, kind):
        """kind: "single" | "dist" | "virtual" -> VortexMerger with the vm_ic field loaded."""
        import numpy as np

        from cfd_julia_amd import VortexMerger
        from cfd_julia_amd.common import vm_ic

        dx, dy = 2 * math.pi / nx, 2 * math.pi / ny
        if kind == "dist":
            uid = VortexMerger.unique_id() if self.rank == 0 else bytes(128)
            t = self.torch.frombuffer(bytearray(uid), dtype=self.torch.uint8)
            if self.world > 1:
                self.dist.broadcast(t, src=0)
            h = VortexMerger(nx, ny, dx, dy, RE, device=self.local_rank, kind="dist",
                             nranks=self.world, rank=self.rank,
                             nccl_id=bytes(t.numpy().tobytes()))
        elif kind == "virtual":
            h = VortexMerger(nx, ny, dx, dy, RE, device=self.local_rank, kind="virtual",
                             nranks=self.args.virtual)
        else:
            h = VortexMerger(nx, ny, dx, dy, RE, device=self.local_rank)
        # vm.jl:107-128 IC on the global ghosted grid; each rank evaluates (and uploads) only
        # its own rows -- np.zeros pages stay untouched elsewhere, so host memory is one slab
        x = dx * np.arange(nx + 1)
        y = dy * np.arange(ny + 1)
        row0, rows = h.slab()
        wn = np.zeros((nx + 2, ny + 2), order="F")
        vm_ic(nx, rows - 1, x, y[row0:], wn[:, row0:])  # wn[1:nx+2, row0+1:row0+rows+1]
        h.upload(wn)
        del wn
        return h

    def timed(self, h, dt, steps, instrumented):
        """One timed region of exactly `steps` steps, barrier + device sync on both sides,
        max over ranks."""
        h.set_timing(instrumented)
        self.barrier()
        self.torch.cuda.synchronize()
        t0 = time.perf_counter()
        h.step_async(dt, steps)
        h.sync()
        self.torch.cuda.synchronize()
        self.barrier()
        el = time.perf_counter() - t0
        kern = (h.timing(), h.stage_timing()) if instrumented else None
        h.set_timing(False)
        return self.max_over_ranks(el), kern

    def measure(self, h, nx, ny, instrumented=True):
        """Warm-up, `repeats` timed regions (median reported), one instrumented region."""
        a = self.args
        dt = stable_dt(nx, ny)
        # warm-up: also captures the HIP graph of K steps that the timed regions replay
        h.step(dt, a.warmup)
        h.step_async(dt, a.steps)
        h.sync()
        # (1) headline regions: graph replay (single-GPU fused path), no instrumentation
        regions = [self.timed(h, dt, a.steps, False)[0] for _ in range(max(a.repeats, 1))]
        elapsed = statistics.median(regions)
        # (2) the same K steps again with HIP events around every kernel on the handle's
        # stream (eager launches: event nodes cannot be captured into graphs on this ROCm;
        # on RCCL slabs the instrumented region also runs every exchange on the main stream,
        # so its `comm` time is the un-overlapped cost of the exchanges)
        if instrumented:
            elapsed_i, (kern, kern_stage) = self.timed(h, dt, a.steps, True)
        else:
            from cfd_julia_amd import _lib

            elapsed_i, kern, kern_stage = None, {k: (0.0, 0) for k in _lib.K_NAMES}, [(0.0, 0)] * 3
        # sanity: the state stays finite and bounded (conservative scheme)
        h.set_check_finite(True)
        h.sync()
        h.set_check_finite(False)
        return {"elapsed": elapsed, "regions": regions, "elapsed_i": elapsed_i, "kern": kern,
                "kern_stage": kern_stage, "dt": dt}

    def case(self, nx, ny, kind):
        """One ladder entry: its own handle (and RCCL communicator), warm-up and regions."""
        a = self.args
        h = self.handle(nx, ny, kind)
        try:
            ranks = h.comm_ranks()
            path = h.poisson()
            m = self.measure(h, nx, ny, instrumented=not a.no_timing)
        finally:
            h.close()
        ms = m["elapsed"] * 1e3 / a.steps
        comm_ms, comm_n = m["kern"]["comm"]
        return {"grid": f"{nx}x{ny}", "cells_per_gpu": nx * ny // self.n_gpus,
                "ms_per_step": round(ms, 4),
                "mlups": round(nx * ny * a.steps / m["elapsed"] / 1e6, 2),
                "comm_ms_per_step": round(comm_ms / a.steps, 4) if comm_n else None,
                "ms_per_step_instrumented": (round(m["elapsed_i"] * 1e3 / a.steps, 4)
                                             if m["elapsed_i"] else None),
                "repeat_ms_per_step": [round(r * 1e3 / a.steps, 4) for r in m["regions"]],
                "poisson": path, "rccl_ranks": ranks}

    def multi_rank_parity(self, nx, ny, steps=2):
        """The RCCL y-slab run against the single-GPU path of the same grid, both through
        libcfdj.so (every rank runs the single-GPU path on its own GPU and compares the
        all-gathered field with it): max |difference| over ranks, relative to max |w|."""
        import numpy as np

        dt = stable_dt(nx, ny)
        with self.handle(nx, ny, "single") as h1:
            h1.step(dt, steps)
            ref = h1.download()
        h = self.handle(nx, ny, "dist")
        try:
            h.step(dt, steps)
            got = h.download()
        finally:
            h.close()
        err = float(np.abs(got - ref).max() / np.abs(ref).max())
        del got, ref
        return {"grid": f"{nx}x{ny}", "steps": steps, "linf_rel": self.max_over_ranks(err),
                "against": "single-GPU path of libcfdj.so on every rank's own GPU",
                "tolerance": 1e-10}


FALLBACK_ENV = {"CFDJ_NO_OVERLAP": "1", "CFDJ_SLAB_W_HALO": "exchange",
                "CFDJ_SLAB_PSI_HALO": "exchange", "CFDJ_SLAB_LATE_CS": "0"}


class Watchdog:
    """A rank of a multi-GPU run that makes no progress for `seconds` (a collective whose peer
    never arrives leaves the host blocked inside the library, where no exception can reach)
    writes one JSON line naming the phase it was in and leaves the process with status 3, so a
    hang costs the run its limit instead of the caller's.  `touch(phase)` restarts the clock."""

    def __init__(self, seconds, write, leave=os._exit):
        import threading

        self.seconds, self.write, self.leave = seconds, write, leave
        self.phase, self.timer, self.threading = "start", None, threading
        self.touch("start")

    def touch(self, phase):
        self.phase = phase
        if self.timer is not None:
            self.timer.cancel()
        if self.seconds > 0:
            self.timer = self.threading.Timer(self.seconds, self.expire)
            self.timer.daemon = True
            self.timer.start()

    def expire(self):
        self.write({"error": f"no progress for {self.seconds} s in phase '{self.phase}'",
                    "phase": self.phase})
        self.leave(3)

    def stop(self):
        if self.timer is not None:
            self.timer.cancel()
            self.timer = None


def parity_with_fallback(run_parity, environ=os.environ):
    """The multi-rank field check with the default schedule of the y-slab step (substructured
    path: one all-gather per solve carries everything, psi's halo rows are computed; other
    paths: halo exchanges on a side stream) and, if that one does not meet the tolerance, once
    more with the plainest schedule -- every halo row exchanged, on the one stream
    (FALLBACK_ENV, read by every handle created afterwards: the ladders then run that schedule
    too).  `run_parity` returns the same dictionary on every rank (its error is the maximum
    over ranks), so all ranks take the same branch."""
    first = run_parity()
    first["schedule"] = "default"
    if first["linf_rel"] < first["tolerance"]:
        return first
    environ.update(FALLBACK_ENV)
    second = run_parity()
    second["schedule"] = "fallback: " + " ".join(f"{k}={v}" for k, v in FALLBACK_ENV.items())
    second["first_try"] = {"schedule": first["schedule"], "linf_rel": first["linf_rel"]}
    return second


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--repeats", type=int, default=5,
                    help="timed regions of K steps each; the median is reported")
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
    ap.add_argument("--no-ladders", action="store_true",
                    help="multi-GPU runs: only the headline grid, no strong-4096 / weak entries")
    ap.add_argument("--no-parity", action="store_true",
                    help="multi-GPU runs: skip the slab-vs-single-GPU field comparison")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true",
                    help="do not record per-kernel HIP events in the timed region")
    ap.add_argument("--watchdog", type=float, default=300.0, metavar="SECONDS",
                    help="multi-GPU runs: give up (status 3, one JSON error line) when a phase "
                         "makes no progress for this long; 0 = never")
    args = ap.parse_args(argv)
    if args.gpus < 1 or args.steps < 1:
        raise SystemExit("--gpus and --steps must be >= 1")

    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        # not under torch.distributed.run: start the ranks (before any GPU call)
        raise SystemExit(launch_ranks(args.gpus, argv))
    world = int(world_env or "1")
    if args.gpus != max(world, 1):
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # RCCL prints its version banner on stdout at communicator init: send everything the
    # libraries write to fd 1 to stderr, so stdout carries only the one JSON line
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    rank_env = int(os.environ.get("RANK", "0"))

    def watchdog_line(d):
        d = dict(d, rank=rank_env, n_gpus=args.gpus)
        sys.stderr.write(f"bench.py watchdog: {d}\n")
        sys.stderr.flush()
        if rank_env == 0:
            os.write(json_fd, (json.dumps(d) + "\n").encode())

    dog = Watchdog(args.watchdog if world > 1 else 0.0, watchdog_line)

    # torch first: its HIP runtime must be the one in the process before libcfdj.so loads
    import torch  # noqa: F401

    from cfd_julia_amd import _lib

    _lib.require_gpu()
    if args.dist:
        os.environ["CFDJ_FORCE_SLAB"] = "1"
    job = Job(args)
    rank, n_gpus = job.rank, job.n_gpus
    multi = world > 1 or args.dist
    kind = "dist" if multi else "virtual" if args.virtual else "single"

    nx, ny, scaling, ladder_note = grid_for(n_gpus, args.ladder, args.nx, args.ny, args.strong)

    ladders = None
    parity = None
    if multi:
        # the single-GPU reference of the efficiencies: BASELINE config 3 on rank 0's GPU
        # (every rank runs it on its own GPU at the same time; rank 0's figure is used)
        ladders = {}
        if not args.no_ladders:
            dog.touch("single-GPU reference 4096x4096")
            h1 = job.handle(4096, 4096, "single")
            try:
                m1 = job.measure(h1, 4096, 4096, instrumented=False)
            finally:
                h1.close()
            n1_mlups = 4096 * 4096 * args.steps / m1["elapsed"] / 1e6
            ladders["n1_reference"] = {
                "grid": "4096x4096", "ms_per_step": round(m1["elapsed"] * 1e3 / args.steps, 4),
                "mlups": round(n1_mlups, 2),
                "note": "single-GPU path, measured on the ranks' own GPUs in this invocation "
                        "(max over ranks)"}
        if not args.no_parity:
            dog.touch(f"multi-rank parity {nx}x{ny}")
            parity = parity_with_fallback(lambda: job.multi_rank_parity(nx, ny))

    dog.touch(f"headline {nx}x{ny}")
    h = job.handle(nx, ny, kind)
    h.set_poisson(args.poisson)
    if args.rows_per_wave:
        h.set_rows_per_wave(args.rows_per_wave)
    rccl_ranks = h.comm_ranks()
    if multi and rccl_ranks != n_gpus:
        raise SystemExit(f"RCCL reports {rccl_ranks} ranks, the job has {n_gpus}")
    m = job.measure(h, nx, ny, instrumented=not args.no_timing)
    elapsed, elapsed_i, kern, kern_stage, dt = (m["elapsed"], m["elapsed_i"], m["kern"],
                                                m["kern_stage"], m["dt"])

    # (3) per-kernel roofline: each kernel of the step launched KB_LAUNCHES times back to
    # back between two HIP events on the handle's stream (runs after (1)/(2): it clobbers
    # the stage buffers).  Single-GPU fused path only; slab runs use (2)'s events.
    kb = {}
    if kind == "single" and h.poisson() == "fused":
        for kid, name in _lib.KB_NAMES.items():
            us = h.kernel_bench(kid, dt, KB_LAUNCHES) * 1e3
            alg = KB_BYTES_PER_CELL[kid] * nx * ny
            kb[name] = {"us_per_launch": round(us, 2), "alg_bytes": alg,
                        "alg_gbs": round(alg / (us * 1e-6) / 1e9, 1),
                        "frac": round(alg / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
    poisson_path = h.poisson()
    stage_tile = h.stage_row_group()
    h.close()

    parallelism = "single" if n_gpus == 1 else f"yslab{n_gpus}"
    if args.virtual:
        parallelism = f"virtual-yslab{args.virtual} (1 GPU rehearsal)"
    elif args.dist and world == 1:
        parallelism = "rccl-yslab1 (1 GPU rehearsal)"
    cells = nx * ny
    value = cells * args.steps / elapsed / 1e6
    ms_step = elapsed * 1e3 / args.steps
    local_cells = cells / n_gpus
    # cells one stage-kernel launch covers: a slab (virtual slabs: one launch per slab)
    launch_cells = local_cells / max(args.virtual, 1)
    kname = "vm_stage"
    stage_kernel = ("vm_stage_tile_kernel<1..3>" if stage_tile else
                    "vm_stage_tall_kernel / vm_stage_kernel<1..3>" if kind != "single" else
                    "vm_stage_kernel<1..3>")
    # Roofline of the stage kernels from their IN-STEP launch times: HIP events around every
    # stage-kernel launch of the instrumented timed region (the kernels run in the step's
    # own sequence, between the Poisson passes), algorithmic bytes 24 / 32 / 32 per cell
    # The back-to-back microbenchmark figure is kept beside it as frac_isolated.
    alg_cell = (24, 32, 32)
    per_stage = []
    for i, (ms_i, n_i) in enumerate(kern_stage):
        if n_i:
            us_i = ms_i * 1e3 / n_i
            gbs_i = alg_cell[i] * launch_cells / (us_i * 1e-6) / 1e9
            per_stage.append({"stage": i + 1, "avg_launch_us": round(us_i, 2),
                              "alg_bytes": int(alg_cell[i] * launch_cells),
                              "achieved": round(gbs_i, 1),
                              "frac": round(gbs_i / HBM_PEAK_GBS, 4), "launches": n_i})
    stage_ms, stage_n = kern["stage"]
    stage_us = stage_ms * 1e3 / max(stage_n, 1)
    stage_alg = sum(alg_cell) / 3.0 * launch_cells
    source = ("HIP events around every stage-kernel launch on the handle stream, in the "
              "step's own kernel sequence, over one more timed region of the same K steps "
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
    pmc = load_pmc(nx) if kind == "single" else None
    if pmc:
        roofline["traffic"] = pmc["stage_bytes_per_launch"]
        roofline["traffic_source"] = pmc["source"]
    step_gbs = STEP_BYTES_PER_CELL * local_cells * args.steps / elapsed / 1e9
    breakdown = {k: {"ms_per_step": round(v[0] / args.steps, 4), "launches": v[1]}
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
                   "re": RE, "parallelism": parallelism, "poisson": poisson_path,
                   "cells_per_gpu": cells // n_gpus},
        "repeats": len(m["regions"]),
        "repeat_ms_per_step": [round(r * 1e3 / args.steps, 4) for r in m["regions"]],
        "timing_rule": "median of `repeats` timed regions of exactly K steps each (barrier + "
                       "device sync on both sides, max over ranks)",
        "ms_per_step_instrumented": round(elapsed_i * 1e3 / args.steps, 4) if elapsed_i else None,
        "achieved_hbm_gbs_step": round(step_gbs, 1),
        "step_roofline_frac": round(step_gbs / HBM_PEAK_GBS, 4),
        "kernels": breakdown,
        "kernel_bench": kb or None,
        "roofline": roofline,
    }
    if multi:
        line["rccl_ranks"] = rccl_ranks
        comm_ms, comm_n = kern["comm"]
        head = {"grid": f"{nx}x{ny}", "cells_per_gpu": cells // n_gpus,
                "ms_per_step": round(ms_step, 4), "mlups": round(value, 2),
                "comm_ms_per_step": round(comm_ms / args.steps, 4) if comm_n else None,
                "poisson": poisson_path, "rccl_ranks": rccl_ranks}
        ladders["headline"] = head
        if not args.no_ladders:
            sx, sy, _, _ = grid_for(n_gpus, strong=4096)
            wx, wy, _, _ = grid_for(n_gpus, "weak")
            rungs = [("c5_8192", (8192, 8192)), ("strong_4096", (sx, sy)), ("weak", (wx, wy))]
            if n_gpus in (4, 8):
                # aggregate-throughput rung: the largest square grid of the substructured path
                # (67 / 33.5 M cells per GPU at N = 4 / 8 -- more work per GPU than n1's)
                rungs.append(("square_16384", (16384, 16384)))
            for key, (gx, gy) in rungs:
                if (gx, gy) == (nx, ny) and args.poisson == "auto" and not args.rows_per_wave:
                    entry = dict(head)
                else:
                    dog.touch(f"ladder {key} {gx}x{gy}")
                    entry = job.case(gx, gy, "dist")
                entry["efficiency_vs_n1"] = round(
                    entry["mlups"] / (n_gpus * ladders["n1_reference"]["mlups"]), 4)
                ladders[key] = entry
            ladders["efficiency_rule"] = ("mlups / (n_gpus x n1_reference.mlups): strong "
                                          "ladders at fixed total work, weak at fixed work "
                                          "per GPU, square_16384 at 2-4x n1's work per GPU")
        line["ladders"] = ladders
        line["multi_rank_parity"] = parity
        if parity and not parity["linf_rel"] < parity["tolerance"]:
            line["error"] = "multi-rank field differs from the single-GPU path"
    if rank == 0 and n_gpus == 1 and not args.no_cpu_baseline and not args.virtual:
        workers = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
                      or os.cpu_count() or 1)
        line["cpu_baseline"] = cpu_baseline(nx, ny, args.cpu_steps, workers, warmup=1)
    dog.stop()
    if rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    if world > 1:
        job.dist.destroy_process_group()
    if line.get("error"):
        raise SystemExit(line["error"])


if __name__ == "__main__":
    main()
