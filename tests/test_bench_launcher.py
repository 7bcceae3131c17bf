"""`bench.py --gpus N` starts its own N ranks (CPU tests of the parent side; no GPU call).

The parent must: refuse when fewer than N GPUs are visible (non-zero status, reason on
stderr, nothing on stdout), otherwise run `python -m torch.distributed.run ... bench.py
--gpus N ...` as a CHILD process (never replace itself), relay exactly the child's last JSON
line on stdout and return the child's exit status.
"""
import io
import json
import os
import subprocess
import sys
import types

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class StubRun:
    def __init__(self, stdout, returncode=0):
        self.stdout, self.returncode, self.calls = stdout, returncode, []

    def __call__(self, cmd, **kw):
        self.calls.append((cmd, kw))
        return types.SimpleNamespace(stdout=self.stdout, returncode=self.returncode)


def test_launcher_refuses_without_enough_gpus():
    out, err = io.StringIO(), io.StringIO()
    run = StubRun("")
    rc = bench.launch_ranks(8, ["--gpus", "8"], device_count=lambda: 1, run=run, out=out,
                            err=err)
    assert rc != 0 and not run.calls and out.getvalue() == ""
    assert "needs 8 visible GPUs" in err.getvalue() and "shows 1" in err.getvalue()


def test_launcher_starts_torch_distributed_run_and_relays_one_line():
    line = json.dumps({"metric": "m", "value": 1.0, "n_gpus": 4, "rccl_ranks": 4})
    run = StubRun("RCCL banner\n" + json.dumps({"not": "the last"}) + "\n" + line + "\n")
    out, err = io.StringIO(), io.StringIO()
    argv = ["--gpus", "4", "--steps", "7", "--warmup", "2"]
    rc = bench.launch_ranks(4, argv, device_count=lambda: 8, run=run, out=out, err=err)
    assert rc == 0
    assert out.getvalue() == line + "\n"          # exactly one line on stdout
    assert "RCCL banner" in err.getvalue()        # everything else goes to stderr
    (cmd, kw), = run.calls
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert 0 < int(cmd[cmd.index("--master-port") + 1]) < 65536
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv                    # the ranks get the same arguments
    assert kw["env"].get("HSA_ENABLE_IPC_MODE_LEGACY") == "0"
    assert "WORLD_SIZE" not in kw["env"] or kw["env"]["WORLD_SIZE"] == os.environ.get("WORLD_SIZE")


def test_launcher_returns_the_ranks_status():
    out, err = io.StringIO(), io.StringIO()
    rc = bench.launch_ranks(2, ["--gpus", "2"], device_count=lambda: 2,
                            run=StubRun("rank 1 died\n", returncode=17), out=out, err=err)
    assert rc == 17 and out.getvalue() == ""
    rc = bench.launch_ranks(2, ["--gpus", "2"], device_count=lambda: 2,
                            run=StubRun("no json here\n", returncode=0), out=out, err=err)
    assert rc != 0                                # success without a line is a failure


def test_grid_ladders_are_the_north_star_grids():
    assert bench.grid_for(1)[:3] == (4096, 4096, "weak")
    for n in (2, 4, 8):
        assert bench.grid_for(n)[:3] == (8192, 8192, "strong")          # BASELINE config 5
        assert bench.grid_for(n, strong=4096)[:3] == (4096, 4096, "strong")
        nx, ny, label, _ = bench.grid_for(n, "weak")
        assert nx * ny == n * 4096 * 4096 and label == "weak" and ny <= nx


def test_gpus_2_without_two_gpus_exits_nonzero_with_the_reason():
    """The real entry point, in a fresh process: this container shows no GPU (a one-GPU box
    shows one), so `--gpus 2` must fail before any rank starts."""
    import pytest
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("a multi-GPU node would really start the job")
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and r.stdout.strip() == ""
    assert "needs 2 visible GPUs" in r.stderr


def test_parity_falls_back_to_the_single_stream_schedule():
    """bench.parity_with_fallback: a multi-rank field check that fails under the default
    schedule is repeated with the plainest one (bench.FALLBACK_ENV, which the handles created
    afterwards read); a passing first check leaves the environment alone."""
    import bench

    env = {}
    ok = bench.parity_with_fallback(lambda: {"linf_rel": 3e-16, "tolerance": 1e-10}, env)
    assert ok["schedule"] == "default" and not env
    results = iter([{"linf_rel": 2e-3, "tolerance": 1e-10}, {"linf_rel": 4e-16, "tolerance": 1e-10}])
    got = bench.parity_with_fallback(lambda: next(results), env)
    assert env == {"CFDJ_NO_OVERLAP": "1", "CFDJ_SLAB_W_HALO": "exchange",
                   "CFDJ_SLAB_PSI_HALO": "exchange", "CFDJ_SLAB_LATE_CS": "0"}
    assert got["schedule"].startswith("fallback: CFDJ_NO_OVERLAP=1") and got["linf_rel"] == 4e-16
    assert got["first_try"] == {"schedule": "default", "linf_rel": 2e-3}
    # not-a-number counts as a failure, and a second failure is reported as it is
    env2 = {}
    results = iter([{"linf_rel": float("nan"), "tolerance": 1e-10}, {"linf_rel": 1.0, "tolerance": 1e-10}])
    bad = bench.parity_with_fallback(lambda: next(results), env2)
    assert env2 == bench.FALLBACK_ENV and bad["linf_rel"] == 1.0


def test_watchdog_reports_the_stalled_phase():
    """bench.Watchdog: no progress for its limit -> one error line naming the phase, status 3;
    touch() restarts the clock, stop() disarms it, a limit of 0 never fires."""
    import time

    import bench

    lines, codes = [], []
    dog = bench.Watchdog(0.2, lines.append, codes.append)
    dog.touch("headline 8192x8192")
    time.sleep(0.1)
    dog.touch("ladder weak")
    time.sleep(0.1)
    assert not lines and not codes  # touched in time
    time.sleep(0.3)
    assert codes == [3] and lines[0]["phase"] == "ladder weak" and "no progress" in lines[0]["error"]
    lines.clear(), codes.clear()
    dog = bench.Watchdog(0.1, lines.append, codes.append)
    dog.stop()
    never = bench.Watchdog(0.0, lines.append, codes.append)
    never.touch("anything")
    time.sleep(0.3)
    assert not lines and not codes
