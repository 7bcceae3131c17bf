"""Multi-rank RCCL parity (tools/dist_parity.py under torch.distributed.run).

With one visible GPU only the one-rank form runs (the slab code over a one-rank
communicator); the 2-, 4- and 8-rank forms need that many GPUs on the node and are skipped
otherwise -- on such a node they are the parity test against the oracle (tolerance 1e-10 of
max|w|) of the substructured path's one all-gather per stage (traces, column sums, packed
column, the neighbours' vorticity rows) and, in the "fused" case, of the transpose path's
all-to-alls and its halo send/recv pairing.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def visible_gpus():
    import torch

    return torch.cuda.device_count()


@pytest.mark.parametrize("ranks,nx,poisson", [(1, 1024, "auto"), (2, 1024, "auto"),
                                              (2, 1024, "fused"), (4, 2048, "auto"),
                                              (8, 4096, "auto")])
def test_gpu_dist_parity_vs_oracle(ranks, nx, poisson):
    if visible_gpus() < ranks:
        pytest.skip(f"needs {ranks} GPUs on this node")
    port = 29517 + ranks
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={ranks}", "--master-addr", "127.0.0.1", "--master-port",
           str(port), os.path.join(ROOT, "tools", "dist_parity.py"), "--nx", str(nx),
           "--steps", "3", "--poisson", poisson]
    print("dist parity case:", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    out = json.loads(lines[-1])
    assert out["ok"] and out["ranks"] == ranks and out["linf_rel"] < 1e-10, out
