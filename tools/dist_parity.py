#!/usr/bin/env python3
"""Multi-rank parity check of the RCCL y-slab path (one process per GPU).

  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port 29517 tools/dist_parity.py [--nx 1024] [--steps 3] [--poisson auto]

Every rank creates its slab handle over one RCCL communicator (unique id broadcast over
gloo, CPU tensors only), uploads the vm_ic initial condition, takes K RK3 steps and joins
the collective download; rank 0 compares the global field with the NumPy oracle
(oracle/vm_oracle.py, the checker) and prints one JSON line.  Exit status 0 = parity within
1e-10 of max|w|.  With one rank (N = 1) the slab code runs over a one-rank communicator.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=1024)
    ap.add_argument("--ny", type=int, default=None)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--poisson", default="auto", choices=["auto", "fused", "rocfft", "schur"])
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1:
        os.environ["CFDJ_FORCE_SLAB"] = "1"

    import numpy as np
    import torch
    import torch.distributed as dist

    from cfd_julia_amd import VortexMerger, _lib
    from oracle import vm_oracle as vo  # the checker only

    _lib.require_gpu()
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("gloo")
    nx, ny = a.nx, a.ny or a.nx
    dx, dy, x, y = vo.vm_grid(nx, ny)
    dt = 5e-4 * 2.0 * 4096.0 ** 2 / (nx ** 2 + ny ** 2)
    uid = VortexMerger.unique_id() if rank == 0 else bytes(128)
    t = torch.frombuffer(bytearray(uid), dtype=torch.uint8)
    if world > 1:
        dist.broadcast(t, src=0)
    w0 = vo.vm_ic(nx, ny, x, y)
    with VortexMerger(nx, ny, dx, dy, 1000.0, device=local_rank, kind="dist", nranks=world,
                      rank=rank, nccl_id=bytes(t.numpy().tobytes())) as h:
        h.set_poisson(a.poisson)
        path = h.poisson()
        h.upload(vo.to_ghosted(w0))
        h.step(dt, a.steps)
        w = h.download()[1:-1, 1:-1]  # collective: every rank ends with the global field
    ok = True
    if rank == 0:
        ref = vo.numerical(w0, a.steps, dt, dx, dy, 1000.0)
        err = float(np.abs(w - ref).max() / np.abs(ref).max())
        ok = bool(np.isfinite(err) and err < 1e-10)
        print(json.dumps({"ranks": world, "nx": nx, "ny": ny, "steps": a.steps,
                          "poisson": path, "linf_rel": err, "ok": ok}), flush=True)
    if world > 1:
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.broadcast(flag, src=0)
        ok = bool(flag[0])
        dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
