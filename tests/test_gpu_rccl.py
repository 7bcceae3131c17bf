"""RCCL slab path on a one-GPU box: a one-rank communicator (CFDJ_FORCE_SLAB=1) runs every
RCCL call of the y-slab code (ncclAllToAll transposes, grouped self send/recv halos,
ncclAllGather download) against the oracle.  Multi-rank runs need one GPU per rank (RCCL
refuses two ranks on a device) and happen in the driver's 8-GPU scaling job."""
import os

import numpy as np
import pytest

from oracle import vm_oracle as vo

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,steps", [(64, 5), (256, 5)])
def test_gpu_rccl_one_rank_slab(monkeypatch, n, steps):
    from cfd_julia_amd import VortexMerger, _lib

    _lib.require_gpu()
    monkeypatch.setenv("CFDJ_FORCE_SLAB", "1")
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.vm_ic(n, n, x, y)
    ref = vo.numerical(w0, steps, 0.01, dx, dy, 1000.0)
    uid = VortexMerger.unique_id()
    with VortexMerger(n, n, dx, dy, 1000.0, device=0, kind="dist", nranks=1, rank=0,
                      nccl_id=uid) as h:
        assert h.slab() == (0, n)
        h.upload_interior(w0)
        h.set_timing(True)
        h.step(0.01, steps)
        t = h.timing()
        w = h.download_interior()
    assert t["comm"][1] > 0  # the RCCL transposes / halos ran
    assert np.abs(w - ref).max() < 1e-10
