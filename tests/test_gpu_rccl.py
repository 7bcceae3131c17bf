"""RCCL slab path on a one-GPU box: a one-rank communicator (CFDJ_FORCE_SLAB=1) runs every
RCCL call of the y-slab code (ncclAllToAll transposes, grouped self send/recv halos,
ncclAllGather download) against the oracle.  Multi-rank runs need one GPU per rank (RCCL
refuses two ranks on a device) and happen in the driver's 8-GPU scaling job."""
import os

import numpy as np
import pytest

from oracle import vm_oracle as vo

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,steps,path", [(64, 5, "rocfft"), (256, 5, "rocfft"),
                                          (1024, 3, "fused"), (1024, 3, "rocfft"),
                                          (1024, 3, "schur")])
def test_gpu_rccl_one_rank_slab(monkeypatch, n, steps, path):
    from cfd_julia_amd import VortexMerger, _lib

    _lib.require_gpu()
    monkeypatch.setenv("CFDJ_FORCE_SLAB", "1")
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.vm_ic(n, n, x, y)
    dt = min(0.01, 5e-4 * (4096 / n) ** 2)
    ref = vo.numerical(w0, steps, dt, dx, dy, 1000.0)
    uid = VortexMerger.unique_id()
    with VortexMerger(n, n, dx, dy, 1000.0, device=0, kind="dist", nranks=1, rank=0,
                      nccl_id=uid) as h:
        assert h.slab() == (0, n)
        h.set_poisson(path)
        assert h.poisson() == path
        h.upload_interior(w0)
        h.set_timing(True)
        h.step(dt, steps)
        t = h.timing()
        w = h.download_interior()
    assert t["comm"][1] > 0  # the RCCL transposes / halos ran
    assert np.abs(w - ref).max() < 1e-10


@pytest.mark.parametrize("n,path", [(256, "rocfft"), (1024, "fused"), (1024, "schur")])
def test_gpu_rccl_halo_overlap(monkeypatch, n, path):
    """Halo exchanges on the side stream (omega during the Poisson passes, psi during the
    interior rows of the stage kernel; timing off) give the same field, bit for bit, as the
    single-stream sequence (CFDJ_NO_OVERLAP=1), and match the oracle."""
    from cfd_julia_amd import VortexMerger, _lib

    _lib.require_gpu()
    monkeypatch.setenv("CFDJ_FORCE_SLAB", "1")
    dx, dy, x, y = vo.vm_grid(n, n)
    w0 = vo.vm_ic(n, n, x, y)
    dt, steps = min(0.01, 5e-4 * (4096 / n) ** 2), 4
    ref = vo.numerical(w0, steps, dt, dx, dy, 1000.0)
    out = {}
    for ov in ("0", "1"):
        monkeypatch.setenv("CFDJ_NO_OVERLAP", ov)
        with VortexMerger(n, n, dx, dy, 1000.0, device=0, kind="dist", nranks=1, rank=0,
                          nccl_id=VortexMerger.unique_id()) as h:
            h.set_poisson(path)
            h.upload_interior(w0)
            h.step(dt, 2)
            h.step(dt, 2)
            out[ov] = h.download_interior()
    assert np.array_equal(out["0"], out["1"])
    assert np.abs(out["0"] - ref).max() < 1e-10
