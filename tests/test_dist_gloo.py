"""CPU multi-process tests (torch.distributed gloo, world_size 2 and 4) of the y-slab
decomposition libcfdj.so uses across GPUs: halo rows + FFT all-to-all transposes.

The decomposition is restated in oracle/slab_oracle.py with the same pack layout
(S[q][jl][kl], kb = ceil((nx/2+1)/P)) and message roles as cfdj_api.hip; over real
process groups it must reproduce the single-domain oracle step to round-off."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, ws, port, nx, nsteps, q, poisson="transpose"):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from oracle import slab_oracle as so
        from oracle import vm_oracle as vo

        ny = nx
        dx, dy, x, y = vo.vm_grid(nx, ny)
        w = vo.vm_ic(nx, ny, x, y) + 0.1 * np.sin(3 * x[:nx, None]) * np.cos(2 * y[None, :ny])
        comm = so.DistComm()
        mine = [so.split(w, ws)[rank]]
        for _ in range(nsteps):
            if poisson == "one-gather":
                mine = so.slab_rk3_step_one_gather(mine, 0.01, nx, ny, dx, dy, 1000.0, 1e-6, comm)
            else:
                mine = so.slab_rk3_step(mine, 0.01, nx, ny, dx, dy, 1000.0, 1e-6, comm,
                                        poisson=poisson)
        if poisson == "one-gather":  # three solves per step, nothing else on the wire
            assert comm.calls == {"alltoall": 0, "allgather": 3 * nsteps, "halo": 0}, comm.calls
        # gather the slabs on rank 0 and compare with the single-domain oracle
        import torch

        t = torch.from_numpy(np.ascontiguousarray(mine[0]))
        parts = [torch.empty_like(t) for _ in range(ws)] if rank == 0 else None
        dist.gather(t, parts, dst=0)
        if rank == 0:
            full = np.concatenate([p.numpy() for p in parts], axis=1)
            ref = vo.numerical(w, nsteps, 0.01, dx, dy, 1000.0, workers=1)
            q.put(float(np.abs(full - ref).max()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws,nx", [(2, 32), (4, 48), (2, 40)])
def test_slab_decomposition_matches_single_domain(ws, nx):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    mp.start_processes(_worker, args=(ws, port, nx, 3, q), nprocs=ws, start_method="spawn",
                       join=True)
    err = q.get(timeout=5)
    assert err < 1e-13, err


@pytest.mark.parametrize("ws,nx", [(2, 64), (4, 64)])
def test_schur_slab_decomposition_matches_single_domain(ws, nx):
    # the substructured solve (all-gathers only) over real process groups
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    mp.start_processes(_worker, args=(ws, port, nx, 3, q, "schur"), nprocs=ws,
                       start_method="spawn", join=True)
    err = q.get(timeout=5)
    assert err < 1e-13, err


@pytest.mark.parametrize("ws,nx", [(2, 64), (4, 64)])
def test_one_gather_stage_matches_single_domain(ws, nx):
    """The y-slab step as libcfdj.so runs it on the substructured path: one all-gather per
    solve carries the traces, the untransformed column sums, the packed-column pieces and the
    first / last vorticity rows; psi's halo rows come out of the slab's own solve.  Over real
    process groups: the single-domain oracle to round-off, and exactly three collectives per
    step (asserted in the worker)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    mp.start_processes(_worker, args=(ws, port, nx, 3, q, "one-gather"), nprocs=ws,
                       start_method="spawn", join=True)
    err = q.get(timeout=5)
    assert err < 1e-13, err


def test_one_gather_halo_rows_are_the_neighbours_rows():
    """The halo rows the one-gather solve returns, against the neighbouring slabs' own rows
    (what the exchanging schedule would have sent), P = 1, 2, 4, 8."""
    from oracle import slab_oracle as so
    from oracle import vm_oracle as vo

    n = 128
    dx, dy, x, y = vo.vm_grid(n, n)
    w = vo.vm_ic(n, n, x, y) + 0.05 * np.random.default_rng(3).standard_normal((n, n))
    for P in (1, 2, 4, 8):
        comm = so.LocalComm(P)
        ws = so.split(w, P)
        res = so.slab_poisson_schur_one_gather(ws, n, n, dx, dy, 1e-6, comm)
        assert comm.calls == {"alltoall": 0, "allgather": 1}
        ref = so.slab_poisson_schur(ws, n, n, dx, dy, 1e-6, so.LocalComm(P))
        scale = np.abs(np.concatenate(ref, axis=1)).max()
        for p, (psi, slo, shi, wlo, whi) in enumerate(res):
            assert np.abs(psi - ref[p]).max() < 1e-13 * scale
            assert np.abs(slo - ref[(p - 1) % P][:, -1]).max() < 1e-12 * scale
            assert np.abs(shi - ref[(p + 1) % P][:, 0]).max() < 1e-12 * scale
            assert np.array_equal(wlo, ws[(p - 1) % P][:, -1])
            assert np.array_equal(whi, ws[(p + 1) % P][:, 0])


def test_schur_oracle_matches_fps():
    from oracle import schur_oracle as sc
    from oracle import vm_oracle as vo

    for n in (64, 256):
        dx, dy, x, y = vo.vm_grid(n, n)
        f = -(vo.vm_ic(n, n, x, y) + 0.01 * np.random.default_rng(n).standard_normal((n, n)))
        ref = vo.fps(f, dx, dy)
        for P in (1, 2, 4, 8):
            s = sc.schur_fps(f, dx, dy, P)
            assert np.abs(s - ref).max() < 1e-13 * np.abs(ref).max(), (n, P)


def test_schur_local_comm_matches_single_process():
    from oracle import schur_oracle as sc
    from oracle import slab_oracle as so
    from oracle import vm_oracle as vo

    n, P = 128, 4
    dx, dy, x, y = vo.vm_grid(n, n)
    w = vo.vm_ic(n, n, x, y)
    a = np.concatenate(so.slab_poisson_schur(so.split(w, P), n, n, dx, dy, 1e-6,
                                             so.LocalComm(P)), axis=1)
    b = sc.schur_fps(-w, dx, dy, P)
    assert np.abs(a - b).max() < 1e-15 * np.abs(b).max() * 10


def test_slab_local_comm_many_ranks():
    from oracle import slab_oracle as so
    from oracle import vm_oracle as vo

    nx = ny = 64
    dx, dy, x, y = vo.vm_grid(nx, ny)
    w = vo.vm_ic(nx, ny, x, y)
    ref = vo.numerical(w, 2, 0.01, dx, dy, 1000.0, workers=1)
    for P in (1, 2, 8, 16, 32):  # P = 32: 2 rows per slab, kb = 2 with padding
        ws = so.split(w, P)
        comm = so.LocalComm(P)
        for _ in range(2):
            ws = so.slab_rk3_step(ws, 0.01, nx, ny, dx, dy, 1000.0, 1e-6, comm)
        assert np.abs(np.concatenate(ws, axis=1) - ref).max() < 1e-13, P


def test_pack_unpack_roundtrip():
    from oracle import slab_oracle as so

    rng = np.random.default_rng(0)
    for nxh, rows, P in ((17, 4, 4), (9, 3, 2), (33, 2, 8)):
        kb = -(-nxh // P)
        X = rng.standard_normal((nxh, rows)) + 1j * rng.standard_normal((nxh, rows))
        S = so.pack(X, P, kb)
        assert S.shape == (P, rows, kb)
        assert np.array_equal(so.unpack(S, nxh), X)
        # padding columns are zero
        assert np.all(S.reshape(P * rows, kb)[:, :][np.repeat(np.arange(P), rows)[:, None] * kb
                                                     + np.arange(kb)[None, :] >= nxh] == 0)
