"""Multi-rank host logic on CPU (gloo, world_size 2): ring-name agreement,
slab split / assembly of states and snapshot matrices in the reference
layout.  The GPU side of the halo is covered by
test_gpu_parity.py::test_slab_halo_two_processes_one_gpu."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from finitedifference_amd.dist import (agree_halo_name, assemble_snaps, assemble_state,
                                       slab_rows, slab_state)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, nx, ny, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        name = agree_halo_name(dist)
        # every rank builds the same global trajectory and keeps its slab
        rng = np.random.default_rng(7)
        snaps = rng.random((2 * nx * ny, 4))
        mine = np.stack([slab_state(snaps[:, j], nx, ny, rank, world) for j in range(4)], axis=1)
        parts = [None] * world
        dist.all_gather_object(parts, mine)
        ok = np.array_equal(assemble_snaps(parts, nx, ny), snaps)
        names = [None] * world
        dist.all_gather_object(names, name)
        q.put((rank, ok, len(set(names)) == 1, mine.shape))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nx,ny,world", [(8, 13, 2), (5, 6, 3)])
def test_slab_split_and_name_agreement_over_gloo(nx, ny, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nx, ny, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, same_name, shape in res:
        assert ok and same_name
        assert shape == (2 * nx * slab_rows(ny, world, rank)[1], 4)


def test_state_split_roundtrip():
    nx, ny, world = 7, 10, 4
    w = np.arange(2.0 * nx * ny)
    parts = [slab_state(w, nx, ny, r, world) for r in range(world)]
    assert sum(p.size for p in parts) == w.size
    assert np.array_equal(assemble_state(parts, nx, ny), w)
    # the u block of rank r is rows [row0, row0+rows) of the (ny, nx) u plane
    row0, rows = slab_rows(ny, world, 2)
    assert np.array_equal(parts[2][:rows * nx], w[row0 * nx:(row0 + rows) * nx])


def test_single_process_name_is_fresh():
    a, b = agree_halo_name(None), agree_halo_name(None)
    assert a != b and "/" not in a and 0 < len(a) <= 64


class _OracleSlab:
    """Stand-in for a slab FOMContext whose slab_residual is the CPU oracle's
    residual on the slab's rows plus the halo row below (the checker's view of
    burg_slab_residual): exercises dist.slab_residual_norms' exchange and
    reduction without a GPU."""

    def __init__(self, nx, ny, rank, world):
        from oracle import oracle
        self.P = oracle.Problem(nx, ny, Ly=100.0 * ny / nx, allow_nonsquare=nx != ny)
        self.nx, self.rank, self.world = nx, rank, world
        self.row0, self.ny = slab_rows(ny, world, rank)

    def slab_residual(self, w, wp, hw=None, hwp=None):
        import ctypes
        from oracle import oracle
        nx, r0, rows = self.nx, self.row0, self.ny
        lo = r0 - 1 if hw is not None else r0
        ext = rows + (1 if hw is not None else 0)

        def extend(x, h):
            x = np.asarray(x).reshape(2, rows, nx)
            if h is None:
                return np.ascontiguousarray(x).ravel()
            return np.ascontiguousarray(np.concatenate((np.asarray(h).reshape(2, 1, nx), x),
                                                       axis=1)).ravel()
        we, wpe = extend(w, hw), extend(wp, hwp)
        iy = np.ascontiguousarray(self.P.inv_dy[lo:lo + ext])
        lb = np.ascontiguousarray(self.P.lbc[lo:lo + ext])
        r = np.empty(2 * nx * ext)
        p = oracle._p
        oracle.lib().orc_residual(nx, ext, p(self.P.inv_dx), p(iy), p(self.P.src), p(lb),
                                  ctypes.c_double(self.P.dt), p(we), p(wpe), p(r))
        r = r.reshape(2, ext, nx)[:, ext - rows:, :].ravel()
        return r, float(np.dot(r, r))


def _res_worker(rank, world, port, nx, ny, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from finitedifference_amd.dist import slab_residual_norms
        rng = np.random.default_rng(11)
        w = rng.uniform(1, 6, 2 * nx * ny)
        wp = rng.uniform(1, 6, 2 * nx * ny)
        ctx = _OracleSlab(nx, ny, rank, world)
        g, s = slab_residual_norms(ctx, slab_state(w, nx, ny, rank, world),
                                   slab_state(wp, nx, ny, rank, world), dist)
        from finitedifference_amd.dist import exchange_halo_rows, top_row
        mine_w = slab_state(w, nx, ny, rank, world)
        mine_wp = slab_state(wp, nx, ny, rank, world)
        got = exchange_halo_rows(np.concatenate((top_row(mine_w, nx, ctx.ny),
                                                 top_row(mine_wp, nx, ctx.ny))), nx, rank, world,
                                 dist)
        r, _ = ctx.slab_residual(mine_w, mine_wp, *((None, None) if got is None else
                                                    (got[:2 * nx], got[2 * nx:])))
        q.put((rank, g, s, r))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nx,ny,world", [(9, 14, 2), (6, 10, 3)])
def test_slab_residual_norms_over_gloo(orc, nx, ny, world):
    """dist.slab_residual_norms (the multi-GPU bench's self-check): the south
    halo rows travel one way (rank k -> k+1, send/recv), each slab's residual
    with them equals the single-domain residual's rows bit for bit, and the
    summed norm equals the single-domain norm."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_res_worker, args=(r, world, port, nx, ny, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in range(world)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    P = orc.Problem(nx, ny, Ly=100.0 * ny / nx, allow_nonsquare=True)
    rng = np.random.default_rng(11)
    w = rng.uniform(1, 6, 2 * nx * ny)
    wp = rng.uniform(1, 6, 2 * nx * ny)
    want = P.residual(w, wp)
    assert np.array_equal(assemble_state([t[3] for t in res], nx, ny), want)
    g = np.linalg.norm(want)
    for rank, gn, sn, r in res:
        assert abs(gn - g) <= 1e-14 * g
        assert abs(sn - np.linalg.norm(r)) <= 1e-14 * g
