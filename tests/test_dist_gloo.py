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
