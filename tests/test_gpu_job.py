"""GPU: the reference API on a multi-GPU job, rehearsed
on the box's one GPU -- several processes, each a rank as torchrun would
start it (RANK / WORLD_SIZE / MASTER_*), every one on device 0 (on an 8-GPU
node: LOCAL_RANK).  Each rank calls the reference's own entry point
(run_fom.main -> load_or_compute_snaps -> inviscid_burgers_implicit2D), marches
its row slab with the one-way halo streamed from the rank below, and writes
its u rows and v rows straight into the one cache file of the whole grid
(burg_run_npy_ex).  The file must be the single-GPU file byte for byte.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

REF_TOL = 1e-10  # BASELINE.json north star: snapshots within 1e-10 rel-L2


def _run_job(out, world, args, timeout=300):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    worker = os.path.join(os.path.dirname(__file__), "job_worker.py")
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BURG_SPIN_SECONDS="20",
                   BURG_SNAP_DIR=str(out))
        procs.append(subprocess.Popen([sys.executable, worker, str(out)] + [str(a) for a in args],
                                      env=env))
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=timeout))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert codes == [0] * world, codes
    return [json.load(open(os.path.join(out, f"rank{r}.json"))) for r in range(world)]


def _files_equal(a, b, chunk=1 << 28):
    if os.path.getsize(a) != os.path.getsize(b):
        return False
    with open(a, "rb") as fa, open(b, "rb") as fb:
        while True:
            x, y = fa.read(chunk), fb.read(chunk)
            if x != y:
                return False
            if not x:
                return True


def test_run_fom_fine750_on_eight_ranks(gpu, tmp_path):
    """BurgersFD_CleanFine/run_fom.py:28 (750^2, 500 steps) through
    run_fom.main on 8 ranks (uneven 94/93-row slabs): the cache file
    mu1_5.19+mu2_0.026.npy equals the single-GPU direct cache byte for byte,
    every rank got the whole (2 750^2, 501) matrix (a copy-on-write map), and
    its u slices are within 1e-10 of the author's Fine HDM pickle."""
    from finitedifference_amd import hypernet2D as H
    N, T, world = 750, 500, 8
    job = tmp_path / "job"
    job.mkdir()
    infos = _run_job(job, world, ["fine750"])
    fn = job / "param_snaps" / "mu1_5.19+mu2_0.026.npy"
    assert sorted(os.listdir(job / "param_snaps")) == ["mu1_5.19+mu2_0.026.npy"]
    assert {i["digest"] for i in infos} and len({i["digest"] for i in infos}) == 1
    assert all(i["shape"] == [2 * N * N, T + 1] and i["memmap"] and i["writeable"] for i in infos)
    single = tmp_path / "single"
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    H.load_or_compute_snaps((5.19, 0.026), gx, gy, np.ones(2 * N * N), 0.05, T,
                            snap_folder=str(single), direct=True, mmap=True)
    assert _files_equal(fn, single / "mu1_5.19+mu2_0.026.npy")
    g = golden("author_pickles.npz")
    S = np.load(fn, mmap_mode="r")
    for k, col in enumerate(range(0, T + 1, 100)):
        U = np.asarray(S[:N * N, col]).reshape(N, N)
        for got, want in ((U[N // 2, :], g["fine_u_row"][k]), (U[:, N // 2], g["fine_u_col"][k])):
            assert np.linalg.norm(got - want) / np.linalg.norm(want) <= REF_TOL


def test_thinned_cache_16384x2048_on_two_ranks(gpu, tmp_path):
    """configs[4]'s row length: a 16384 x 2048 grid on 2 ranks (1024-row
    slabs, W = 1024), snap_every = 10, through load_or_compute_snaps: the
    thinned cache (+every10) equals the single-GPU direct file byte for byte."""
    from finitedifference_amd import hypernet2D as H
    nx, ny, T = 16384, 2048, 100
    job = tmp_path / "job"
    job.mkdir()
    infos = _run_job(job, 2, ["slab16384", T])
    name = "mu1_5.19+mu2_0.026+every10.npy"
    assert sorted(os.listdir(job / "param_snaps")) == [name]
    assert all(i["shape"] == [2 * nx * ny, T // 10 + 1] for i in infos)
    assert len({i["digest"] for i in infos}) == 1
    gx = np.linspace(0, 100, nx + 1)
    gy = np.linspace(0, 100.0 * ny / nx, ny + 1)
    single = tmp_path / "single"
    H.load_or_compute_snaps((5.19, 0.026), gx, gy, np.ones(2 * nx * ny), 0.05 * 1024 / nx, T,
                            snap_folder=str(single), direct=True, mmap=True, snap_every=10,
                            allow_nonsquare=True)
    assert _files_equal(job / "param_snaps" / name, single / name)
