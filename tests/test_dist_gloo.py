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


# ---- the reference API on a multi-GPU job (hypernet2D under torchrun) --------
class _FakeJobSlab:
    """Stand-in for a slab FOMContext on a CPU: run_to_npy does what
    burg_run_npy_ex(NPY_GLOBAL | NPY_EXISTING) does -- checks the file's
    header and size, then writes this slab's u rows and v rows of the
    trajectory (the CPU oracle's march of the whole grid) at their global row
    offsets with pwrite.  Exercises the job protocol of dist.slabs_to_npy /
    hypernet2D (file creation by rank 0, barriers, error agreement, rename,
    copy-on-write maps) without a GPU."""

    def __init__(self, nx, ny, rank, world, fail=False):
        self.nx, self.ny_total, self.rank, self.world, self.fail = nx, ny, rank, world, fail
        self.row0, self.ny = slab_rows(ny, world, rank)

    def set_problem(self, grid_x, grid_y, dt, mu, allow_nonsquare=False):
        self.dt, self.mu = dt, tuple(mu)

    def close(self):
        pass

    def run_to_npy(self, w0_slab, T, path, snap_every=1, flags=0):
        from oracle import oracle
        from finitedifference_amd.dist import npy_header
        from finitedifference_amd.solver import NPY_EXISTING, NPY_GLOBAL
        assert flags == NPY_GLOBAL | NPY_EXISTING
        if self.fail:
            raise RuntimeError("injected slab failure")
        nx, ny = self.nx, self.ny_total
        n, ncols = nx * ny, T // snap_every + 1
        hdr = npy_header(2 * n, ncols)
        with open(path, "rb") as f:
            assert f.read(len(hdr)) == hdr
        assert os.path.getsize(path) == len(hdr) + 16 * n * ncols
        P = oracle.Problem(nx, dt=self.dt, mu=self.mu)
        ref, _, _ = P.fom(np.ones(2 * n), T)
        S = np.stack([ref[j * snap_every] for j in range(ncols)], axis=1)  # (2n, ncols)
        assert np.array_equal(slab_state(S[:, 0], nx, ny, self.rank, self.world), w0_slab)
        fd = os.open(path, os.O_RDWR)
        try:
            a, b = self.row0 * nx, (self.row0 + self.ny) * nx
            for lo in (a, n + a):  # u rows, then v rows
                os.pwrite(fd, np.ascontiguousarray(S[lo:lo + b - a]).tobytes(),
                          len(hdr) + 8 * ncols * lo)
        finally:
            os.close(fd)
        return {"loop_ms": 0.0}


def _job_worker(rank, world, port, N, T, every, mode, tmpdir, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank), BURG_SNAP_DIR=tmpdir)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from finitedifference_amd import hypernet2D as H
        made = []

        def fake_ctx(nx, ny, device, d, r, w, **opts):
            assert device == rank and opts.get("engine") == "pipe"
            made.append(1)
            return _FakeJobSlab(nx, ny, r, w, fail=(mode == "fail" and r == 1))
        H.job_context = fake_ctx
        gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
        w0 = np.ones(2 * N * N)
        out = {}
        if mode in ("implicit", "fail"):
            try:
                s = H.inviscid_burgers_implicit2D(gx, gy, w0, 0.05, T, (5.19, 0.026), verbose=0,
                                                  snap_every=every)
                out["snaps"] = np.array(s)
                out["cow"] = isinstance(s, np.memmap) and s.flags.writeable
            except RuntimeError as e:
                out["error"] = str(e)
            dist.barrier()  # (rank 0 unlinks the name after the ranks' maps exist)
            out["left"] = sorted(os.listdir(tmpdir))
        elif mode == "runfom":
            from finitedifference_amd import run_fom
            os.chdir(tmpdir)
            el, s = run_fom.main(5.19, 0.026, save_snaps=True, num_cells=N, num_steps=T,
                                 snap_folder=os.path.join(tmpdir, "param_snaps"))
            out["snaps"] = np.array(s)
            dist.barrier()
            out["files"] = sorted(os.listdir(tmpdir))
        else:
            folder = os.path.join(tmpdir, "param_snaps")
            s = H.load_or_compute_snaps((5.19, 0.026), gx, gy, w0, 0.05, T, snap_folder=folder,
                                        snap_every=every)
            out["snaps"] = np.array(s)
            dist.barrier()
            s2 = H.load_or_compute_snaps((5.19, 0.026), gx, gy, w0, 0.05, T, snap_folder=folder,
                                         snap_every=every)  # now a cache hit
            out["hit"] = np.array(s2)
            out["files"] = sorted(os.listdir(folder))
            out["made"] = len(made)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _run_job(world, N, T, every, mode, tmpdir):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_job_worker, args=(r, world, port, N, T, every, mode, tmpdir, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("N,T,every,world", [(12, 5, 1, 2), (13, 6, 3, 3)])
def test_implicit2D_on_a_job_assembles_the_whole_matrix(orc, tmp_path, N, T, every, world):
    """inviscid_burgers_implicit2D under a multi-rank job (gloo here; torchrun
    on the GPU box): every rank gets the whole reference-layout matrix (a
    copy-on-write map of the file all ranks wrote their rows into), equal to
    the single-domain march, and the shared file is gone afterwards."""
    res = _run_job(world, N, T, every, "implicit", str(tmp_path))
    ref, _, _ = orc.Problem(N).fom(np.ones(2 * N * N), T)
    want = np.stack([ref[j * every] for j in range(T // every + 1)], axis=1)
    for r in range(world):
        assert np.array_equal(res[r]["snaps"], want)
        assert res[r]["cow"]
        assert res[r]["left"] == []


def test_load_or_compute_snaps_on_a_job_writes_one_cache(orc, tmp_path):
    """load_or_compute_snaps under a multi-rank job: one cache file under the
    reference's name, written by all ranks (rank 0 renames it), equal to the
    single-domain march; the second call is a hit on every rank."""
    N, T, every, world = 11, 4, 2, 2
    res = _run_job(world, N, T, every, "cache", str(tmp_path))
    ref, _, _ = orc.Problem(N).fom(np.ones(2 * N * N), T)
    want = np.stack([ref[j * every] for j in range(T // every + 1)], axis=1)
    for r in range(world):
        assert np.array_equal(res[r]["snaps"], want)
        assert np.array_equal(res[r]["hit"], want)
        assert res[r]["files"] == ["mu1_5.19+mu2_0.026+every2.npy"]
        assert res[r]["made"] == 1
    assert np.array_equal(np.load(tmp_path / "param_snaps" / "mu1_5.19+mu2_0.026+every2.npy"), want)


def test_a_failed_rank_fails_every_rank(tmp_path):
    """One rank's slab fails: every rank raises (none waits forever or returns
    a half-written matrix) and the shared file is removed."""
    res = _run_job(2, 10, 3, 1, "fail", str(tmp_path))
    for r in range(2):
        assert "injected slab failure" in res[r]["error"] and "rank 1" in res[r]["error"]
        assert res[r]["left"] == []


def test_npy_header_is_numpys_layout(tmp_path):
    """dist.npy_header / create_npy (the header burg_run_npy writes) make a
    file np.load reads as a (m, ncols) float64 C-order array."""
    from finitedifference_amd.dist import create_npy, npy_header
    for m, n in [(2, 3), (2 * 750 * 750, 501), (10 ** 12, 1)]:
        h = npy_header(m, n)
        assert len(h) % 64 == 0 and h.endswith(b"\n")
    p = str(tmp_path / "x.npy")
    create_npy(p, 6, 4)
    a = np.load(p)
    assert a.shape == (6, 4) and a.dtype == np.float64 and not a.any()


def test_run_fom_main_on_a_job(orc, tmp_path, capfd):
    """run_fom.main (C/run_fom.py:9-52) under a multi-rank job: every rank
    returns the whole matrix, the cache is written once, rank 0 alone prints
    the timing line and saves hdm_snaps_*.npy."""
    N, T = 10, 3
    res = _run_job(2, N, T, 1, "runfom", str(tmp_path))
    ref, _, _ = orc.Problem(N).fom(np.ones(2 * N * N), T)
    want = np.stack(ref[:T + 1], axis=1)
    for r in range(2):
        assert np.array_equal(res[r]["snaps"], want)
        assert res[r]["files"] == ["hdm_snaps_mu1_5.19_mu2_0.026.npy", "param_snaps"]
    assert np.array_equal(np.load(tmp_path / "hdm_snaps_mu1_5.19_mu2_0.026.npy"), want)
    out = capfd.readouterr().out
    assert out.count("Elapsed FOM time") == 1 and out.count("HDM snapshots saved") == 1
