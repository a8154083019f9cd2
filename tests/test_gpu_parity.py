"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
reference's golden vectors.  Bars: bitwise for equal op order and tiling,
rel-L2 <= 1e-10 against the reference trajectory (north-star tolerance).
"""
import os

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

TOL4ULP = 2.0 ** -50
REF_TOL = 1e-10  # BASELINE.json north star: snapshots within 1e-10 rel-L2


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(b))


def make_ctx(N, mu=(5.19, 0.026), dt=0.05, ny=None, **opts):
    from finitedifference_amd.solver import FOMContext
    ny = N if ny is None else ny
    ctx = FOMContext(N, ny, **opts)
    gx = np.linspace(0, 100, N + 1)
    gy = np.linspace(0, 100, ny + 1)
    ctx.set_problem(gx, gy, dt, mu, allow_nonsquare=(ny != N))
    return ctx


def state_after(orc, P, steps):
    w = np.ones(P.m)
    for _ in range(steps):
        w = P.march_step(w)
    return w


# ---------------------------------------------------------------- K1 / K2 --
@pytest.mark.parametrize("N", [16, 64, 250])
def test_residual_bitwise_vs_oracle_and_reference(gpu, orc, N):
    g = golden("ref_ops.npz")
    mu = tuple(g[f"n{N}_mu"])
    w, wp = g[f"n{N}_w"], g[f"n{N}_wp"]
    ctx = make_ctx(N, mu)
    r, nrm = ctx.residual(w, wp)
    P = orc.Problem(N, mu=mu)
    ro = P.residual(w, wp)
    assert np.array_equal(r, ro), "GPU residual must equal the oracle bit for bit"
    assert abs(nrm - np.linalg.norm(ro)) <= 1e-13 * np.linalg.norm(ro)
    if N <= 64:
        assert rel(r, g[f"n{N}_res"]) <= 1e-15
    else:
        assert np.allclose(r[g["n250_res_idx"]], g["n250_res_at"], rtol=1e-14, atol=0)


@pytest.mark.parametrize("N", [16, 64, 250])
def test_jvp_bitwise_vs_oracle_and_reference(gpu, orc, N):
    g = golden("ref_ops.npz")
    w, x = g[f"n{N}_w"], g[f"n{N}_x"]
    ctx = make_ctx(N, tuple(g[f"n{N}_mu"]))
    y = ctx.jvp(w, x)
    P = orc.Problem(N, mu=tuple(g[f"n{N}_mu"]))
    assert np.array_equal(y, P.jvp(w, x))
    if N <= 64:
        assert rel(y, g[f"n{N}_jx"]) <= 1e-14
    else:
        assert np.allclose(y[g["n250_res_idx"]], g["n250_jx_at"], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("nx,ny", [(300, 70), (520, 300), (257, 33), (1024, 1024)])
def test_stencils_bitwise_ragged_strips(gpu, orc, nx, ny):
    """Row-marching stencils (256-column strips, south terms carried, west
    terms by DPP): ragged last strip, several strips, partial row blocks --
    bit-equal to the oracle's one-cell-at-a-time restatement."""
    P = orc.Problem(nx, ny, Ly=100.0 * ny / nx, allow_nonsquare=(nx != ny))
    rng = np.random.default_rng(1234557)
    w = rng.uniform(1.0, 6.0, P.m)
    wp = rng.uniform(1.0, 6.0, P.m)
    x = rng.standard_normal(P.m)
    ctx = make_ctx(nx, ny=ny)
    ctx.set_problem(P.grid_x, P.grid_y, P.dt, P.mu, allow_nonsquare=(nx != ny))
    r, nrm = ctx.residual(w, wp)
    ro = P.residual(w, wp)
    assert np.array_equal(r, ro)
    assert abs(nrm - np.linalg.norm(ro)) <= 1e-13 * np.linalg.norm(ro)
    assert np.array_equal(ctx.jvp(w, x), P.jvp(w, x))


def test_kernel_bench_runs(gpu):
    ctx = make_ctx(512)
    ctx.upload(np.ones(ctx.m))
    for k in ("residual", "jvp"):
        ms = ctx.kernel_bench(k, reps=3)
        assert 0.0 < ms < 100.0


@pytest.mark.parametrize("N", [16, 64])
def test_block_solve_matches_spsolve(gpu, orc, N):
    g = golden("ref_ops.npz")
    w, r = g[f"n{N}_w"], g[f"n{N}_res"]
    ctx = make_ctx(N, tuple(g[f"n{N}_mu"]), tol=0.0)
    d = ctx.block_solve(w, r)
    P = orc.Problem(N, mu=tuple(g[f"n{N}_mu"]))
    assert np.array_equal(d, P.block_solve(w, r)), "tol=0 reaches the sequential fixed point"
    assert rel(d, g[f"n{N}_solve"]) <= 1e-13  # SuperLU spsolve (C/hypernet2D.py:1854)


# ------------------------------------------------------------------ march --
@pytest.mark.parametrize("N,tw,par", [(13, 64, 3), (64, 64, 3), (100, 64, 3), (250, 64, 3),
                                      (250, 128, 3), (300, 128, 3), (300, 64, 1)])
def test_march_step_bitwise_sequential(gpu, orc, N, tw, par):
    """tol = 0: the tile engine's fixed point is the sequential march (needs
    ~#tile rows passes in y-uniform regions: exercises the tail path)."""
    P = orc.Problem(N)
    wp = state_after(orc, P, 7)
    ctx = make_ctx(N, tile_w=tw, tol=0.0, par_passes=par, engine="tiles")
    snaps, st, its, _ = ctx.run(wp, 1)
    assert st["unconverged_steps"] == 0
    assert np.array_equal(snaps[:, 1], P.march_step(wp))


@pytest.mark.parametrize("N,tw,par", [(250, 64, 3), (333, 64, 3), (512, 128, 3), (333, 64, 1),
                                      (512, 64, 2)])
def test_march_step_bitwise_tiled_schedule(gpu, orc, N, tw, par):
    """tol = 4 ulp: the GPU reproduces the CPU schedule simulator bit for bit,
    and both sit within ~1e-16 of the sequential march.  par < 3 leaves passes
    to the final kernel's last workgroup (the tail path)."""
    P = orc.Problem(N)
    wp = state_after(orc, P, 20)
    ctx = make_ctx(N, tile_w=tw, tol=TOL4ULP, par_passes=par, engine="tiles")
    snaps, st, its, _ = ctx.run(wp, 1)
    ws, k, _ = P.march_tiled(wp, tw=tw, tol=TOL4ULP)
    assert np.array_equal(snaps[:, 1], ws)
    assert its[0] == k
    assert rel(ws, P.march_step(wp)) <= 1e-14


# ------------------------------------------------------ streaming engine --
@pytest.mark.parametrize("N,ny,W,tiles,T", [
    (13, 13, 8, 0, 5), (64, 64, 16, 0, 4), (100, 100, 0, 0, 6), (250, 250, 0, 0, 5),
    (250, 250, 64, 0, 3), (333, 333, 32, 0, 3), (130, 70, 8, 0, 4), (96, 200, 16, 0, 4),
    (512, 512, 0, 4096, 2), (300, 300, 256, 0, 3), (200, 129, 0, 64, 7)])
def test_stream_bitwise_sequential_march(gpu, orc, N, ny, W, tiles, T):
    """The streaming engine IS the sequential march: every snapshot bit-equal
    to the oracle's orc_march_step trajectory, for any tiling (partial tiles,
    partial strips, non-square grids, one tile column, many tiles)."""
    P = orc.Problem(N, ny, Ly=100.0 * ny / N, allow_nonsquare=(N != ny))
    w0 = state_after(orc, P, 3)
    ctx = FOMContext_for(N, ny, engine="stream", stream_w=W, tiles_target=tiles)
    ctx.set_problem(P.grid_x, P.grid_y, P.dt, P.mu, allow_nonsquare=(N != ny))
    snaps, st, its, _ = ctx.run(w0, T)
    ref, _, _ = P.fom(w0, T)
    for j in range(T + 1):
        assert np.array_equal(snaps[:, j], ref[j]), f"step {j}"
    assert st["engine"] == 0 and st["steps"] == T and st["stream_launches"] == 1
    assert st["tile_marches"] == T * st["stream_tiles"]
    assert np.all(its == 1)


def FOMContext_for(nx, ny, **opts):
    from finitedifference_amd.solver import FOMContext
    return FOMContext(nx, ny, **opts)


@pytest.mark.parametrize("chunk", [1, 3, 7])
def test_stream_chunked_run_and_snap_every(gpu, orc, monkeypatch, chunk):
    """Runs longer than the ring (forced small chunks) and snap_every > 1 give
    the same columns as one long launch."""
    N, T = 96, 12
    P = orc.Problem(N)
    w0 = np.ones(P.m)
    ref, _, _ = P.fom(w0, T)
    monkeypatch.setenv("BURG_STREAM_CHUNK", str(chunk))
    ctx = make_ctx(N, engine="stream", stream_w=16)
    snaps, st, _, _ = ctx.run(w0, T)
    assert st["stream_launches"] == -(-T // chunk)
    assert all(np.array_equal(snaps[:, j], ref[j]) for j in range(T + 1))
    sub, _, _, _ = ctx.run(w0, T, snap_every=5)
    assert sub.shape == (P.m, T // 5 + 1)
    assert all(np.array_equal(sub[:, j], ref[5 * j]) for j in range(T // 5 + 1))


def test_stream_advance_matches_run(gpu, orc):
    N = 200
    P = orc.Problem(N)
    ref, _, _ = P.fom(np.ones(P.m), 9)
    ctx = make_ctx(N, engine="stream")
    ctx.upload(np.ones(P.m))
    for k in (2, 3, 4):  # several launches continue the same trajectory
        ctx.advance(k)
    assert np.array_equal(ctx.download(), ref[9])


def test_stream_and_tiles_engines_agree_at_tol0(gpu):
    N, T = 160, 5
    a = make_ctx(N, engine="stream").run(np.ones(2 * N * N), T)[0]
    b = make_ctx(N, engine="tiles", tol=0.0).run(np.ones(2 * N * N), T)[0]
    assert np.array_equal(a, b)


def test_march_solves_the_reference_residual(gpu):
    """Size-independent property at the bench size: R(w_next; w) ~ 0."""
    N = 1024
    ctx = make_ctx(N)
    w0 = np.ones(2 * N * N)
    snaps, st, its, _ = ctx.run(w0, 3)
    r0, n0 = ctx.residual(snaps[:, 2], snaps[:, 2])
    r1, n1 = ctx.residual(snaps[:, 3], snaps[:, 2])
    assert n1 / n0 < 1e-13
    assert st["unconverged_steps"] == 0


# ------------------------------------------------------ full trajectories --
@pytest.mark.parametrize("tag", ["n8", "n13", "n16", "n16b", "n50", "n100"])
def test_small_trajectories_vs_reference(gpu, tag):
    g = golden("ref_small.npz")
    N, T, mu1, mu2, dt = g[f"{tag}_meta"]
    N, T = int(N), int(T)
    ctx = make_ctx(N, (mu1, mu2), dt)
    snaps, st, its, _ = ctx.run(np.ones(2 * N * N), T)
    ref = g[f"{tag}_snaps"]
    assert snaps.shape == ref.shape and snaps.flags.c_contiguous
    worst = max(rel(snaps[:, j], ref[:, j]) for j in range(1, T + 1))
    assert worst <= REF_TOL, worst


@pytest.mark.parametrize("tag", ["n8", "n13", "n16b", "n50"])
def test_newton_mode_counts_match_reference(gpu, tag):
    """solver='newton' is the reference algorithm: same Newton update counts
    per step as the reference's printed log."""
    g = golden("ref_small.npz")
    N, T, mu1, mu2, dt = g[f"{tag}_meta"]
    N, T = int(N), min(int(T), 60)
    ctx = make_ctx(N, (mu1, mu2), dt)
    snaps, st, its, rl = ctx.run(np.ones(2 * N * N), T, solver="newton")
    assert np.array_equal(its, g[f"{tag}_its"][:T])
    ref = g[f"{tag}_snaps"][:, :T + 1]
    assert max(rel(snaps[:, j], ref[:, j]) for j in range(1, T + 1)) <= 1e-13


def test_coarse250_full_run_vs_reference(gpu, orc):
    """C/run_fom.py defaults: 250^2, 500 steps, mu=(5.19, 0.026)."""
    g = golden("ref_coarse250.npz")
    N, T = 250, 500
    ctx = make_ctx(N)
    snaps, st, its, _ = ctx.run(np.ones(2 * N * N), T)
    assert st["unconverged_steps"] == 0
    for j in (1, 2, 100, 500):
        assert rel(snaps[:, j], g[f"state_{j}"]) <= REF_TOL
    norms = np.sqrt(np.square(snaps).sum(axis=0))
    assert np.allclose(norms, g["col_norm"], rtol=1e-12, atol=0)
    n = N * N
    U = snaps[:n].reshape(N, N, -1)
    steps = g["slice_steps"]
    assert rel(U[N // 2, :, steps].T, g["u_row"].T) <= REF_TOL
    ws = orc.Problem(N).fom(np.ones(2 * n), T)[0]
    # streaming engine = the sequential march, bit for bit, over all 500 steps
    assert all(np.array_equal(snaps[:, j], ws[j]) for j in range(0, T + 1, 7))
    assert np.array_equal(snaps[:, T], ws[T])


def test_fine750_vs_author_pickle(gpu):
    """F/ grid, 500 steps: the author's pickled HDM mid-line slices."""
    g = golden("author_pickles.npz")
    N, T = 750, 500
    ctx = make_ctx(N)
    snaps, st, its, _ = ctx.run(np.ones(2 * N * N), T, snap_every=100)
    n = N * N
    U = snaps[:n].reshape(N, N, -1)
    for k in range(6):
        assert rel(U[N // 2, :, k], g["fine_u_row"][k]) <= REF_TOL
        assert rel(U[:, N // 2, k], g["fine_u_col"][k]) <= REF_TOL


def test_snap_every_layout(gpu):
    N, T = 64, 12
    ctx = make_ctx(N)
    full, _, _, _ = ctx.run(np.ones(2 * N * N), T)
    sub, _, _, _ = ctx.run(np.ones(2 * N * N), T, snap_every=4)
    assert sub.shape == (2 * N * N, 4)
    assert np.array_equal(sub, full[:, ::4])


@pytest.mark.parametrize("engine", ["stream", "tiles"])
def test_device_resident_advance_matches_run(gpu, engine):
    N, T = 128, 9
    ctx = make_ctx(N, engine=engine)
    full, _, _, _ = ctx.run(np.ones(2 * N * N), T)
    ctx.upload(np.ones(2 * N * N))
    st = ctx.advance(T)
    assert st["steps"] == T
    assert np.array_equal(ctx.download(), full[:, T])


# ----------------------------------------------------------- pipe engine --
@pytest.mark.parametrize("N,ny,W,T", [
    (13, 13, 8, 5), (64, 64, 16, 4), (100, 100, 0, 6), (250, 250, 0, 5), (130, 70, 8, 4),
    (96, 200, 16, 4), (200, 129, 0, 7), (40, 64, 8, 9), (176, 64, 16, 3), (520, 300, 16, 3),
    (1024, 1024, 0, 2)])
def test_pipe_bitwise_sequential_march(gpu, orc, N, ny, W, T):
    """The pipe engine IS the sequential march: every snapshot bit-equal to
    the oracle's orc_march_step trajectory, for any tiling: one tile, partial
    strips, partial workgroups (tile columns not a multiple of 4), non-square."""
    P = orc.Problem(N, ny, Ly=100.0 * ny / N, allow_nonsquare=(N != ny))
    w0 = state_after(orc, P, 3)
    ctx = FOMContext_for(N, ny, engine="pipe", stream_w=W)
    ctx.set_problem(P.grid_x, P.grid_y, P.dt, P.mu, allow_nonsquare=(N != ny))
    snaps, st, its, _ = ctx.run(w0, T)
    ref, _, _ = P.fom(w0, T)
    assert st["engine"] == 2, "pipe engine expected (no fallback at these sizes)"
    for j in range(T + 1):
        assert np.array_equal(snaps[:, j], ref[j]), f"step {j}"
    assert st["steps"] == T and st["stream_launches"] == 1
    assert st["tile_marches"] == T * st["stream_tiles"]


def test_pipe_many_launches_cycle_sentinel_colours(gpu, orc):
    """Launch lengths that are not multiples of the mailbox depth (8 steps):
    the absolute step counter carries the sentinel colours across launches."""
    N = 136
    P = orc.Problem(N)
    ks = (1, 2, 3, 5, 7, 9, 11, 13)
    ref, _, _ = P.fom(np.ones(P.m), sum(ks))
    ctx = make_ctx(N, engine="pipe", stream_w=8)
    ctx.upload(np.ones(P.m))
    for k in ks:
        st = ctx.advance(k)
        assert st["engine"] == 2
    assert np.array_equal(ctx.download(), ref[sum(ks)])


def test_pipe_and_stream_engines_agree(gpu):
    N, T = 300, 6
    a = make_ctx(N, engine="pipe").run(np.ones(2 * N * N), T)[0]
    b = make_ctx(N, engine="stream").run(np.ones(2 * N * N), T)[0]
    assert np.array_equal(a, b)


def _halo_modes(tmp_path, world):
    """(in, out) halo ring placement each slab worker reported."""
    return [tuple(int(x) for x in open(os.path.join(tmp_path, f"slab{r}.halo")).read().split())
            for r in range(world)]


@pytest.mark.parametrize("N,world,T,halo", [(128, 2, 9, "device"), (150, 3, 7, "device"),
                                            (150, 3, 7, "host"), (150, 3, 7, "reject")])
def test_slab_halo_two_processes_one_gpu(gpu, orc, tmp_path, N, world, T, halo):
    """Multi-GPU path, rehearsed on one GPU: `world` processes, one slab each,
    all on device 0, exchanging the halo while their time loops run
    concurrently -- through each consumer's device-memory ring opened over IPC
    (the default), or the pinned host rings (BURG_HALO=host; "reject": the
    device rings pass the producer's probe but every consumer's
    burg_slab_verify rejects them, so both sides must move to the host ring).
    The assembled trajectory is the single-grid sequential march bit for bit."""
    env = {"device": {}, "host": {"BURG_HALO": "host"}, "reject": {"BURG_HALO_REJECT": "1"}}[halo]
    _run_slabs(tmp_path, N, T, world, **env)
    mode = 2 if halo == "device" else 1
    want = [(0 if r == 0 else mode, 0 if r == world - 1 else mode) for r in range(world)]
    assert _halo_modes(tmp_path, world) == want
    # the launch diagnostics a multi-GPU bench line reports per rank (DESIGN.md
    # section 7): rank 0 has no inbound halo; the others waited for it, within
    # their launch's ramp; only a halo strip counts halo waits
    import json
    for r in range(world):
        d = json.load(open(os.path.join(tmp_path, f"slab{r}.stats")))
        assert 0 < d["ramp_ms"] < d["loop_ms"], (r, d)
        if r == 0:
            assert d["halo_wait_ms"] == -1 and d["south_waits_halo"] == 0, d
        else:
            assert 0 <= d["halo_wait_ms"] <= d["ramp_ms"], (r, d)
        assert d["south_wait_ms_halo"] >= 0 and d["south_wait_ms_local"] >= 0
        assert d["bounds_hits"] == 0 and d["bounds_checks"] >= 1
    from finitedifference_amd.dist import assemble_snaps
    parts = [np.load(os.path.join(tmp_path, f"slab{r}.npy")) for r in range(world)]
    snaps = assemble_snaps(parts, N, N)
    ref, _, _ = orc.Problem(N).fom(np.ones(2 * N * N), T)
    for j in range(T + 1):
        assert np.array_equal(snaps[:, j], ref[j]), f"step {j}"


def test_slab_halo_sweep_two_processes_one_gpu(gpu, orc, tmp_path):
    """The multi-GPU halo stream carries a mu sweep too: 2 slab processes on
    one GPU, 3 trajectories back to back; each assembled trajectory is the
    single-grid march for its mu, bit for bit."""
    N, T, world = 128, 6, 2
    _run_slabs(tmp_path, N, T, world, mode="sweep")
    from finitedifference_amd.dist import assemble_snaps
    from slab_worker import SWEEP_MUS
    for j, mu in enumerate(SWEEP_MUS):
        parts = [np.load(os.path.join(tmp_path, f"slab{r}_mu{j}.npy")) for r in range(world)]
        snaps = assemble_snaps(parts, N, N)
        ref, _, _ = orc.Problem(N, mu=mu).fom(np.ones(2 * N * N), T)
        for k in range(T + 1):
            assert np.array_equal(snaps[:, k], ref[k]), f"mu {mu} step {k}"


def _run_slabs(tmp_path, N, T, world, mode="run", timeout=110, **env_extra):
    """Start `world` slab_worker processes on device 0 (gloo rendezvous) and
    wait for them; env_extra: SLAB_NY, SLAB_W, SLAB_TILES, SLAB_SNAP_EVERY,
    BURG_HALO."""
    import subprocess
    import sys
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    worker = os.path.join(os.path.dirname(__file__), "slab_worker.py")
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), BURG_SPIN_SECONDS="20")
        env.update({k: str(v) for k, v in env_extra.items()})
        procs.append(subprocess.Popen([sys.executable, worker, str(N), str(T), str(tmp_path),
                                       mode], env=env))
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=timeout))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert codes == [0] * world, codes


# ------------------------------------------------- pipe engine, wide tiles --
@pytest.mark.parametrize("N,ny,W,T", [
    (300, 300, 32, 4), (520, 300, 64, 3), (1000, 130, 128, 3), (700, 200, 256, 2),
    (2100, 64, 512, 2), (1500, 100, 1024, 2), (333, 129, 256, 3)])
def test_pipe_wide_bitwise_sequential_march(gpu, orc, N, ny, W, T):
    """Wide tiles (previous state streamed from the HBM ring, not LDS): every
    snapshot bit-equal to the oracle's sequential march -- partial tiles
    (nx not a multiple of W), partial strips, one tile column, non-square."""
    P = orc.Problem(N, ny, Ly=100.0 * ny / N, allow_nonsquare=(N != ny))
    w0 = state_after(orc, P, 3)
    ctx = FOMContext_for(N, ny, engine="pipe", stream_w=W)
    ctx.set_problem(P.grid_x, P.grid_y, P.dt, P.mu, allow_nonsquare=(N != ny))
    snaps, st, its, _ = ctx.run(w0, T)
    ref, _, _ = P.fom(w0, T)
    assert st["engine"] == 2 and st["stream_w"] == W
    for j in range(T + 1):
        assert np.array_equal(snaps[:, j], ref[j]), f"step {j}"
    assert st["tile_marches"] == T * st["stream_tiles"]
    assert st["nonfinite_diagonals"] == 0


def test_pipe_4096_bitwise(gpu, orc):
    """BASELINE config 3 (4096^2, one GPU) on the engine the planner picks
    (pipe, W = 256: 1024 tiles): 3 steps from w0 = 1, bit-equal to the oracle."""
    N, T = 4096, 3
    P = orc.Problem(N)
    ctx = make_ctx(N)
    snaps, st, _, _ = ctx.run(np.ones(P.m), T)
    assert st["engine"] == 2 and st["stream_w"] == 256 and st["stream_tiles"] == 1024
    ref, _, _ = P.fom(np.ones(P.m), T)
    for j in range(T + 1):
        assert np.array_equal(snaps[:, j], ref[j]), f"step {j}"


def test_pipe_4096_trajectory_matches_run(gpu, orc):
    """The bench's unit of work at 4096^2 (burg_trajectory, state resident in
    HBM) leaves the same final state as burg_run."""
    N, T = 4096, 4
    ctx = make_ctx(N)
    w0 = np.ones(2 * N * N)
    snaps, _, _, _ = ctx.run(w0, T, snap_every=T)
    ctx.upload(w0)
    st = ctx.trajectory(T)
    assert st["engine"] == 2 and st["stream_w"] == 256
    assert np.array_equal(ctx.download(), snaps[:, 1])


def test_reserve_then_trajectory(gpu, orc):
    """burg_reserve_trajectory allocates what burg_trajectory needs without
    launching (the multi-GPU bench calls it before its barrier); the
    trajectories that follow -- including a longer one, which grows the
    ring, and a repeat, which reuses it -- are the oracle's march bit for bit."""
    N = 200
    P = orc.Problem(N)
    ref, _, _ = P.fom(np.ones(P.m), 7)
    ctx = make_ctx(N)
    ctx.upload(np.ones(P.m))
    ctx.reserve(5)
    ctx.reserve(5)
    st = ctx.trajectory(5)
    assert st["engine"] == 2
    assert np.array_equal(ctx.download(), ref[5])
    for _ in range(2):
        ctx.trajectory(7)
        assert np.array_equal(ctx.download(), ref[7])


def test_pipe_8192_chunked_property(gpu, monkeypatch):
    """8192^2 on one GPU (W = 1024, 1024 tiles): a run forced into 2-step
    launches; size-independent property: the last step solves the reference
    residual, R(w_n+1; w_n) / R(w_n; w_n) < 1e-13.  dt = 0.05 * 1024 / N keeps
    the 1024^2 configuration's CFL number: with dt = 0.05 the reference
    scheme itself turns v negative at the boundary (dt > 2h) and reaches NaN
    within a few steps at N >= 4096 (oracle)."""
    N, T = 8192, 3
    monkeypatch.setenv("BURG_STREAM_CHUNK", "2")
    ctx = make_ctx(N, dt=0.05 * 1024 / N)
    snaps, st, _, _ = ctx.run(np.ones(2 * N * N), T)
    assert st["engine"] == 2 and st["stream_launches"] == 2 and st["stream_w"] == 1024
    _, n0 = ctx.residual(snaps[:, T - 1], snaps[:, T - 1])
    _, n1 = ctx.residual(snaps[:, T], snaps[:, T - 1])
    assert n1 / n0 < 1e-13, (n1, n0)


def test_sweep_1024_bench_config_bitwise(gpu, orc):
    """The headline configuration's kernel (pipe_kernel<16, true>, 1024^2,
    the 9 training mu of get_snapshot_params, 256 workgroups): 3 steps per
    trajectory, each trajectory bit-equal to the oracle's march for its mu."""
    from finitedifference_amd.config import get_snapshot_params
    N, T = 1024, 3
    mus = get_snapshot_params()[:9]
    ctx = make_ctx(N)
    snaps, st = ctx.sweep(mus, T, w0=np.ones(2 * N * N))
    assert st["engine"] == 2 and st["stream_w"] == 16 and st["stream_launches"] == 1
    for mu, sn in zip(mus, snaps):
        ref, _, _ = orc.Problem(N, mu=tuple(mu)).fom(np.ones(2 * N * N), T)
        for j in range(T + 1):
            assert np.array_equal(sn[:, j], ref[j]), f"mu={mu} step {j}"


def test_sweep_wide_tiles_one_launch_per_mu(gpu, orc):
    """burg_sweep on wide tiles (no sweep kernel): one launch per mu, each
    trajectory bit-equal to the oracle."""
    N, ny, T = 600, 130, 3
    mus = [(4.25, 0.015), (5.19, 0.026), (5.5, 0.03)]
    P0 = orc.Problem(N, ny, Ly=100.0 * ny / N, allow_nonsquare=True)
    ctx = FOMContext_for(N, ny, engine="pipe", stream_w=128)
    ctx.set_problem(P0.grid_x, P0.grid_y, P0.dt, P0.mu, allow_nonsquare=True)
    snaps, st = ctx.sweep(mus, T, w0=np.ones(P0.m))
    assert st["stream_w"] == 128 and st["stream_launches"] == 3
    for mu, sn in zip(mus, snaps):
        P = orc.Problem(N, ny, mu=mu, Ly=100.0 * ny / N, allow_nonsquare=True)
        ref, _, _ = P.fom(np.ones(P.m), T)
        for j in range(T + 1):
            assert np.array_equal(sn[:, j], ref[j]), f"mu={mu} step {j}"


@pytest.mark.parametrize("engine", ["pipe", "stream"])
def test_nan_in_w0_raises_enan(gpu, engine):
    """A NaN planted in w0 makes the march report BURG_ENAN (SURVEY.md 5,
    failure detection) instead of silently writing NaN snapshots."""
    from finitedifference_amd._lib import BurgersError, BURG_ENAN
    N = 96
    ctx = make_ctx(N, engine=engine)
    w0 = np.ones(2 * N * N)
    w0[N * 40 + 17] = np.nan
    with pytest.raises(BurgersError) as ei:
        ctx.run(w0, 2)
    assert ei.value.code == BURG_ENAN
    snaps, st, _, _ = ctx.run(np.ones(2 * N * N), 2)  # the context stays usable
    assert st["nonfinite_diagonals"] == 0 and np.isfinite(snaps).all()


def test_slab_wide_rows_two_processes_one_gpu(gpu, orc, tmp_path):
    """Multi-GPU slabs with 8192-wide rows (the per-GPU row length of BASELINE
    config 4), rehearsed as 2 processes on one GPU (each limited to 512 tiles,
    so both grids are resident together -> wide tiles): the assembled
    trajectory is the single-domain march bit for bit."""
    N, ny, T, world = 8192, 256, 3, 2
    dt = 0.05 * 1024 / N  # the 1024^2 CFL (see test_pipe_8192_chunked_property)
    _run_slabs(tmp_path, N, T, world, SLAB_NY=ny, SLAB_TILES=512, SLAB_DT=repr(dt))
    widths = {open(os.path.join(tmp_path, f"slab{r}.w")).read() for r in range(world)}
    assert widths == {"32"}, widths
    from finitedifference_amd.dist import assemble_snaps
    parts = [np.load(os.path.join(tmp_path, f"slab{r}.npy")) for r in range(world)]
    snaps = assemble_snaps(parts, N, ny)
    P = orc.Problem(N, ny, dt=dt, Ly=100.0 * ny / N, allow_nonsquare=True)
    ref, _, _ = P.fom(np.ones(P.m), T)
    for j in range(T + 1):
        assert np.array_equal(snaps[:, j], ref[j]), f"step {j}"


@pytest.mark.parametrize("W,N,T,world", [(128, 1024, 12, 2), (256, 1024, 6, 2), (1024, 2048, 2, 2),
                                         (128, 768, 10, 3)])
def test_slab_wide_tile_steady_blocks_one_gpu(gpu, orc, tmp_path, W, N, T, world):
    """Slabs whose tiles run the steady / steady-edge blocks (W > 64) on the
    strips that write the halo ring -- the multi-GPU bench's tiling (W = 256
    at 4096 x 4096 per GPU).  The halo ring's row is the whole slab width, so
    a steady block must still stop at its own tile's last column (a block
    that ran on into the next tile's slots stalled both ranks at step 0).
    Two or three processes share the GPU (W forced, all grids resident; the
    middle one of three both reads and writes a halo ring, and 768 / 128 = 6
    tiles per strip leave its second workgroup half full); the assembled
    trajectory is the single-domain march bit for bit."""
    dt = 0.05 * 1024 / N
    _run_slabs(tmp_path, N, T, world, SLAB_W=W, SLAB_DT=repr(dt))
    widths = {open(os.path.join(tmp_path, f"slab{r}.w")).read() for r in range(world)}
    assert widths == {str(W)}, widths
    assert _halo_modes(tmp_path, world) == [(0 if r == 0 else 2, 0 if r == world - 1 else 2)
                                            for r in range(world)]
    from finitedifference_amd.dist import assemble_snaps
    parts = [np.load(os.path.join(tmp_path, f"slab{r}.npy")) for r in range(world)]
    snaps = assemble_snaps(parts, N, N)
    P = orc.Problem(N, dt=dt)
    ref, _, _ = P.fom(np.ones(P.m), T)
    for j in range(T + 1):
        assert np.array_equal(snaps[:, j], ref[j]), f"step {j}"


def test_fine750_eight_uneven_slabs_one_gpu(gpu, orc, tmp_path):
    """SURVEY.md 8(d) C5 parity case on one GPU: 750^2 over 8 slab processes
    (uneven 94/93-row slabs), 500 steps with snap_every=100: assembled
    snapshots bit-equal to the single-domain march and within 1e-10 of the
    author's Fine HDM slices (F/run_fom.py:28, F/predict_mu_5.19e+00_2.60e-02_hprom.pickle)."""
    N, T, world = 750, 500, 8
    _run_slabs(tmp_path, N, T, world, timeout=300, SLAB_SNAP_EVERY=100)
    from finitedifference_amd.dist import assemble_snaps, slab_rows
    assert [slab_rows(N, world, r)[1] for r in range(world)] == [94] * 6 + [93] * 2
    parts = [np.load(os.path.join(tmp_path, f"slab{r}.npy")) for r in range(world)]
    snaps = assemble_snaps(parts, N, N)
    g = golden("author_pickles.npz")
    n = N * N
    U = snaps[:n].reshape(N, N, -1)
    for k in range(6):
        assert rel(U[N // 2, :, k], g["fine_u_row"][k]) <= REF_TOL
        assert rel(U[:, N // 2, k], g["fine_u_col"][k]) <= REF_TOL
    single = make_ctx(N).run(np.ones(2 * n), T, snap_every=100)[0]
    assert np.array_equal(snaps, single)


def test_trajectory_from_initial_is_repeatable(gpu, orc):
    """burg_trajectory (the bench's unit of work): from the uploaded w0 every
    time, or continuing from the resident state; final states = oracle."""
    N, T = 144, 11
    P = orc.Problem(N)
    ref, _, _ = P.fom(np.ones(P.m), 2 * T)
    ctx = make_ctx(N)
    ctx.upload(np.ones(P.m))
    for _ in range(2):
        st = ctx.trajectory(T)
        assert st["engine"] == 2 and st["steps"] == T
        assert np.array_equal(ctx.download(), ref[T])
    ctx.trajectory(T, from_initial=False)
    assert np.array_equal(ctx.download(), ref[2 * T])


# ------------------------------------------------------ parameter sweep --
SWEEP_MUS = [(4.25, 0.015), (5.19, 0.026), (5.5, 0.03), (4.875, 0.0225), (4.56, 0.019)]


@pytest.mark.parametrize("N,ny,W,T,nmu,group", [
    (64, 64, 16, 5, 3, 0), (130, 70, 8, 4, 5, 2), (96, 200, 16, 3, 4, 0), (40, 64, 8, 9, 2, 1),
    (136, 136, 0, 6, 12, 0)])
def test_sweep_each_trajectory_bitwise(gpu, orc, monkeypatch, N, ny, W, T, nmu, group):
    """burg_sweep: every trajectory of the sweep (own mu, all from w0) is
    bit-equal to the oracle's sequential march for that mu -- across the
    state resets and coefficient switches inside one launch, across launch
    groups (forced small groups; 12 mu > the 10 a launch holds)."""
    if group:
        monkeypatch.setenv("BURG_SWEEP_GROUP", str(group))
    mus = [SWEEP_MUS[i % len(SWEEP_MUS)] for i in range(nmu)]
    mus = [(m1 + 0.01 * i, m2) for i, (m1, m2) in enumerate(mus)]
    P0 = orc.Problem(N, ny, Ly=100.0 * ny / N, allow_nonsquare=(N != ny))
    w0 = state_after(orc, P0, 2)
    ctx = FOMContext_for(N, ny, engine="pipe", stream_w=W)
    ctx.set_problem(P0.grid_x, P0.grid_y, P0.dt, P0.mu, allow_nonsquare=(N != ny))
    snaps, st = ctx.sweep(mus, T, w0=w0)
    assert st["engine"] == 2 and st["steps"] == nmu * T
    for mu, sn in zip(mus, snaps):
        P = orc.Problem(N, ny, mu=mu, Ly=100.0 * ny / N, allow_nonsquare=(N != ny))
        ref, _, _ = P.fom(w0, T)
        for j in range(T + 1):
            assert np.array_equal(sn[:, j], ref[j]), f"mu={mu} step {j}"
    # the last trajectory's final state is left resident
    assert np.array_equal(ctx.download(), snaps[-1][:, T])


def test_sweep_snap_every_and_resident(gpu, orc):
    N, T = 64, 9
    mus = SWEEP_MUS[:3]
    ctx = make_ctx(N, engine="pipe")
    w0 = np.ones(ctx.m)
    full, _ = ctx.sweep(mus, T, w0=w0)
    sub, _ = ctx.sweep(mus, T, w0=w0, snap_every=3)
    for a, b in zip(full, sub):
        assert np.array_equal(a[:, ::3], b)
    none, st = ctx.sweep(mus, T, w0=w0, keep_snaps=False)
    assert none is None and st["steps"] == 3 * T
    assert np.array_equal(ctx.download(), full[-1][:, T])


def test_sweep_api_matches_single_runs(gpu, tmp_path):
    """hypernet2D.load_or_compute_snaps_sweep writes the same cache files
    (reference names, C/hypernet2D.py:3081-3105) with the same snapshots as
    one load_or_compute_snaps call per mu."""
    from finitedifference_amd import hypernet2D as H
    N, T = 50, 6
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    w0 = np.ones(2 * N * N)
    mus = SWEEP_MUS[:4]
    a = H.load_or_compute_snaps_sweep(mus, gx, gy, w0, 0.05, T, snap_folder=str(tmp_path / "a"))
    for mu, sa in zip(mus, a):
        sb = H.load_or_compute_snaps(mu, gx, gy, w0, 0.05, T, snap_folder=str(tmp_path / "b"))
        assert np.array_equal(sa, sb)
    again = H.load_or_compute_snaps_sweep(mus, gx, gy, w0, 0.05, T, snap_folder=str(tmp_path / "a"))
    for x, y in zip(a, again):
        assert np.array_equal(x, y)


# ------------------------------------------------ ECSW training matrix --
@pytest.mark.parametrize("tag", ["n16", "n24"])
def test_ecsw_matrix_vs_reference_and_oracle(gpu, orc, tag):
    """compute_ECSW_training_matrix_2D on the GPU (burg_ecsw_matrix): bit-equal
    to the oracle restatement and within round-off of the reference's own
    output (its res2D / exact_jac2D callbacks, the driver's offset sampling)."""
    from finitedifference_amd import hypernet2D as H
    g = golden("ref_ecsw.npz")
    N, T, m1, m2, dt, npod, f = g[f"{tag}_meta"]
    N, T, f = int(N), int(T), int(f)
    sn, basis = g[f"{tag}_snaps"], g[f"{tag}_basis"]
    s_use, s_prev = sn[:, 3:T:f], sn[:, 0:T - 3:f]
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    C = H.compute_ECSW_training_matrix_2D(s_use, s_prev, basis, None, None, gx, gy, dt, (m1, m2))
    P = orc.Problem(N, mu=(m1, m2), dt=dt)
    assert np.array_equal(C, P.ecsw_matrix(s_use, s_prev, basis))
    assert rel(C, g[f"{tag}_C"]) <= 1e-14


def test_ecsw_matrix_multiblock_bitwise(gpu, orc):
    """Several 256-column blocks, ragged last block, many basis vectors."""
    N, ns, npod = 300, 3, 17
    P = orc.Problem(N)
    rng = np.random.default_rng(1234557)
    snaps = rng.uniform(1.0, 6.0, (P.m, ns))
    prev = rng.uniform(1.0, 6.0, (P.m, ns))
    basis = np.linalg.qr(rng.standard_normal((P.m, npod)))[0]
    ctx = make_ctx(N)
    C, st = ctx.ecsw_matrix(snaps, prev, basis, return_stats=True)
    assert C.shape == (npod * ns, N * N) and st["steps"] == ns
    assert np.array_equal(C, P.ecsw_matrix(snaps, prev, basis))


def _variant_case(name):
    """(callable, args, host decoder pair) of one ECSW decoder variant on the
    ref_ecsw_variants.npz problem (tests/ecsw_models.py rebuilds its models)."""
    import ecsw_models as em
    from finitedifference_amd import hypernet2D as H
    from finitedifference_amd import rom_decoders as rd
    g = golden("ref_ecsw_variants.npz")
    N, T, m1, m2, dt, rp, rs, eps, k = g["meta"]
    N, T, k = int(N), int(T), int(k)
    sn, B, B2, P, Q = g["snaps"], g["basis"], g["basis2"], g["P"], g["Q"]
    s_use, s_prev = sn[:, 3:T:3], sn[:, 0:T - 3:3]
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    scaler = em.scaler_of(g["qp_raw"])
    common = (gx, gy, dt, (m1, m2))
    kind, _, kt = name.partition("_")
    if kind == "nn":
        tree = em.kdtree_of(P)
        qmap = rd.RBFNearestNeighborsMap(tree, P, Q, eps, k, scaler, kt)
        return (H.compute_ECSW_training_matrix_2D_rbf_nearest_neighbors,
                (s_use, s_prev, B, B2, eps, k, tree, P, Q, None, None) + common + (scaler, kt),
                qmap, g, s_use, s_prev, N, (m1, m2), dt)
    if kind == "glob":
        W = g[f"glob_{kt}_W"]
        return (H.compute_ECSW_training_matrix_2D_rbf_global,
                (s_use, s_prev, B, B2, W, P, Q, None, None) + common + (scaler, eps, kt),
                rd.RBFGlobalMap(W, P, eps, scaler, kt), g, s_use, s_prev, N, (m1, m2), dt)
    if kind == "gp":
        gp = em.gp_of(P, Q, *g["gp_par"])
        return (H.compute_ECSW_training_matrix_2D_gp,
                (s_use, s_prev, B, B2, gp, None, None) + common + (scaler,),
                rd.GPMap(gp, scaler), g, s_use, s_prev, N, (m1, m2), dt)
    approx, jacf = em.nn_decoder_of(B, B2, g["rnm_A"], g["rnm_b"])
    return (H.compute_ECSW_training_matrix_2D_rnm,
            (s_use, s_prev, B, approx, jacf, None, None) + common, (approx, jacf), g, s_use,
            s_prev, N, (m1, m2), dt)


ECSW_VARIANTS = (["nn_gaussian", "nn_imq", "nn_linear", "nn_multiquadric", "glob_gaussian",
                  "glob_imq", "glob_linear", "glob_multiquadric", "glob_matern", "gp", "rnm"])


@pytest.mark.parametrize("name", ECSW_VARIANTS)
def test_ecsw_decoder_variants_vs_reference(gpu, orc, capsys, name):
    """compute_ECSW_training_matrix_2D_{rbf_nearest_neighbors, rbf_global, gp,
    rnm} (C/hypernet2D.py:2742-3072) on the GPU against the reference's own
    matrices (tests/golden/ref_ecsw_variants.npz): the same per-snapshot
    residual prints (3 significant digits) and C within 1e-10 rel-L2 for the
    float64 POD-RBF / POD-GP refits (device products vs numpy: round-off
    only).  rnm: 2e-6 -- its refit is the caller's float32 torch code on
    the host CPU, whose float32 products round differently from machine to
    machine (4.7e-7 on the GPU box's host, 5.7e-10 where the fixture was
    made, the rest being the reference's float32 fluxes in res2D /
    exact_jac2D where the kernel uses float64).  Then the block itself:
    C equals the oracle's ECSW restatement on the refit state, Jacobian and
    previous state (the kernel is the oracle's op order; the decoded inputs
    differ from host numpy's by round-off, so 1e-12)."""
    import re
    fn, args, dec, g, s_use, s_prev, N, mu, dt = _variant_case(name)
    C, coords = fn(*args, return_coords=True)
    printed = [float(m.group(3)) for m in
               map(re.compile(r"^(Initial|Final)( reconstruction)? residual: (\S+)$").match,
                   capsys.readouterr().out.splitlines()) if m]
    assert printed == list(g[f"{name}_resid"]), printed
    assert C.shape == g[f"{name}_C"].shape
    assert rel(C, g[f"{name}_C"]) <= (2e-6 if name == "rnm" else 1e-10)
    P = orc.Problem(N, mu=mu, dt=dt)
    B, B2 = g["basis"], g["basis2"]
    npod = B.shape[1]
    for i in range(s_use.shape[1]):
        y = coords[:, i]
        if name == "rnm":
            import torch
            yt = torch.tensor(y, dtype=torch.float)
            w = dec[0](yt).detach().numpy().astype(np.float64)
            V = dec[1](yt).detach().numpy().astype(np.float64)
        else:
            w, V = B @ y + B2 @ dec.q(y), B + B2 @ dec.dq(y)
        Ci = P.ecsw_matrix(w[:, None], s_prev[:, i:i + 1], V)
        assert rel(C[i * npod:(i + 1) * npod], Ci) <= 1e-12, i


def test_ecsw_block_device_refuses_host_memory(gpu):
    """burg_ecsw_block_device takes device pointers only: a host array is
    BURG_EINVAL with a message (never a GPU fault)."""
    import torch
    from finitedifference_amd import _lib
    ctx = make_ctx(16)
    dev = torch.device("cuda", 0)
    w = torch.ones(ctx.m, dtype=torch.float64, device=dev)
    Vt = torch.zeros((2, ctx.m), dtype=torch.float64, device=dev)
    out = torch.empty((2, ctx.m // 2), dtype=torch.float64, device=dev)
    host = np.zeros(ctx.m)
    code = ctx._L.burg_ecsw_block_device(ctx._h, host.ctypes.data, w.data_ptr(), 2, Vt.data_ptr(),
                                         out.data_ptr(), None)
    assert code == _lib.BURG_EINVAL
    assert "state" in ctx._L.burg_last_error().decode()
    with pytest.raises(ValueError):
        ctx.ecsw_block_device(w.cpu(), w, Vt, out)
    assert ctx.ecsw_block_device(w, w, Vt, out) >= 0.0
    assert torch.count_nonzero(out).item() == 0  # J V = 0 for V = 0


# ------------------------------------------------ LSPG PROM --
@pytest.mark.parametrize("tag", ["n16", "n24", "n32"])
def test_lspg_vs_reference_and_oracle(gpu, orc, tag):
    """inviscid_burgers_implicit2D_LSPG on the GPU (burg_lspg: fused J.basis +
    Gram kernel, Cholesky of the normal equations) against the reference's own
    ROM trajectory (tests/golden/ref_lspg.npz: POD bases of reference
    snapshots, out-of-sample mu) and the oracle restatement (lstsq).  Bars:
    same Gauss-Newton count every step; trajectory within 1e-10 rel-L2 (the
    north-star fp64 bar); reduced coordinates consistent with the snapshots."""
    from finitedifference_amd import hypernet2D as H
    g = golden("ref_lspg.npz")
    N, T, m1, m2, dt, npod = g[f"{tag}_meta"]
    N, T, npod = int(N), int(T), int(npod)
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    B = g[f"{tag}_basis"]
    snaps, (nits, tj, tr, tl), red = H.inviscid_burgers_implicit2D_LSPG(
        gx, gy, np.ones(2 * N * N), dt, T, (m1, m2), B, verbose=False, return_coords=True)
    assert snaps.shape == (2 * N * N, T + 1) and red.shape == (npod, T + 1)
    assert nits == int(g[f"{tag}_its"].sum())
    assert rel(snaps, g[f"{tag}_snaps"]) <= REF_TOL
    P = orc.Problem(N, dt=dt, mu=(m1, m2))
    osnaps, oits, _ = P.lspg(np.ones(2 * N * N), T, B)
    assert np.array_equal(oits, g[f"{tag}_its"])
    assert rel(snaps, osnaps) <= REF_TOL
    assert rel(B @ red, snaps) <= 1e-14
    assert min(tj, tr, tl) >= 0.0


def test_lspg_step_counts_and_rank_errors(gpu, orc):
    """Per-step counts/relative norms through the context API; a ragged grid
    (N not a multiple of the 16-cell tile), npod at the 127 cap, and the
    errors the boundary promises (non-square grid, npod out of range,
    rank-deficient basis)."""
    from finitedifference_amd import _lib
    N, T = 37, 4
    P = orc.Problem(N, mu=(4.9, 0.021))
    sn, _, _ = P.fom(np.ones(P.m), 12, solver="march")
    S = sn.T
    rng = np.random.default_rng(7)
    B = np.linalg.qr(np.hstack([S, rng.standard_normal((P.m, 127 - S.shape[1]))]))[0]
    ctx = make_ctx(N, mu=(4.9, 0.021))
    snaps, red, its, rels, times, st = ctx.lspg(np.ones(P.m), T, B)
    osnaps, oits, orels = P.lspg(np.ones(P.m), T, B)
    assert np.array_equal(its, oits)
    assert int((its - 1).sum()) <= st["newton_updates"] <= int(its.sum())
    assert rel(snaps, osnaps) <= REF_TOL
    assert np.allclose(rels, orels, rtol=1e-6, atol=1e-12)
    with pytest.raises(_lib.BurgersError):
        ctx.lspg(np.ones(P.m), 1, np.zeros((P.m, 128)))
    with pytest.raises(_lib.BurgersError) as ei:  # J basis rank-deficient: two equal columns
        ctx.lspg(np.ones(P.m), 1, np.hstack([B[:, :3], B[:, :1]]))
    assert ei.value.code == _lib.BURG_ENOCONV, str(ei.value)
    sq = make_ctx(N, ny=N + 3)
    with pytest.raises(_lib.BurgersError):
        sq.lspg(np.ones(2 * N * (N + 3)), 1, np.ones((2 * N * (N + 3), 2)))


def test_streamed_snapshot_cache(gpu, tmp_path):
    """load_or_compute_snaps(stream=True) writes the snapshots from HBM straight
    into a memory map of the cache file: same file (np.save format, reference
    name) and same array as the reference's array-then-np.save flow
    (stream=False); no partial file left; mmap=True hands back the map."""
    from finitedifference_amd import hypernet2D as H
    N, T = 64, 9
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    w0 = np.ones(2 * N * N)
    mu = (4.56, 0.019)
    a = H.load_or_compute_snaps(mu, gx, gy, w0, 0.05, T, snap_folder=str(tmp_path / "s"),
                                stream=True)
    b = H.load_or_compute_snaps(mu, gx, gy, w0, 0.05, T, snap_folder=str(tmp_path / "n"),
                                stream=False)
    assert np.array_equal(a, b) and a.shape == (2 * N * N, T + 1)
    fa = H.param_to_snap_fn(mu, str(tmp_path / "s"))
    fb = H.param_to_snap_fn(mu, str(tmp_path / "n"))
    assert open(fa, "rb").read() == open(fb, "rb").read()
    assert sorted(os.listdir(tmp_path / "s")) == [os.path.basename(fa)]
    c = H.load_or_compute_snaps(mu, gx, gy, w0, 0.05, 5, snap_folder=str(tmp_path / "s"), mmap=True)
    assert isinstance(c.base, np.memmap) or isinstance(c, np.memmap)
    assert np.array_equal(c, a[:, :6])
    d = H.load_or_compute_snaps(mu, gx, gy, w0, 0.05, T, snap_folder=str(tmp_path / "m"),
                                stream=True, mmap=True)
    assert np.array_equal(d, a)
    mus = SWEEP_MUS[:3]
    sw = H.load_or_compute_snaps_sweep(mus, gx, gy, w0, 0.05, T, snap_folder=str(tmp_path / "w"),
                                       stream=True)
    sn = H.load_or_compute_snaps_sweep(mus, gx, gy, w0, 0.05, T, snap_folder=str(tmp_path / "x"),
                                       stream=False)
    for x, y, mu_ in zip(sw, sn, mus):
        assert np.array_equal(x, y)
        assert (open(H.param_to_snap_fn(mu_, str(tmp_path / "w")), "rb").read() ==
                open(H.param_to_snap_fn(mu_, str(tmp_path / "x")), "rb").read())


# ----------------------------------------------------- POD --
def _pod_mode_mask(s, rel_floor=1e-6, rel_gap=1e-6):
    """modes the SVD determines to ~1e-10: not noise, separated from neighbours"""
    gap = np.full(s.size, np.inf)
    gap[:-1] = np.minimum(gap[:-1], s[:-1] - s[1:])
    gap[1:] = np.minimum(gap[1:], s[:-1] - s[1:])
    return (s > rel_floor * s[0]) & (gap > rel_gap * s[0])


@pytest.mark.parametrize("tag", ["n16", "n24"])
def test_pod_vs_reference_and_oracle(gpu, orc, tag):
    """POD on the GPU (burg_pod: rocSOLVER QR + SVD of R) against the
    reference's np.linalg.svd output and sklearn's seeded randomized_svd
    (tests/golden/ref_pod.npz).  Bars: singular values to 1e-12 of s[0];
    well-determined modes (above 1e-6 s[0], gaps above 1e-6 s[0]) to 1e-8
    after sign normalisation; U orthonormal; S reproduced by U U^T S."""
    from finitedifference_amd import hypernet2D as H
    g = golden("ref_pod.npz")
    S = g[f"{tag}_S"]
    u, s = H.POD(S, method="svd")
    assert u.shape == g[f"{tag}_u"].shape and s.shape == g[f"{tag}_s"].shape
    assert np.allclose(s, g[f"{tag}_s"], rtol=0, atol=1e-12 * s[0])
    ur = orc.svd_flip_u(g[f"{tag}_u"])
    keep = _pod_mode_mask(g[f"{tag}_s"])
    assert keep.sum() >= 8
    assert np.max(np.abs(u[:, keep] - ur[:, keep])) < 1e-8
    assert np.max(np.abs(u.T @ u - np.eye(u.shape[1]))) < 1e-12
    assert rel(u @ (u.T @ S), S) < 1e-13
    uo, so = orc.pod_svd(S)
    assert np.max(np.abs(u[:, keep] - uo[:, keep])) < 1e-8
    u10, s10 = H.POD(S, num_modes=10, method="rsvd", random_state=0)
    assert u10.shape == (S.shape[0], 10)
    assert np.allclose(s10, g[f"{tag}_sr"], rtol=1e-8, atol=0)
    assert np.all(np.abs(np.sum(u10 * g[f"{tag}_ur"], axis=0)) > 1 - 1e-8)


def test_pod_tall_ragged_and_errors(gpu):
    """A tall matrix with sizes off every tile (m = 2*37^2, ns = 45) against
    numpy's SVD, and the error paths (k out of range, wide matrix)."""
    from finitedifference_amd import _lib
    from finitedifference_amd import hypernet2D as H
    rng = np.random.default_rng(11)
    m, ns = 2 * 37 * 37, 45
    S = rng.standard_normal((m, 8)) @ rng.standard_normal((8, ns)) + 1e-3 * rng.standard_normal((m, ns))
    u, s = H.POD(S, num_modes=20, method="svd")
    un, sn, _ = np.linalg.svd(S, full_matrices=False)
    assert np.allclose(s, sn, rtol=1e-12)
    u, s = u[:, :20], s[:20]
    keep = _pod_mode_mask(sn[:20], rel_floor=1e-12, rel_gap=1e-8)
    assert np.all(np.abs(np.sum(u[:, keep] * un[:, :20][:, keep], axis=0)) > 1 - 1e-9)
    ur, sr = H.POD(S, num_modes=8, method="rsvd", random_state=3)  # the rank-8 part
    assert np.allclose(sr, sn[:8], rtol=1e-10)
    assert np.all(np.abs(np.sum(ur * un[:, :8], axis=0)) > 1 - 1e-10)
    with pytest.raises(ValueError):
        H.POD(S.T)
    L = _lib.load()
    out = np.zeros((m, 1))
    sv = np.zeros(1)
    assert L.burg_pod(0, m, ns, _lib.dptr(np.ascontiguousarray(S)), 0, _lib.dptr(out),
                      _lib.dptr(sv), None) == _lib.BURG_EINVAL


@pytest.mark.parametrize("k,nrand,occ", [(95, 105, 2), (95, 105, 1), (100, 128, 2), (30, 40, 2),
                                         (120, 129, 2)])
def test_pod_rsvd_mfma_products_vs_rocblas(gpu, monkeypatch, k, nrand, occ):
    """The randomized SVD on the tall-skinny MFMA products (default for
    nrand <= 128: S used in place, thin matrices row-major) against the same
    algorithm on rocBLAS dgemm (BURG_POD_GEMM=rocblas) and against numpy's
    SVD, on sizes off every tile (m = 2*61^2 rows, ns = 301 columns, ranks
    padded to 48 / 112 / 128; nrand = 129 takes the library path either
    way; occ: BURG_POD_GEMM_OCC, one or two workgroups per CU).  Bars:
    singular values to 1e-11 relative between the two paths and
    to 1e-9 of numpy's for the leading half of the modes; well-separated modes equal up
    to 1e-9 in |cos|."""
    from finitedifference_amd import _lib
    rng = np.random.default_rng(5)
    m, ns = 2 * 61 * 61, 301
    decay = np.exp(-np.arange(160) / 12.0)
    S = (rng.standard_normal((m, 160)) * decay) @ rng.standard_normal((160, ns))
    S += 1e-9 * rng.standard_normal((m, ns))
    S = np.ascontiguousarray(S)
    # column-major (ns x nrand): its C-order transpose
    omega = np.ascontiguousarray(np.random.default_rng(7).standard_normal((nrand, ns)))
    L = _lib.load()

    monkeypatch.setenv("BURG_POD_GEMM_OCC", str(occ))

    def run(path):
        monkeypatch.setenv("BURG_POD_GEMM", path)
        U = np.zeros((m, k))
        sv = np.zeros(k)
        rc = L.burg_pod_rsvd(0, m, ns, _lib.dptr(S), k, nrand, 4, _lib.dptr(omega), _lib.dptr(U),
                             _lib.dptr(sv), None)
        assert rc == 0, L.burg_last_error().decode()
        return U, sv

    um, sm = run("mfma")
    ur, sr = run("rocblas")
    assert np.allclose(sm, sr, rtol=1e-11, atol=0)
    sn = np.linalg.svd(S, compute_uv=False)
    lead = min(k // 2, 40)  # the rsvd approximation's own error grows toward mode k
    assert np.allclose(sm[:lead], sn[:lead], rtol=1e-9, atol=0)
    keep = _pod_mode_mask(sr, rel_floor=1e-8, rel_gap=1e-4)
    assert keep.sum() >= min(k, 30)
    assert np.all(np.abs(np.sum(um[:, keep] * ur[:, keep], axis=0)) > 1 - 1e-9)
    assert np.max(np.abs(um[:, keep] - ur[:, keep])) < 1e-7  # same svd_flip signs
    assert np.max(np.abs(um.T @ um - np.eye(k))) < 1e-12


def test_lspg_solve_kernel_path(gpu, monkeypatch):
    """BURG_LSPG_SOLVE=kernel selects the one-workgroup Cholesky kernel instead
    of rocSOLVER potrf/potrs: same Gauss-Newton counts and trajectory (within
    round-off) on the reference's n24 case, and the rank check still fires
    (BURG_ENOCONV, not a HIP error)."""
    from finitedifference_amd import _lib
    from finitedifference_amd import hypernet2D as H
    g = golden("ref_lspg.npz")
    N, T, m1, m2, dt, npod = g["n24_meta"]
    N, T = int(N), int(T)
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    B = g["n24_basis"]
    a, (na, *_) = H.inviscid_burgers_implicit2D_LSPG(gx, gy, np.ones(2 * N * N), dt, T, (m1, m2), B,
                                                     verbose=False)
    monkeypatch.setenv("BURG_LSPG_SOLVE", "kernel")
    b, (nb, *_) = H.inviscid_burgers_implicit2D_LSPG(gx, gy, np.ones(2 * N * N), dt, T, (m1, m2), B,
                                                     verbose=False)
    assert na == nb == int(g["n24_its"].sum())
    assert rel(b, a) <= 1e-13 and rel(b, g["n24_snaps"]) <= REF_TOL
    with pytest.raises(_lib.BurgersError) as ei:
        H.inviscid_burgers_implicit2D_LSPG(gx, gy, np.ones(2 * N * N), dt, 1, (m1, m2),
                                           np.hstack([B[:, :3], B[:, :1]]), verbose=False)
    assert ei.value.code == _lib.BURG_ENOCONV, str(ei.value)  # the rank check, not a HIP error


# ------------------------------------------------- drop-in host surface --
def test_run_fom_main_dropin(gpu, tmp_path, monkeypatch, capsys):
    """run_fom.main (C/run_fom.py:9-52) end to end in a scratch cwd: the
    cache file and the hdm_snaps file carry the reference's names, the
    trajectory is the reference's (ref_small n50: 50^2, 20 steps, mu =
    (4.75, 0.02)), the per-step lines of C/hypernet2D.py:122 are printed, and
    a second call is served from the cache."""
    from finitedifference_amd import run_fom
    g = golden("ref_small.npz")
    monkeypatch.chdir(tmp_path)
    el, snaps = run_fom.main(4.75, 0.02, num_cells=50, num_steps=20)
    out = capsys.readouterr().out
    assert " ... Working on timestep 19" in out and "Computing new snaps" in out
    assert os.path.exists("param_snaps/mu1_4.75+mu2_0.02.npy")
    assert os.path.exists("hdm_snaps_mu1_4.75_mu2_0.020.npy")
    ref = g["n50_snaps"]
    assert snaps.shape == ref.shape
    assert max(rel(snaps[:, j], ref[:, j]) for j in range(1, 21)) <= REF_TOL
    el2, snaps2 = run_fom.main(4.75, 0.02, num_cells=50, num_steps=20)
    assert "Loading saved snaps" in capsys.readouterr().out
    assert np.array_equal(snaps2, snaps)
    assert np.array_equal(np.load("hdm_snaps_mu1_4.75_mu2_0.020.npy"), snaps)


@pytest.mark.parametrize("N", [16, 64])
def test_reference_residual_jacobian_newton_api(gpu, N):
    """The reference's operator-level API (drop-in names): res2D_alt and
    res2D (C/hypernet2D.py:2512,2468), exact_jac2D(w) @ x (:2627) with the
    operators the reference builds (get_ops), and newton_raphson (:1811) with
    the JacobianOperator -- against the reference's own outputs (ref_ops)."""
    from finitedifference_amd import hypernet2D as H
    g = golden("ref_ops.npz")
    mu = tuple(g[f"n{N}_mu"])
    w, wp, x = g[f"n{N}_w"], g[f"n{N}_wp"], g[f"n{N}_x"]
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    Dxec, Dyec, JDxec, JDyec, Eye = H.get_ops(gx, gy)
    r = H.inviscid_burgers_res2D_alt(w, gx, gy, 0.05, wp, mu, JDxec, JDyec)
    assert rel(r, g[f"n{N}_res"]) <= 1e-15
    r1 = H.inviscid_burgers_res2D(w, gx, gy, 0.05, wp, mu, Dxec, Dyec)
    assert rel(r1, g[f"n{N}_res1d"]) <= 1e-15
    J = H.inviscid_burgers_exact_jac2D(w, 0.05, JDxec, JDyec, Eye)
    assert rel(J @ x, g[f"n{N}_jx"]) <= 1e-14
    assert rel(J.solve(g[f"n{N}_res"]), g[f"n{N}_solve"]) <= 1e-13
    # one implicit step by the reference's Newton with the drop-in callbacks
    res = lambda v: H.inviscid_burgers_res2D_alt(v, gx, gy, 0.05, wp, mu)  # noqa: E731
    jac = lambda v: H.inviscid_burgers_exact_jac2D(v, 0.05, grid_x=gx, grid_y=gy)  # noqa: E731
    wn, norms = H.newton_raphson(res, jac, wp, 100, 1e-12)
    assert norms[-1] / norms[0] < 1e-12 and len(norms) <= 8
    ctx = make_ctx(N, mu)
    snaps, _, _, _ = ctx.run(wp, 1)
    assert rel(wn, snaps[:, 1]) <= 1e-13


def test_plot_snaps_slices(gpu):
    """plot_snaps (C/hypernet2D.py:3147-3180): the plotted lines are the
    mid-row / mid-column slices of u the author pickled."""
    import matplotlib
    matplotlib.use("Agg")
    from finitedifference_amd import hypernet2D as H
    N, T = 64, 4
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    snaps = H.inviscid_burgers_implicit2D(gx, gy, np.ones(2 * N * N), 0.05, T, (5.19, 0.026),
                                          verbose=0)
    fig, ax1, ax2 = H.plot_snaps(gx, gy, snaps, [0, T], label="HDM")
    U = snaps[:N * N].reshape(N, N, -1)
    assert np.array_equal(ax1.lines[1].get_ydata(), U[N // 2, :, T])
    assert np.array_equal(ax2.lines[1].get_ydata(), U[:, N // 2, T])
    assert ax1.lines[0].get_label() == "HDM"
    fig2, _, _ = H.plot_snaps(gx, gy, snaps, [2], fig_ax=(fig, ax1, ax2))
    assert fig2 is fig and len(ax1.lines) == 3


def test_snapshot_cache_snap_every_and_short_files(gpu, tmp_path):
    """load_or_compute_snaps: a thinned (snap_every > 1) run is cached under a
    name of its own, never under the reference's per-step name; a cached file
    with too few columns is returned short, as the reference does
    (C/hypernet2D.py:3138, np.load(fn)[:, :num_steps+1]), and recomputed only
    with recompute_short=True."""
    from finitedifference_amd import hypernet2D as H
    N, T = 32, 12
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    w0 = np.ones(2 * N * N)
    d = str(tmp_path / "ps")
    thin = H.load_or_compute_snaps((5.19, 0.026), gx, gy, w0, 0.05, T, snap_folder=d,
                                   snap_every=4)
    assert thin.shape[1] == 4
    assert os.path.exists(os.path.join(d, "mu1_5.19+mu2_0.026+every4.npy"))
    assert not os.path.exists(os.path.join(d, "mu1_5.19+mu2_0.026.npy"))
    full = H.load_or_compute_snaps((5.19, 0.026), gx, gy, w0, 0.05, T, snap_folder=d)
    assert full.shape[1] == T + 1 and np.array_equal(full[:, ::4], thin)
    np.save(os.path.join(d, "mu1_5.19+mu2_0.026.npy"), full[:, :5])  # a short cache
    short = H.load_or_compute_snaps((5.19, 0.026), gx, gy, w0, 0.05, T, snap_folder=d)
    assert np.array_equal(short, full[:, :5])
    again = H.load_or_compute_snaps((5.19, 0.026), gx, gy, w0, 0.05, T, snap_folder=d,
                                    recompute_short=True)
    assert np.array_equal(again, full)
    assert np.load(os.path.join(d, "mu1_5.19+mu2_0.026.npy")).shape[1] == T + 1


def test_direct_npy_writer(gpu, tmp_path, monkeypatch):
    """burg_run_npy (load_or_compute_snaps(direct=True)): the file the
    library writes through its pinned buffers and writer pool (pwrite at
    each row block's offset, blocks finishing out of order) is np.save's
    .npy of the reference's snapshot matrix, byte-identical to np.save of
    burg_run's matrix; snap_every, multi-block files and 1 / 3 / 8 writers
    included."""
    from finitedifference_amd import hypernet2D as H
    N, T = 300, 9
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    w0 = np.ones(2 * N * N)
    ref = make_ctx(N).run(w0, T)[0]
    np.save(tmp_path / "ref.npy", ref)
    d = str(tmp_path / "ps")
    got = H.load_or_compute_snaps((5.19, 0.026), gx, gy, w0, 0.05, T, snap_folder=d, direct=True)
    fn = os.path.join(d, "mu1_5.19+mu2_0.026.npy")
    assert open(fn, "rb").read() == open(tmp_path / "ref.npy", "rb").read()
    assert np.array_equal(got, ref)
    monkeypatch.setenv("BURG_NPY_BLOCK_ROWS", "7001")  # 26 row blocks, ragged last one
    ctx = make_ctx(N)
    st = ctx.run_to_npy(w0, T, str(tmp_path / "thin.npy"), snap_every=4)
    assert np.array_equal(np.load(tmp_path / "thin.npy"), ref[:, ::4])
    assert st["loop_ms"] > 0 and st["flush_ms"] > 0
    monkeypatch.setenv("BURG_NPY_BLOCK_ROWS", "997")  # 181 blocks
    for nw in ("1", "3", "8"):
        monkeypatch.setenv("BURG_NPY_WRITERS", nw)
        ctx.run_to_npy(w0, T, str(tmp_path / f"w{nw}.npy"))
        assert open(tmp_path / f"w{nw}.npy", "rb").read() == open(tmp_path / "ref.npy", "rb").read(), nw


def test_direct_npy_writer_failure_returns(gpu, tmp_path, monkeypatch):
    """A failed row-block copy in burg_run_npy (forced with the test knob
    BURG_TEST_FAIL_NPY_BLOCK on block 0, a middle block and the last) returns
    BURG_EHIP instead of hanging in the writer drain (the taken
    pinned buffer goes back to the pool); the context then writes a correct
    file.  burg_run_npy_ex: a file made for another matrix is refused
    (NPY_EXISTING), and a slab-less context with NPY_GLOBAL writes the same
    bytes as burg_run_npy."""
    from finitedifference_amd._lib import BurgersError, BURG_EHIP, BURG_EINVAL
    from finitedifference_amd.dist import create_npy
    from finitedifference_amd.solver import NPY_EXISTING, NPY_GLOBAL
    N, T = 200, 5
    ctx = make_ctx(N)
    w0 = np.ones(2 * N * N)
    ref = ctx.run(w0, T)[0]
    monkeypatch.setenv("BURG_NPY_BLOCK_ROWS", "4001")  # 20 row blocks
    for blk in ("0", "7", "19"):
        monkeypatch.setenv("BURG_TEST_FAIL_NPY_BLOCK", blk)
        with pytest.raises(BurgersError) as ei:
            ctx.run_to_npy(w0, T, str(tmp_path / "f.npy"))
        assert ei.value.code == BURG_EHIP and "row block copy failed" in str(ei.value)
    monkeypatch.delenv("BURG_TEST_FAIL_NPY_BLOCK")
    ctx.run_to_npy(w0, T, str(tmp_path / "ok.npy"))
    assert np.array_equal(np.load(tmp_path / "ok.npy"), ref)
    ctx.run_to_npy(w0, T, str(tmp_path / "g.npy"), flags=NPY_GLOBAL)
    assert open(tmp_path / "g.npy", "rb").read() == open(tmp_path / "ok.npy", "rb").read()
    create_npy(str(tmp_path / "e.npy"), 2 * N * N, T + 1)
    ctx.run_to_npy(w0, T, str(tmp_path / "e.npy"), flags=NPY_GLOBAL | NPY_EXISTING)
    assert open(tmp_path / "e.npy", "rb").read() == open(tmp_path / "ok.npy", "rb").read()
    create_npy(str(tmp_path / "bad.npy"), 2 * N * N, T)  # one column short
    with pytest.raises(BurgersError) as ei:
        ctx.run_to_npy(w0, T, str(tmp_path / "bad.npy"), flags=NPY_GLOBAL | NPY_EXISTING)
    assert ei.value.code == BURG_EINVAL
