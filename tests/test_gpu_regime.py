"""GPU parity in the regime the bench times (VERDICT r02 "pin the regime").

* The IEEE slow path: diagonals whose operands leave the short exact
  sequences' range [2^-900, 2^900) are recomputed with IEEE sqrt / division
  (cell_math.h).  Here it is forced with FINITE tiny and subnormal v planted in
  w0, on narrow (W = 16, run and sweep kernels) and wide (W = 256, 1024) tiles
  and on the streaming engine; every snapshot must equal the oracle's
  sequential march (orc_march_step, IEEE arithmetic on the host) bit for bit.
* Long trajectories: 1024^2 x 500 steps (run_fom.main's unit, dt = 0.05) and
  the bench's own 4096^2 x 500 steps at dt = 0.0125 (burg_trajectory, one
  launch over a 134 GB ring) against the oracle's row-pipelined march
  (orc_march_traj_par: the same loop body, bit-identical to orc_march_step).
  These cover the slow path as it arises naturally: the inlet column's v
  shrinks by 1/(1 + dt u/dx) per step and leaves the fast window after ~480
  steps.
* Ring wrap across launch boundaries at wide tile widths (BURG_STREAM_CHUNK
  forces several launches over a ring that wraps).
Reference time loop: C/hypernet2D.py:72-131.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# BENCH_r02.json engine.ieee_diagonals of the driver's bench (4096^2,
# dt = 0.0125, 500 steps, W = 256, burg_trajectory): the test below makes the
# same call, so the count must be the same.
BENCH_4096_IEEE_DIAGONALS = 578752

TINY_V = [2.0 ** -950, 2.0 ** -1000, 5e-320, 2.0 ** -1070, 0.0, 2.0 ** -901, 2.0 ** -899,
          1e-310, 2.0 ** -1022]


def planted_w0(nx, ny, width=40):
    """w0 = 1 with finite tiny and subnormal v in the first `width` columns
    (every row) and subnormal u in columns 60-63.  The block starts at the
    inlet column, whose west inflow is zero, so its v stays tiny over the
    whole trajectory (inflows from tiny neighbours), as the inlet column's v
    does in the bench's last ~40 steps: thousands of cells per step outside
    the fast path's range, subnormals among them (checked on the CPU oracle)."""
    w = np.ones((2, ny, nx))
    cols = np.arange(0, min(nx, width))
    vals = np.array(TINY_V)
    w[1][:, cols] = vals[(np.arange(ny)[:, None] + cols[None, :]) % len(vals)]
    w[0][:, 60:64] = 3e-315
    return w.ravel()


def _ctx(nx, ny, dt=0.05, mu=(5.19, 0.026), **eng):
    from finitedifference_amd.solver import FOMContext
    ctx = FOMContext(nx, ny, **eng)
    ctx.set_problem(np.linspace(0, 100, nx + 1), np.linspace(0, 100.0 * ny / nx, ny + 1), dt,
                    mu, allow_nonsquare=(nx != ny))
    return ctx


def _problem(orc, nx, ny, dt=0.05, mu=(5.19, 0.026)):
    return orc.Problem(nx, ny, dt=dt, mu=mu, Ly=100.0 * ny / nx, allow_nonsquare=(nx != ny))


@pytest.mark.parametrize("nx,ny,engine,W,T", [
    (256, 128, "pipe", 16, 7), (200, 70, "pipe", 8, 6), (700, 200, "pipe", 256, 5),
    (1500, 100, "pipe", 1024, 3), (300, 130, "stream", 0, 6)])
def test_ieee_slow_path_planted_bitwise(gpu, orc, nx, ny, engine, W, T):
    P = _problem(orc, nx, ny)
    w0 = planted_w0(nx, ny)
    ref, _, _ = P.fom(w0, T)
    ctx = _ctx(nx, ny, engine=engine, stream_w=W)
    snaps, st, _, _ = ctx.run(w0, T)
    if engine == "pipe":
        assert st["engine"] == 2 and st["stream_w"] == W
    assert st["ieee_diagonals"] > 0, "the planted values must take the IEEE path"
    assert st["nonfinite_diagonals"] == 0
    for j in range(T + 1):
        assert np.array_equal(snaps[:, j], ref[j]), f"step {j}"
    # subnormal states are produced and kept (no flush to zero)
    assert np.any((snaps[:, T] != 0) & (np.abs(snaps[:, T]) < 2.0 ** -1022))


@pytest.mark.parametrize("nx,ny,engine,W", [(64, 64, "pipe", 16), (256, 64, "pipe", 64),
                                           (128, 70, "stream", 0)])
def test_large_h_fast_window_bitwise(gpu, orc, nx, ny, engine, W):
    """The top of the fast window: with h_x = dt/4 / dx = 2^57
    (dt = 2^60, allowed by burg_set_problem's (0, 2^100) bound) and mu2 = 5.56
    the source term dt*0.02*exp(mu2*x) reaches 2^850 in the last columns, so
    Cu is far above 2^798 and q = 0.25 + h_x Cu + h_y Cv above 2^900 --
    outside the range sqrt_normal is verified on.  Those cells must take the
    IEEE path (ieee_diagonals > 0) and the step must equal the oracle's IEEE
    arithmetic bit for bit.  (Step 2 of this problem overflows: one step.)"""
    dt, mu = 2.0 ** 60, (5.19, 5.56)
    P = _problem(orc, nx, ny, dt=dt, mu=mu)
    ref, _, _ = P.fom(np.ones(P.m), 1)
    assert np.isfinite(ref[1]).all() and np.abs(ref[1]).max() > 2.0 ** 300
    ctx = _ctx(nx, ny, dt=dt, mu=mu, engine=engine, stream_w=W)
    snaps, st, _, _ = ctx.run(np.ones(P.m), 1)
    if engine == "pipe":
        assert st["engine"] == 2 and st["stream_w"] == W
    assert st["ieee_diagonals"] > 0 and st["nonfinite_diagonals"] == 0
    assert np.array_equal(snaps[:, 1], ref[1])


def test_ieee_slow_path_planted_sweep_bitwise(gpu, orc):
    """The narrow sweep kernel (pipe_kernel<16, true>, the 1024^2 sweep's)
    with the planted w0: each trajectory bit-equal to the oracle for its mu."""
    nx, ny, T = 256, 192, 6
    mus = [(4.25, 0.015), (5.19, 0.026), (5.5, 0.03)]
    w0 = planted_w0(nx, ny)
    ctx = _ctx(nx, ny, engine="pipe", stream_w=16)
    snaps, st = ctx.sweep(mus, T, w0=w0)
    assert st["stream_w"] == 16 and st["stream_launches"] == 1
    assert st["ieee_diagonals"] > 0
    for mu, sn in zip(mus, snaps):
        ref, _, _ = _problem(orc, nx, ny, mu=mu).fom(w0, T)
        for j in range(T + 1):
            assert np.array_equal(sn[:, j], ref[j]), f"mu={mu} step {j}"


def test_pipe_1024_500_steps_bitwise(gpu, orc):
    """run_fom.main's unit (1024^2, dt = 0.05, 500 steps, w0 = 1) on the
    planner's W = 16 tiles: every 10th state over the whole trajectory and
    every state of the last 50 steps bit-equal to the oracle's march; the
    trajectory takes the IEEE path on its own (v at the inlet column)."""
    N, T = 1024, 500
    P = orc.Problem(N)
    ref = P.march_traj(np.ones(P.m), T, snap_every=10)
    ctx = _ctx(N, N)
    snaps, st, _, _ = ctx.run(np.ones(P.m), T, snap_every=10)
    assert st["engine"] == 2 and st["stream_w"] == 16
    assert st["ieee_diagonals"] > 0 and st["nonfinite_diagonals"] == 0
    for j in range(T // 10 + 1):
        assert np.array_equal(snaps[:, j], ref[j]), f"step {10 * j}"
    tail = P.march_traj(ref[45], 50, snap_every=1)
    snaps2, _, _, _ = ctx.run(ref[45], 50)
    for j in range(51):
        assert np.array_equal(snaps2[:, j], tail[j]), f"step {450 + j}"
    ctx.upload(np.ones(P.m))
    st = ctx.trajectory(T)
    assert st["stream_launches"] == 1
    assert np.array_equal(ctx.download(), ref[-1])


def test_pipe_4096_bench_regime_bitwise(gpu, orc):
    """The bench's own unit of work: 4096^2, dt = 0.0125, 500 steps from
    w0 = 1 in ONE burg_trajectory launch (W = 256, 1024 tiles, the trajectory
    kept in a 134 GB HBM ring).  Its final state, and every 100th state of a
    burg_run of the same trajectory (chunked over a ring of a third of free
    HBM), equal the oracle's march bit for bit; the last step is checked on
    its own (orc_march_step(w_499) == w_500) and the IEEE-path count is the
    bench's."""
    N, T, dt = 4096, 500, 0.05 * 1024 / 4096
    P = orc.Problem(N, dt=dt)
    ref = P.march_traj(np.ones(P.m), T, snap_every=100)
    ctx = _ctx(N, N, dt=dt)
    ctx.upload(np.ones(P.m))
    st = ctx.trajectory(T)
    assert st["engine"] == 2 and st["stream_w"] == 256 and st["stream_tiles"] == 1024
    assert st["stream_launches"] == 1
    assert st["ieee_diagonals"] == BENCH_4096_IEEE_DIAGONALS
    assert st["nonfinite_diagonals"] == 0
    w500 = ctx.download()
    assert np.array_equal(w500, ref[-1])
    ctx.trajectory(T - 1)
    w499 = ctx.download()
    assert np.array_equal(P.march_step(w499), w500)
    snaps, st2, _, _ = ctx.run(np.ones(P.m), T, snap_every=100)
    for j in range(T // 100 + 1):
        assert np.array_equal(snaps[:, j], ref[j]), f"step {100 * j}"


@pytest.mark.parametrize("nx,ny,W,T,chunk", [(2100, 64, 1024, 12, 5), (700, 200, 256, 11, 4),
                                             (1000, 130, 128, 13, 3), (256, 128, 16, 13, 5)])
def test_chunked_ring_wrap_bitwise(gpu, orc, monkeypatch, nx, ny, W, T, chunk):
    """Trajectories split into several launches over a ring that wraps
    (BURG_STREAM_CHUNK; what every 8192^2 and 16384-wide trajectory does when
    its ring is capped at 85 % of free HBM): burg_run's snapshots and
    burg_trajectory's final state bit-equal to the oracle, from the planted
    w0 so the slow path crosses the launch boundaries too."""
    monkeypatch.setenv("BURG_STREAM_CHUNK", str(chunk))
    P = _problem(orc, nx, ny)
    w0 = planted_w0(nx, ny)
    ref, _, _ = P.fom(w0, T)
    ctx = _ctx(nx, ny, engine="pipe", stream_w=W)
    snaps, st, _, _ = ctx.run(w0, T)
    assert st["stream_w"] == W and st["stream_launches"] == math.ceil(T / chunk)
    for j in range(T + 1):
        assert np.array_equal(snaps[:, j], ref[j]), f"step {j}"
    ctx.upload(w0)
    st = ctx.trajectory(T)
    assert st["stream_launches"] == math.ceil(T / chunk)
    assert np.array_equal(ctx.download(), ref[T])
    st = ctx.trajectory(T, from_initial=False)  # continue: the ring wraps again
    ref2, _, _ = P.fom(ref[T], T)
    assert np.array_equal(ctx.download(), ref2[T])


@pytest.mark.parametrize("nx,ny,W,T", [(2048, 130, 64, 6), (512, 192, 16, 7), (2100, 100, 256, 5)])
def test_workgroup_order_bitwise(gpu, orc, monkeypatch, nx, ny, W, T):
    """Both workgroup orders of the pipe kernel (BURG_WG_MAP: 0 row-major, 1
    column-major -- the planner's choice when a strip has a multiple of 8
    workgroups, the per-GPU slabs of the N > 1 bench and the 1024^2 narrow
    tiles) produce the oracle's trajectory bit for bit, from the planted w0
    (slow path included); a ragged top strip and a partial last workgroup
    (2100 / 256 = 9 tiles) included."""
    P = _problem(orc, nx, ny)
    w0 = planted_w0(nx, ny)
    ref, _, _ = P.fom(w0, T)
    for order in ("0", "1"):
        monkeypatch.setenv("BURG_WG_MAP", order)
        ctx = _ctx(nx, ny, engine="pipe", stream_w=W)
        snaps, st, _, _ = ctx.run(w0, T)
        assert st["stream_w"] == W
        for j in range(T + 1):
            assert np.array_equal(snaps[:, j], ref[j]), f"order {order} step {j}"
        ctx.close()


@pytest.mark.parametrize("nx,ny,W,T,cap", [(2100, 64, 1024, 12, 5), (700, 200, 256, 11, 4),
                                           (1000, 130, 128, 13, 3), (256, 128, 16, 13, 5)])
def test_capped_ring_one_launch_bitwise(gpu, orc, monkeypatch, nx, ny, W, T, cap):
    """A trajectory ring capped below the trajectory's length (BURG_RING_CAP
    stands in for the free-memory cap of the 16384 x 2048 slab) wraps inside
    ONE launch: burg_trajectory's final state bit-equal to the oracle from the
    planted w0, and again when the trajectory continues over the same ring."""
    monkeypatch.setenv("BURG_RING_CAP", str(cap))
    P = _problem(orc, nx, ny)
    w0 = planted_w0(nx, ny)
    ref, _, _ = P.fom(w0, T)
    ctx = _ctx(nx, ny, engine="pipe", stream_w=W)
    ctx.upload(w0)
    st = ctx.trajectory(T)
    assert st["stream_w"] == W and st["stream_launches"] == 1
    assert np.array_equal(ctx.download(), ref[T])
    st = ctx.trajectory(T, from_initial=False)
    assert st["stream_launches"] == 1
    ref2, _, _ = P.fom(ref[T], T)
    assert np.array_equal(ctx.download(), ref2[T])
    ctx.close()


def test_trajectory_ring_not_stale_after_run(gpu, orc):
    """A ring re-allocated by burg_run after a trajectory must not be taken
    for a memory-capped one (ring_maxed was never cleared): the
    next trajectory gets a ring of its own size and runs in one launch."""
    N = 200
    P = orc.Problem(N)
    ctx = _ctx(N, N)
    ctx.upload(np.ones(P.m))
    ctx.trajectory(3)
    ctx.run(np.ones(P.m), 2)
    ctx.upload(np.ones(P.m))
    st = ctx.trajectory(40)
    assert st["stream_launches"] == 1
    ref, _, _ = P.fom(np.ones(P.m), 40)
    assert np.array_equal(ctx.download(), ref[40])


def test_slab_residual_single_context(gpu, orc):
    """burg_slab_residual on a whole-grid context (no halo) is burg_residual."""
    N = 130
    P = orc.Problem(N)
    ref, _, _ = P.fom(np.ones(P.m), 3)
    ctx = _ctx(N, N)
    r, ss = ctx.slab_residual(ref[3], ref[2])
    r2, nrm = ctx.residual(ref[3], ref[2])
    assert np.array_equal(r, r2) and np.array_equal(r, P.residual(ref[3], ref[2]))
    assert abs(math.sqrt(ss) - nrm) <= 1e-15 * nrm
    from finitedifference_amd._lib import BurgersError
    with pytest.raises(BurgersError):
        ctx.slab_residual(ref[3], ref[2], ref[3][:2 * N], ref[2][:2 * N])  # row 0 has no halo


@pytest.mark.parametrize("N,world,T", [(128, 2, 5), (150, 3, 4)])
def test_slab_residual_matches_single_domain(gpu, orc, tmp_path, N, world, T):
    """Multi-GPU runs check their own result (bench.py residual_check): each
    slab's residual of the last step, with the south halo rows sent by the
    rank below (torch.distributed send/recv, here gloo between processes
    sharing the box's GPU), equals the single-domain residual
    (C/hypernet2D.py:2512-2570) bit for bit; the global norm (sum over
    ranks) equals the single-domain norm to round-off, and the last step
    solves the residual (ratio < 1e-13)."""
    from test_gpu_parity import _run_slabs
    import os
    _run_slabs(tmp_path, N, T, world, mode="residual")
    from finitedifference_amd.dist import assemble_snaps, assemble_state
    parts = [np.load(os.path.join(tmp_path, f"slab{r}.npy")) for r in range(world)]
    snaps = assemble_snaps(parts, N, N)
    P = orc.Problem(N)
    ref, _, _ = P.fom(np.ones(P.m), T)
    assert np.array_equal(snaps[:, T], ref[T])
    res = assemble_state([np.load(os.path.join(tmp_path, f"slab{r}_res.npy"))
                          for r in range(world)], N, N)
    want = P.residual(ref[T], ref[T - 1])
    assert np.array_equal(res, want)
    norms = [[float(x) for x in open(os.path.join(tmp_path, f"slab{r}.norms")).read().split()]
             for r in range(world)]
    g1 = np.linalg.norm(want)
    g0 = np.linalg.norm(P.residual(ref[T - 1], ref[T - 1]))
    for ss, n1, s1, n0, s0 in norms:
        assert abs(n1 - g1) <= 1e-14 * g1 and abs(n0 - g0) <= 1e-14 * g0
    assert g1 / g0 < 1e-13
    assert abs(sum(x[0] for x in norms) - g1 ** 2) <= 1e-13 * g1 ** 2


def test_failed_slab_context_refuses_launches(gpu, tmp_path):
    """After a launch of a slab context fails (here the test hook makes the
    device halo ring fail as a stalled wait would), its halo rings hold stale
    step colours: the next launch is refused with BURG_ESTATE (the caller must
    recreate every rank's context, as bench.py does) instead of waiting on
    stale sentinels."""
    from test_gpu_parity import _run_slabs
    from finitedifference_amd._lib import BURG_EHIP, BURG_ESTATE
    import os
    _run_slabs(tmp_path, 96, 3, 2, mode="failstate", BURG_TEST_FAIL_DEVICE_HALO="1")
    for r in range(2):
        codes = [int(x) for x in open(os.path.join(tmp_path, f"slab{r}.codes")).read().split()]
        assert codes == [BURG_EHIP, BURG_ESTATE], (r, codes)


# The per-GPU shapes of the N > 1 bench lines (bench.py DEFAULT_SHAPES, DESIGN.md
# section 8) and the whole 8192^2 grid on one GPU, at full size and full length:
# the code path every rank of the driver's multi-GPU runs executes (rank 0's
# slab is exactly this single-context grid; the other ranks differ only in
# taking their south inflow from the halo ring).  dt = 0.05 * 1024 / nx, as the
# bench.  Each trajectory ring is capped by free HBM (268 / 537 GB would be
# needed) and wraps INSIDE the one launch.
@pytest.mark.parametrize("nx,ny,W", [(8192, 2048, 256), (16384, 2048, 512), (8192, 8192, 1024)])
def test_multi_gpu_rank_shape_500_steps_bitwise(gpu, orc, nx, ny, W):
    """VERDICT r03 item 1 (C/hypernet2D.py:112-129): 500 steps from w0 = 1 in
    ONE burg_trajectory launch at the planner's width; the final state equals
    the oracle's row-pipelined march bit for bit, the last step is checked on
    its own (orc_march_step(w_499) == w_500), and the IEEE-path count is
    recorded (the inlet column's v leaves the fast window in the last ~20
    steps at this CFL, as at 4096^2)."""
    import time
    T, dt = 500, 0.05 * 1024 / nx
    P = _problem(orc, nx, ny, dt=dt)
    t0 = time.perf_counter()
    ref = P.march_traj(np.ones(P.m), T, snap_every=T)
    t_orc = time.perf_counter() - t0
    ctx = _ctx(nx, ny, dt=dt)
    ctx.upload(np.ones(P.m))
    st = ctx.trajectory(T)
    print(f"\n{nx}x{ny}: W={st['stream_w']} tiles={st['stream_tiles']} "
          f"launches={st['stream_launches']} ieee_diagonals={st['ieee_diagonals']} "
          f"kernel {st['loop_ms']:.2f} ms ({nx * ny * T / st['loop_ms'] / 1e6:.1f} "
          f"Gcell-updates/s), oracle {t_orc:.1f} s")
    assert st["engine"] == 2 and st["stream_w"] == W
    assert st["stream_launches"] == 1
    assert st["nonfinite_diagonals"] == 0
    assert st["ieee_diagonals"] > 0
    w500 = ctx.download()
    assert np.array_equal(w500, ref[-1])
    st2 = ctx.trajectory(T - 1)
    assert st2["stream_launches"] == 1
    w499 = ctx.download()
    assert np.array_equal(P.march_step(w499), w500)
    ctx.close()


def test_one_rank_fails_at_a_later_launch(gpu, tmp_path):
    """ONE rank's launch k > 0 fails (test hook
    BURG_TEST_FAIL_DEVICE_HALO=1:1, rank 1's second launch) while its
    neighbour keeps launching: the neighbour's bounded waits give up by
    themselves (BURG_EHIP; T = 12 steps > the 8 halo slots, so the producer
    below must stall), and both contexts then refuse further launches
    (BURG_ESTATE) -- every rank ends failed, which bench.py's agreement turns
    into one collective fall-back (rehearsal: tools/gpu_r4.sh)."""
    from test_gpu_parity import _run_slabs
    from finitedifference_amd._lib import BURG_EHIP, BURG_ESTATE
    import os
    _run_slabs(tmp_path, 96, 12, 2, mode="failone", BURG_TEST_FAIL_DEVICE_HALO="1:1",
               BURG_SPIN_SECONDS="3")
    codes = [[int(x) for x in open(os.path.join(tmp_path, f"slab{r}.codes")).read().split()]
             for r in range(2)]
    assert codes[1] == [0, BURG_EHIP, BURG_ESTATE], codes
    assert codes[0] == [0, BURG_EHIP, BURG_ESTATE], codes
