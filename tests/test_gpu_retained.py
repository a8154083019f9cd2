"""GPU parity of the retained snapshot sets of burg_trajectory_ex (VERDICT r03
item 3; SURVEY.md section 7 "needs a snap_every stride").

The reference keeps every state of a trajectory (C/hypernet2D.py:89-90,126).
burg_trajectory_ex keeps them in HBM: every state while they fit, or with
snap_every = k the states 0, k, 2k, ... in retained windows of the ring
(burg_internal.h ring_pos) -- for grids whose whole
trajectory does not fit (the 8192 x 2048 and 16384 x 2048 per-GPU slabs of
the multi-GPU bench).  Every retained column must equal the oracle's march
bit for bit (and burg_run's snapshot matrix with the same snap_every).
"""
import numpy as np
import pytest

from test_gpu_regime import _ctx, _problem, planted_w0

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nx,ny,W,T,k", [
    (256, 128, 16, 13, 5),    # narrow, windows of 80 diagonals 80 apart (just disjoint)
    (200, 70, 8, 20, 9),      # W = 8, partial strip, T % k != 0
    (256, 128, 16, 13, 3),    # narrow, k W < W + 64: every state kept (plain ring)
    (2048, 130, 64, 12, 2),   # W = 64, k = 2: windows back to back
    (1000, 130, 128, 13, 4),  # blocks of 16, partial last tile
    (700, 200, 256, 11, 2),   # the 4096^2 bench's width, ragged tiles and strips
    (2100, 64, 1024, 7, 3),   # the 8192^2 grid's width
])
def test_trajectory_snap_every_bitwise(gpu, orc, nx, ny, W, T, k):
    P = _problem(orc, nx, ny)
    w0 = planted_w0(nx, ny)
    ref, _, _ = P.fom(w0, T)
    ctx = _ctx(nx, ny, engine="pipe", stream_w=W)
    ctx.upload(w0)
    st = ctx.trajectory(T, snap_every=k)
    assert st["stream_w"] == W and st["stream_launches"] == 1
    first, count, stride = ctx.retained()
    assert (first, count, stride) == (0, T // k + 1, k)
    snaps = ctx.trajectory_snaps()
    assert snaps.shape == (P.m, T // k + 1)
    for j in range(count):
        assert np.array_equal(snaps[:, j], ref[j * k]), f"state {j * k}"
    assert np.array_equal(ctx.download(), ref[T])
    # the same columns as burg_run's snapshot matrix with this snap_every
    run, _, _, _ = ctx.run(w0, T, snap_every=k)
    assert np.array_equal(run, snaps)
    # a column range, and a continuation from the resident state
    ctx.upload(w0)
    ctx.trajectory(T, snap_every=k)
    part = ctx.trajectory_snaps(1, count - 1)
    assert np.array_equal(part, snaps[:, 1:])
    ctx.trajectory(T, from_initial=False, snap_every=k)
    ref2, _, _ = P.fom(ref[T], T)
    cont = ctx.trajectory_snaps()
    for j in range(count):
        assert np.array_equal(cont[:, j], ref2[j * k]), f"continued state {j * k}"
    assert np.array_equal(ctx.download(), ref2[T])
    ctx.close()


def test_trajectory_snaps_to_device(gpu, orc):
    """burg_trajectory_copy into device memory (a torch tensor on the
    context's GPU: the input of a device-resident POD) equals the host copy."""
    import torch
    nx, ny, T, k = 700, 200, 9, 3
    P = _problem(orc, nx, ny)
    ref, _, _ = P.fom(np.ones(P.m), T)
    ctx = _ctx(nx, ny, engine="pipe", stream_w=256)
    ctx.upload(np.ones(P.m))
    ctx.trajectory(T, snap_every=k)
    host = ctx.trajectory_snaps()
    dev = torch.empty((P.m, T // k + 1), dtype=torch.float64, device="cuda:0")
    ctx.trajectory_snaps(out=dev)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), host)
    for j in range(T // k + 1):
        assert np.array_equal(host[:, j], ref[j * k])
    # a wider tensor: columns land at its first T // k + 1 columns
    wide = torch.zeros((P.m, T // k + 3), dtype=torch.float64, device="cuda:0")
    ctx.trajectory_snaps(out=wide)
    torch.cuda.synchronize()
    assert np.array_equal(wide[:, :T // k + 1].cpu().numpy(), host)
    assert not wide[:, T // k + 1:].any()
    ctx.close()


@pytest.mark.parametrize("W,cap", [(256, 4), (1024, 5)])
def test_capped_ring_retains_last_states(gpu, orc, monkeypatch, W, cap):
    """snap_every = 1 with a ring capped below the trajectory (BURG_RING_CAP
    stands in for free HBM): the last cap + 1 states stay resident and equal
    the oracle's; the older ones are reported as gone."""
    monkeypatch.setenv("BURG_RING_CAP", str(cap))
    nx, ny, T = (700, 200, 11) if W == 256 else (2100, 64, 12)
    P = _problem(orc, nx, ny)
    w0 = planted_w0(nx, ny)
    ref, _, _ = P.fom(w0, T)
    ctx = _ctx(nx, ny, engine="pipe", stream_w=W)
    ctx.upload(w0)
    ctx.trajectory(T)
    first, count, stride = ctx.retained()
    assert (first, count, stride) == (T - cap, cap + 1, 1)
    snaps = ctx.trajectory_snaps()
    for j in range(count):
        assert np.array_equal(snaps[:, j], ref[first + j]), f"state {first + j}"
    ctx.close()


def test_trajectory_plan_and_errors(gpu):
    from finitedifference_amd._lib import BurgersError
    nx, ny, T = 512, 256, 20
    ctx = _ctx(nx, ny, engine="pipe", stream_w=64)
    k, n, b = ctx.trajectory_plan(T, 0)  # auto: a small trajectory fits -> every state
    assert k == 1 and n == T + 1 and b > 0
    k, n, b = ctx.trajectory_plan(T, 4)
    assert k == 4 and n == T // 4 + 1
    with pytest.raises(BurgersError):
        ctx.retained()  # nothing resident yet
    ctx.upload(np.ones(2 * nx * ny))
    ctx.trajectory(T, snap_every=4)
    with pytest.raises(BurgersError):
        ctx.trajectory_snaps(0, T)  # beyond the retained columns
    ctx.run(np.ones(2 * nx * ny), 3)  # reuses the ring: the record is gone
    with pytest.raises(BurgersError):
        ctx.retained()
    ctx.close()


def test_n8_slab_keeps_every_10th_state(gpu, orc):
    """The N = 8 bench rank's shape (16384 x 2048, W = 512, dt = 0.05 *
    1024 / 16384) over 500 steps with snap_every = 10: 51 retained states (27
    GB) in ONE launch; states 0, 100, ..., 500 bit-equal to the oracle's march,
    and the launch's rate within 2 % of the same trajectory on the capped
    plain ring, both measured here."""
    nx, ny, T, k = 16384, 2048, 500, 10
    dt = 0.05 * 1024 / nx
    P = _problem(orc, nx, ny, dt=dt)
    ref = P.march_traj(np.ones(P.m), T, snap_every=100)
    ctx = _ctx(nx, ny, dt=dt)
    ctx.upload(np.ones(P.m))
    ctx.trajectory(T)  # warm: the capped plain ring
    plain = ctx.trajectory(T)
    st = ctx.trajectory(T, snap_every=k)
    st2 = ctx.trajectory(T, snap_every=k)
    assert st["stream_w"] == 512 and st["stream_launches"] == 1
    assert ctx.retained() == (0, T // k + 1, k)
    r_plain = nx * ny * T / plain["loop_ms"] / 1e6
    r_ret = nx * ny * T / min(st["loop_ms"], st2["loop_ms"]) / 1e6
    print(f"\n16384x2048 x 500: plain capped ring {r_plain:.1f}, snap_every=10 {r_ret:.1f} "
          f"Gcell-updates/s ({r_ret / r_plain:.3f})")
    assert np.array_equal(ctx.download(), ref[-1])
    for j in range(0, T // k + 1, 10):
        col = ctx.trajectory_snaps(j, 1)
        assert np.array_equal(col[:, 0], ref[j // 10]), f"state {j * k}"
    ctx.close()


def test_set_engine_drops_the_retained_record(gpu):
    """burg_set_engine frees the ring a trajectory left resident: the record
    goes with it (BURG_ESTATE), instead of a copy reading a freed ring
    (ADVICE r04)."""
    from finitedifference_amd._lib import BURG_ESTATE, BurgersError
    nx, ny, T = 512, 130, 6
    ctx = _ctx(nx, ny, engine="pipe", stream_w=64)
    ctx.upload(np.ones(2 * nx * ny))
    ctx.trajectory(T, snap_every=2)
    assert ctx.retained() == (0, T // 2 + 1, 2)
    ctx.set_engine("pipe", stream_w=128)  # a new plan: the ring is freed
    with pytest.raises(BurgersError) as ei:
        ctx.retained()
    assert ei.value.code == BURG_ESTATE
    with pytest.raises(BurgersError) as ei:
        ctx.trajectory_snaps(0, 1)
    assert ei.value.code == BURG_ESTATE
    ctx.close()
