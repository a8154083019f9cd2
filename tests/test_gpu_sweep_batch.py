"""GPU parity of the small-grid snapshot sweep (VERDICT r03 item 6;
DESIGN.md section 4.1e): the reference's drivers fill a snapshot set one
trajectory at a time (C/run_prom.py:59-71 over get_snapshot_params); at its
own 250^2 grid one trajectory leaves most of the chip idle, so burg_sweep runs
G trajectories side by side as separate domains of ONE launch.  Every
trajectory must equal the oracle's march for its mu bit for bit; the
device-resident variant (burg_sweep_device) must equal the host matrices, and
POD on the device-resident set must equal POD on the host copy."""
import numpy as np
import pytest

from test_gpu_regime import _ctx, _problem, planted_w0

pytestmark = pytest.mark.gpu

TRAIN_MUS = [(4.25, 0.015), (4.25, 0.0225), (4.25, 0.03), (4.875, 0.015), (4.875, 0.0225),
             (4.875, 0.03), (5.5, 0.015), (5.5, 0.0225), (5.5, 0.03)]


def test_side_by_side_sweep_250_bitwise(gpu, orc):
    """The reference's own configuration: 250^2, dt = 0.05, the 9 training
    mu, w0 = 1 -- one side-by-side launch; 40 steps per trajectory here (the
    oracle's cost), every state of every trajectory bitwise."""
    N, T = 250, 40
    ctx = _ctx(N, N)
    snaps, st = ctx.sweep(TRAIN_MUS, T, w0=np.ones(2 * N * N))
    assert st["engine"] == 2 and st["stream_launches"] == 1
    print(f"\n250^2 x 9 mu side by side: W={st['stream_w']} tiles={st['stream_tiles']} "
          f"kernel {st['loop_ms']:.3f} ms for {T} steps")
    for mu, sn in zip(TRAIN_MUS, snaps):
        ref, _, _ = _problem(orc, N, N, mu=mu).fom(np.ones(2 * N * N), T)
        for j in range(T + 1):
            assert np.array_equal(sn[:, j], ref[j]), f"mu={mu} step {j}"
    # the resident state is the last trajectory's final state
    assert np.array_equal(ctx.download(), snaps[-1][:, T])
    ctx.close()


@pytest.mark.parametrize("nx,ny,G,nmu,T,k", [(130, 70, 3, 5, 9, 1), (200, 150, 4, 4, 12, 3),
                                              (96, 64, 2, 3, 10, 5)])
def test_side_by_side_groups_bitwise(gpu, orc, monkeypatch, nx, ny, G, nmu, T, k):
    """Forced group sizes (BURG_SWEEP_BATCH): a short last group, ragged strips
    (70 and 150 rows: partial top strips inside the stacked grid), non-square
    grids, snap_every > 1 (retained windows), the planted w0 (slow path)."""
    monkeypatch.setenv("BURG_SWEEP_BATCH", str(G))
    mus = TRAIN_MUS[:nmu]
    w0 = planted_w0(nx, ny)
    ctx = _ctx(nx, ny)
    snaps, st = ctx.sweep(mus, T, w0=w0, snap_every=k)
    assert st["stream_launches"] == -(-nmu // G)
    for mu, sn in zip(mus, snaps):
        ref, _, _ = _problem(orc, nx, ny, mu=mu).fom(w0, T)
        assert sn.shape == (2 * nx * ny, T // k + 1)
        for j in range(T // k + 1):
            assert np.array_equal(sn[:, j], ref[j * k]), f"mu={mu} state {j * k}"
    ctx.close()


def test_sweep_device_and_pod_on_device(gpu):
    """burg_sweep_device leaves np.hstack(per-mu matrices) in HBM, equal to the
    host sweep; POD (rsvd, seeded) of that device tensor equals POD of the
    host copy (the C/run_prom.py:51-86 flow without the host round trip)."""
    import torch
    from finitedifference_amd import hypernet2D as H
    N, T = 250, 30
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    w0 = np.ones(2 * N * N)
    host = H.inviscid_burgers_implicit2D_sweep(gx, gy, w0, 0.05, T, TRAIN_MUS, verbose=0)
    S = np.hstack(host)
    Sd = H.inviscid_burgers_implicit2D_sweep(gx, gy, w0, 0.05, T, TRAIN_MUS, verbose=0,
                                             on_device=True)
    assert isinstance(Sd, torch.Tensor) and Sd.shape == S.shape
    assert np.array_equal(Sd.cpu().numpy(), S)
    u1, s1 = H.POD(S, 20, "rsvd", random_state=0)
    u2, s2 = H.POD(Sd, 20, "rsvd", random_state=0)
    assert np.allclose(s1, s2, rtol=1e-12, atol=0)
    assert np.allclose(u1, u2, rtol=0, atol=1e-10)
    # the serial path's device output too (BURG_SWEEP_BATCH=1 turns batching off)
    import os
    os.environ["BURG_SWEEP_BATCH"] = "1"
    try:
        from finitedifference_amd.solver import FOMContext
        ctx = FOMContext(N, N)
        ctx.set_problem(gx, gy, 0.05, TRAIN_MUS[0])
        Sd2, st = ctx.sweep_device(TRAIN_MUS[:3], T, w0=w0, snap_every=2)
        ref = np.hstack([h[:, ::2] for h in host[:3]])
        assert np.array_equal(Sd2.cpu().numpy(), ref)
        ctx.close()
    finally:
        del os.environ["BURG_SWEEP_BATCH"]
