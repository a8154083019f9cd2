"""GPU: host <-> device copies of caller memory through the library's pinned
bounce buffers (hostxfer.hip).

Round 4's intermittent hipErrorIllegalAddress surfaced at host-memory copies
(burg_download_state into a fresh np.empty, an upload from a per-call
std::vector) after calls that registered caller arrays and copied into them.
The library now hands the HIP runtime only its own pinned buffers and 1-D
copies.  These tests drive the copy paths with the allocation pattern of the
failing runs -- same-sized arrays freed and re-allocated at the same address,
many times -- and with multi-chunk (> 8 MB) and strided transfers, and check
every byte.
"""
import gc

import numpy as np
import pytest

from test_gpu_regime import _ctx

pytestmark = pytest.mark.gpu


def test_state_round_trip_multichunk_and_reallocated(gpu):
    nx, ny = 2048, 1100  # 36 MB per state: five 8 MB bounce chunks
    ctx = _ctx(nx, ny, engine="pipe")
    m = 2 * nx * ny
    rng = np.random.default_rng(5)
    for it in range(12):
        w = rng.standard_normal(m)
        ctx.upload(w)
        del w  # freed: the next array of this size lands at the same address
        gc.collect()
        w = rng.standard_normal(m)  # (a different array, maybe the same address)
        ctx.upload(w)
        back = ctx.download()
        assert np.array_equal(back, w), f"round trip {it}"
        del back
    ctx.close()


def test_snapshot_copies_strided_and_partial(gpu, orc):
    """Column ranges of the retained snapshot matrix (strided host rows, a
    partial last chunk) equal the full copy, repeatedly, into fresh arrays."""
    from test_gpu_regime import _problem, planted_w0
    nx, ny, T, k = 700, 200, 11, 2
    P = _problem(orc, nx, ny)
    w0 = planted_w0(nx, ny)
    ref, _, _ = P.fom(w0, T)
    ctx = _ctx(nx, ny, engine="pipe", stream_w=256)
    ctx.upload(w0)
    ctx.trajectory(T, snap_every=k)
    full = ctx.trajectory_snaps()
    for j in range(T // k + 1):
        assert np.array_equal(full[:, j], ref[j * k])
    for rep in range(6):
        for c0, n in ((0, 1), (1, 3), (2, 4), (5, 1), (0, T // k + 1)):
            part = ctx.trajectory_snaps(c0, n)
            assert np.array_equal(part, full[:, c0:c0 + n]), (rep, c0, n)
            del part
        gc.collect()
    # into a wider caller matrix: the columns land at its first n columns, the rest untouched
    out = np.full((P.m, T // k + 4), 7.0)
    from finitedifference_amd import _lib
    import ctypes
    _lib.check(ctx._L.burg_trajectory_copy(ctx._h, 1, 3, out.ctypes.data_as(ctypes.c_void_p),
                                           out.shape[1], 0))
    assert np.array_equal(out[:, :3], full[:, 1:4])
    assert (out[:, 3:] == 7.0).all()
    ctx.close()


def test_run_snapshots_and_residual_io_repeated(gpu, orc):
    """burg_run's snapshot matrix and the residual / J.x host arrays (all
    through the bounce buffers), many calls with re-allocated arrays."""
    nx, ny, T = 300, 260, 4
    from test_gpu_regime import _problem
    P = _problem(orc, nx, ny)
    ref, _, _ = P.fom(np.ones(P.m), T)
    ctx = _ctx(nx, ny, engine="pipe")
    for it in range(5):
        snaps, _, _, _ = ctx.run(np.ones(P.m), T)
        for j in range(T + 1):
            assert np.array_equal(snaps[:, j], ref[j]), (it, j)
        r, nrm = ctx.residual(snaps[:, T], snaps[:, T - 1])
        assert np.isfinite(nrm)
        del snaps, r
        gc.collect()
    ctx.close()
