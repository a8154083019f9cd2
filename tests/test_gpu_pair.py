"""GPU parity of the paired-halves W = 16 trajectory kernel (pipe.hip PAIR,
DESIGN.md section 4.1f): the tile's two 8-column halves marched by the same
lanes, one step apart -- the same cells in the same op order as the one-cell
kernel, so every state must be bit-identical to the oracle's sequential
march (orc_march_step, C/hypernet2D.py:72-131's implicit step) and to the
one-cell build (BURG_PAIR=0).

The kernel is the default for W = 16 sweeps and long trajectories
(profiles/r05/ab/pair: 1024^2 9-mu sweep 149 -> 172 Gcell/s); these tests
select each build explicitly with BURG_PAIR=1 / 0."""
import os

import numpy as np
import pytest

from test_gpu_regime import _ctx, _problem, planted_w0

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nx,ny,T", [
    (16, 64, 5),      # one tile
    (24, 20, 6),      # one partial tile, one partial strip (ragged B half)
    (256, 128, 13),   # 2 strips x 16 tiles, 4 workgroups per strip
    (200, 70, 9),     # partial last tile (columns 192-199: A real, B padding)
    (520, 130, 7),    # a partial 4-tile workgroup and a 2-row top strip
    (64, 300, 4),     # tall: 5 strips, one workgroup per strip
])
def test_paired_matches_oracle_and_one_cell_kernel(gpu, orc, monkeypatch, nx, ny, T):
    P = _problem(orc, nx, ny)
    w0 = planted_w0(nx, ny)
    ref, _, _ = P.fom(w0, T)
    got = {}
    for pair in ("1", "0"):
        monkeypatch.setenv("BURG_PAIR", pair)
        ctx = _ctx(nx, ny, engine="pipe", stream_w=16)
        snaps, st, _, _ = ctx.run(w0, T)
        assert st["stream_w"] == 16 and st["nonfinite_diagonals"] == 0
        assert (st["paired_launches"] > 0) == (pair == "1")
        for j in range(T + 1):
            assert np.array_equal(snaps[:, j], ref[j]), f"BURG_PAIR={pair} step {j}"
        ctx.upload(w0)
        ctx.trajectory(T)
        assert np.array_equal(ctx.download(), ref[T]), f"BURG_PAIR={pair} trajectory"
        got[pair] = st
        ctx.close()
    assert got["1"]["ieee_diagonals"] > 0  # the planted values take the IEEE path in both


def test_paired_1024_trajectory_rate_and_bits(gpu, orc, monkeypatch):
    """run_fom.main's unit at 1024^2: both builds bit-equal (final state and
    every 50th state) and the paired build's launch time reported."""
    N, T = 1024, 500
    P = orc.Problem(N)
    ref = P.march_traj(np.ones(P.m), T, snap_every=50)
    ms = {}
    for pair in ("0", "1"):
        monkeypatch.setenv("BURG_PAIR", pair)
        ctx = _ctx(N, N)
        ctx.upload(np.ones(P.m))
        ctx.trajectory(T)  # warm
        st = ctx.trajectory(T)
        assert st["stream_w"] == 16 and st["stream_launches"] == 1
        ms[pair] = st["loop_ms"]
        assert np.array_equal(ctx.download(), ref[-1]), f"BURG_PAIR={pair}"
        snaps = ctx.trajectory_snaps()
        for j in range(0, T + 1, 50):
            assert np.array_equal(snaps[:, j], ref[j // 50]), f"BURG_PAIR={pair} step {j}"
        ctx.close()
    print(f"\n1024^2 x 500 trajectory: one-cell {ms['0']:.3f} ms, paired {ms['1']:.3f} ms "
          f"({ms['0'] / ms['1']:.3f}x)")


def test_paired_slab_halo_two_processes_one_gpu(gpu, orc, tmp_path):
    """The paired kernel behind the multi-GPU halo stream: 2 slab processes on
    one GPU with W = 16 tiles (the top strip's north outflow of both halves
    goes through the consumer's device ring)."""
    from test_gpu_parity import _run_slabs
    N, T, world = 256, 9, 2
    _run_slabs(tmp_path, N, T, world, SLAB_W="16", BURG_PAIR="1")
    from finitedifference_amd.dist import assemble_snaps
    parts = [np.load(os.path.join(tmp_path, f"slab{r}.npy")) for r in range(world)]
    snaps = assemble_snaps(parts, N, N)
    ref, _, _ = orc.Problem(N).fom(np.ones(2 * N * N), T)
    for j in range(T + 1):
        assert np.array_equal(snaps[:, j], ref[j]), f"step {j}"


@pytest.mark.parametrize("nx,ny,nmu,T", [(256, 128, 3, 7), (200, 70, 4, 5), (1024, 1024, 9, 20)])
def test_paired_sweep_matches_one_cell_and_oracle(gpu, orc, monkeypatch, nx, ny, nmu, T):
    """burg_sweep on W = 16 tiles with paired halves: every trajectory of the
    mu sweep (back to back in one launch; B switches trajectory 8 diagonals
    after A) bit-equal to the oracle's march for its mu and to BURG_PAIR=0."""
    from finitedifference_amd.config import get_snapshot_params
    mus = get_snapshot_params()[:nmu]
    out = {}
    for pair in ("1", "0"):
        monkeypatch.setenv("BURG_PAIR", pair)
        ctx = _ctx(nx, ny, engine="pipe", stream_w=16)
        ctx.upload(np.ones(2 * nx * ny))
        snaps, st = ctx.sweep(mus, T)
        assert st["stream_w"] == 16
        assert (st["paired_launches"] > 0) == (pair == "1")
        out[pair] = snaps
        ctx.close()
    for j, mu in enumerate(mus):
        assert np.array_equal(out["1"][j], out["0"][j]), f"mu {j}"
        if nx <= 256:
            ref, _, _ = _problem(orc, nx, ny, mu=mu).fom(np.ones(2 * nx * ny), T)
            for q in range(T + 1):
                assert np.array_equal(out["1"][j][:, q], ref[q]), f"mu {mu} step {q}"


def _store_wave_build():
    from finitedifference_amd import _lib
    return "BURG_STORE_WAVE=0" not in _lib.build_flags()


@pytest.mark.parametrize("nx,ny,nmu,T", [(256, 128, 3, 7), (200, 70, 4, 5)])
def test_paired_sweep_uniform_initial_state_not_one(gpu, orc, monkeypatch, nx, ny, nmu, T):
    """The paired sweep kernel with its store wave restarts every trajectory
    from the uniform initial state as a constant (PipeArgs::w0c, DESIGN.md
    section 4.1g): with u0 = 1.5, v0 = 0.5 (not the reference's ones) every
    trajectory bit-equal to the oracle's and to the one-cell sweep."""
    from finitedifference_amd.config import get_snapshot_params
    mus = get_snapshot_params()[:nmu]
    n = nx * ny
    w0 = np.concatenate([np.full(n, 1.5), np.full(n, 0.5)])
    out = {}
    for pair in ("1", "0"):
        monkeypatch.setenv("BURG_PAIR", pair)
        ctx = _ctx(nx, ny, engine="pipe", stream_w=16)
        ctx.upload(w0)
        snaps, st = ctx.sweep(mus, T)
        assert (st["paired_launches"] > 0) == (pair == "1")
        out[pair] = snaps
        ctx.close()
    for j, mu in enumerate(mus):
        assert np.array_equal(out["1"][j], out["0"][j]), f"mu {j}"
        ref, _, _ = _problem(orc, nx, ny, mu=mu).fom(w0, T)
        for q in range(T + 1):
            assert np.array_equal(out["1"][j][:, q], ref[q]), f"mu {mu} step {q}"


def test_paired_sweep_refused_for_nonuniform_initial_state(gpu, orc, monkeypatch):
    """A non-uniform initial state has no constant to restart from: the sweep
    runs one-cell even with BURG_PAIR=1 (store-wave builds; a
    BURG_STORE_WAVE=0 build pairs it, its kernel keeps st0), and every
    trajectory is the oracle's."""
    from finitedifference_amd.config import get_snapshot_params
    nx, ny, nmu, T = 200, 70, 3, 5
    mus = get_snapshot_params()[:nmu]
    w0 = planted_w0(nx, ny)
    monkeypatch.setenv("BURG_PAIR", "1")
    ctx = _ctx(nx, ny, engine="pipe", stream_w=16)
    ctx.upload(w0)
    snaps, st = ctx.sweep(mus, T)
    ctx.close()
    assert (st["paired_launches"] > 0) == (not _store_wave_build())
    for j, mu in enumerate(mus):
        ref, _, _ = _problem(orc, nx, ny, mu=mu).fom(w0, T)
        for q in range(T + 1):
            assert np.array_equal(snaps[j][:, q], ref[q]), f"mu {mu} step {q}"
