"""One rank of the slab tests in tests/test_gpu_parity.py (not a test module):
its slab of an NX x NY grid (default N x N), T steps from w0 = 1, on device 0,
rendezvous over gloo; writes its slab snapshot matrix.

    slab_worker.py N T OUTDIR [run|sweep|residual|failstate]
    env: SLAB_NY (rows, default N), SLAB_W (pipe tile width, 0 = plan),
         SLAB_TILES (tiles target per rank), SLAB_SNAP_EVERY (default 1),
         SLAB_DT (default 0.05); writes slab{rank}.npy, .w (tile width) and
         .halo (halo ring placement: in, out; 1 host, 2 device)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


SWEEP_MUS = [(4.25, 0.015), (5.19, 0.026), (5.5, 0.03)]


def main():
    N, T, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    sweep = len(sys.argv) > 4 and sys.argv[4] == "sweep"  # mu sweep (burg_sweep) instead
    ny = int(os.environ.get("SLAB_NY", N))
    W = int(os.environ.get("SLAB_W", "0"))
    tiles = int(os.environ.get("SLAB_TILES", "0"))
    every = int(os.environ.get("SLAB_SNAP_EVERY", "1"))
    dt = float(os.environ.get("SLAB_DT", "0.05"))
    import torch.distributed as dist
    from finitedifference_amd.dist import make_slab_context, slab_state
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ctx = make_slab_context(N, ny, rank, world, device=0, dist=dist, stream_w=W,
                            tiles_target=tiles)
    gx = np.linspace(0, 100, N + 1)
    gy = np.linspace(0, 100.0 * ny / N, ny + 1)
    ctx.set_problem(gx, gy, dt, (5.19, 0.026), allow_nonsquare=(ny != N))
    w0 = slab_state(np.ones(2 * N * ny), N, ny, rank, world)
    dist.barrier()
    mode = sys.argv[4] if len(sys.argv) > 4 else "run"
    if mode in ("failstate", "failone"):
        # BURG_TEST_FAIL_DEVICE_HALO=1: the first launch fails as a stalled
        # device halo ring would; the context must then refuse to launch.
        # failone (BURG_TEST_FAIL_DEVICE_HALO=R:1): only rank R's second
        # launch fails; its neighbours' waits must give up by themselves
        from finitedifference_amd._lib import BurgersError
        codes = []
        for _ in range(2 if mode == "failstate" else 3):
            try:
                ctx.run(w0, T)
                codes.append(0)
            except BurgersError as e:
                codes.append(e.code)
        with open(os.path.join(out, f"slab{rank}.codes"), "w") as f:
            f.write(" ".join(map(str, codes)))
        dist.barrier()
        ctx.close()
        dist.destroy_process_group()
        return
    if sweep:
        snaps, st = ctx.sweep(SWEEP_MUS, T, w0=w0, snap_every=every)
        assert st["engine"] == 2
        for j, sn in enumerate(snaps):
            np.save(os.path.join(out, f"slab{rank}_mu{j}.npy"), sn)
    else:
        snaps, st, _, _ = ctx.run(w0, T, snap_every=every)
        assert st["engine"] == 2
        np.save(os.path.join(out, f"slab{rank}.npy"), snaps)
        if mode == "residual":
            # the slab residual of the last step with the halo rows sent by
            # the rank below (burg_slab_residual + send/recv over gloo)
            from finitedifference_amd.dist import (exchange_halo_rows, slab_residual_norms,
                                                   top_row)
            rows = ctx.ny
            wT, wP = snaps[:, -1].copy(), snaps[:, -2].copy()
            got = exchange_halo_rows(np.concatenate((top_row(wT, N, rows), top_row(wP, N, rows))),
                                     N, rank, world, dist)
            halo = (None, None) if got is None else (got[:2 * N], got[2 * N:])
            r, ss = ctx.slab_residual(wT, wP, *halo)
            np.save(os.path.join(out, f"slab{rank}_res.npy"), r)
            g1, s1 = slab_residual_norms(ctx, wT, wP, dist)
            g0, s0 = slab_residual_norms(ctx, wP, wP, dist)
            with open(os.path.join(out, f"slab{rank}.norms"), "w") as f:
                f.write(" ".join(repr(x) for x in (ss, g1, s1, g0, s0)))
    with open(os.path.join(out, f"slab{rank}.w"), "w") as f:
        f.write(str(st["stream_w"]))
    import json
    with open(os.path.join(out, f"slab{rank}.stats"), "w") as f:
        json.dump({k: st[k] for k in ("ramp_ms", "halo_wait_ms", "south_waits_local",
                                      "south_waits_halo", "south_wait_ms_local",
                                      "south_wait_ms_halo", "bounds_checks", "bounds_hits",
                                      "loop_ms")}, f)
    with open(os.path.join(out, f"slab{rank}.halo"), "w") as f:
        f.write("%d %d" % ctx.halo_modes())
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
