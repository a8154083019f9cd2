"""Tile-count A/B at 1024^2 (BASELINE configs[1]): one 500-step trajectory
and the 9-mu sweep with the planner's default tiling against a larger tile
target (AB_TARGETS, e.g. "0 2048": W = 8 tiles, two workgroups and so two
compute waves per SIMD), best of `reps` launches by HIP events, with the
final states' checksums (the tiling must not change the bits)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.config import get_snapshot_params  # noqa: E402
from finitedifference_amd.solver import FOMContext  # noqa: E402

reps = int(os.environ.get("AB_REPS", "4"))
nx = int(os.environ.get("AB_NX", "1024"))
dt = 0.05 * 1024 / nx
mus = get_snapshot_params()[:9]
for tgt in [int(x) for x in os.environ.get("AB_TARGETS", "0 2048").split()]:
    ctx = FOMContext(nx, nx, engine="pipe", tiles_target=tgt)
    g = np.linspace(0, 100, nx + 1)
    ctx.set_problem(g, g, dt, (5.19, 0.026))
    ctx.upload(np.ones(ctx.m))
    ctx.trajectory(500)
    tr = []
    for _ in range(reps):
        st = ctx.trajectory(500)
        tr.append(st["loop_ms"])
    c2 = float(np.sum(ctx.download()))
    msg = (f"target {tgt}: W {st['stream_w']} tiles {st['stream_tiles']} | single traj {min(tr):.3f} ms "
           f"({nx*nx*500/min(tr)/1e6:.1f} Gcell/s) blocked {st['slow_diagonals']} checksum {c2:.17g}")
    if os.environ.get("AB_SWEEP", "1") == "1" and nx == 1024:
        try:
            ctx.sweep(mus, 500, keep_snaps=False)
            sw = []
            for _ in range(reps):
                s2 = ctx.sweep(mus, 500, keep_snaps=False)[1]
                sw.append(s2["loop_ms"])
            c1 = float(np.sum(ctx.download()))
            msg += (f" | sweep W {s2['stream_w']} {min(sw):.2f} ms ({nx*nx*4500/min(sw)/1e6:.1f} Gcell/s) "
                    f"checksum {c1:.17g}")
        except Exception as e:  # noqa: BLE001 -- report and go on
            msg += f" | sweep: {e}"
    print(msg, flush=True)
    ctx.close()
