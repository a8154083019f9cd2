"""Retained-window trajectories (snap_every=10) at 16384 x 2048 on a ring
first allocated for the capped plain trajectory (240 GB) vs a fresh ring:
one JSON line with both rates (the chk1 test measured 150 vs 176)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.solver import FOMContext  # noqa: E402

nx, ny, T = 16384, 2048, 500
out = {}
for order in ("plain_first", "fresh"):
    ctx = FOMContext(nx, ny)
    ctx.set_problem(np.linspace(0, 100, nx + 1), np.linspace(0, 100.0 * ny / nx, ny + 1),
                    0.05 * 1024 / nx, (5.19, 0.026), allow_nonsquare=True)
    ctx.upload(np.ones(ctx.m))
    if order == "plain_first":
        ctx.trajectory(T)
        pl = ctx.trajectory(T)["loop_ms"]
        out["plain_ms"] = round(pl, 3)
    ms = [ctx.trajectory(T, snap_every=10)["loop_ms"] for _ in range(3)]
    out[order] = [round(x, 3) for x in ms]
    ctx.close()
print(json.dumps(out), flush=True)
