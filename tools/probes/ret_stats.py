"""Distribution of the retained-window trajectory's launch time at 16384 x
2048 x 500 (snap_every=10) over NREP launches in one context, with each
launch's wait statistics; the plain capped ring alternately for reference."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.solver import FOMContext  # noqa: E402

nx, ny, T = 16384, 2048, 500
ks = [int(x) for x in os.environ.get("KS", "10 1").split()]
ctx = FOMContext(nx, ny)
ctx.set_problem(np.linspace(0, 100, nx + 1), np.linspace(0, 100.0 * ny / nx, ny + 1),
                0.05 * 1024 / nx, (5.19, 0.026), allow_nonsquare=True)
ctx.upload(np.ones(ctx.m))
for k in ks:
    ctx.reserve(T, snap_every=k)
    ctx.trajectory(T, snap_every=k)
    for i in range(int(os.environ.get("NREP", "6"))):
        st = ctx.trajectory(T, snap_every=k)
        print(json.dumps({"k": k, "ms": round(st["loop_ms"], 3), "blocked": st["slow_diagonals"],
                          "spins": st["stall_spins"], "slow_ticks": st["slow_ticks"],
                          "polls": st["comm_polls"]}), flush=True)
