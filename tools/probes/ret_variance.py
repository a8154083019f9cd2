"""Variance of the retained-window trajectory rate across fresh contexts
(each one allocates its own ring): 16384 x 2048 x 500, snap_every=10, and
the plain capped ring for reference; one JSON line per context."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.solver import FOMContext  # noqa: E402

nx, ny, T = 16384, 2048, 500
for i in range(int(os.environ.get("NCTX", "4"))):
    for k in (10, 1):
        ctx = FOMContext(nx, ny)
        ctx.set_problem(np.linspace(0, 100, nx + 1), np.linspace(0, 100.0 * ny / nx, ny + 1),
                        0.05 * 1024 / nx, (5.19, 0.026), allow_nonsquare=True)
        ctx.upload(np.ones(ctx.m))
        ctx.reserve(T, snap_every=k)
        ctx.trajectory(T, snap_every=k)
        ms = [ctx.trajectory(T, snap_every=k)["loop_ms"] for _ in range(3)]
        ctx.close()
        print(json.dumps({"ctx": i, "snap_every": k, "kernel_ms": [round(x, 3) for x in ms],
                          "lw": os.environ.get("BURG_RET_LW", "2")}), flush=True)
