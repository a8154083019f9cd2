"""Rate of burg_trajectory_ex on one GPU: python traj_rate.py NX NY [snap_every] [reps]
(dt = 0.05 * 1024 / NX as the bench; one warm-up, then reps timed launches;
prints one JSON line; the A/B knobs are environment variables; TRAJ_W forces
the tile width)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.solver import FOMContext  # noqa: E402

nx, ny = int(sys.argv[1]), int(sys.argv[2])
k = int(sys.argv[3]) if len(sys.argv) > 3 else 1
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
T = 500
ctx = FOMContext(nx, ny, stream_w=int(os.environ.get("TRAJ_W", "0")))
ctx.set_problem(np.linspace(0, 100, nx + 1), np.linspace(0, 100.0 * ny / nx, ny + 1),
                0.05 * 1024 / nx, (5.19, 0.026), allow_nonsquare=nx != ny)
ctx.upload(np.ones(ctx.m))
ctx.reserve(T, snap_every=k)
ctx.trajectory(T, snap_every=k)
ms = []
t0 = time.perf_counter()
for _ in range(reps):
    ms.append(ctx.trajectory(T, snap_every=k)["loop_ms"])
el = time.perf_counter() - t0
st = ctx.trajectory(T, snap_every=k)
print(json.dumps({"grid": f"{nx}x{ny}", "snap_every": k, "retained": list(ctx.retained()),
                  "W": st["stream_w"], "kernel_ms": [round(x, 3) for x in ms],
                  "gcell_per_s_best": round(nx * ny * T / min(ms) / 1e6, 1),
                  "gcell_per_s_wall": round(nx * ny * T * reps / el / 1e9, 1),
                  "env": {k2: v for k2, v in os.environ.items() if k2.startswith("BURG_")}}),
      flush=True)
