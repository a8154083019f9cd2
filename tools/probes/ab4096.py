"""A/B of library builds (BURG_LIB) on the bench's 4096^2 x 500 trajectory:
best of `reps` launches (HIP events), plus its final state's checksum (a
build must not change the bits)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.solver import FOMContext  # noqa: E402

nx = int(os.environ.get("AB_NX", "4096"))
reps = int(os.environ.get("AB_REPS", "5"))
ctx = FOMContext(nx, nx, engine="pipe")
g = np.linspace(0, 100, nx + 1)
ctx.set_problem(g, g, 0.05 * 1024 / nx, (5.19, 0.026))
ctx.upload(np.ones(ctx.m))
ctx.trajectory(500)
ms = [ctx.trajectory(500)["loop_ms"] for _ in range(reps)]
w = ctx.download()
tag = os.environ.get("BURG_LIB", "default").split("/")[-1]
print(f"{tag}: {nx}^2 traj best {min(ms):.2f} ms median {sorted(ms)[len(ms)//2]:.2f} "
      f"({nx*nx*500/min(ms)/1e6:.0f} Gcell/s) checksum {float(np.sum(w)):.17g}", flush=True)
