"""A/B of the paired-halves W = 16 kernel (BURG_PAIR, pipe.hip PAIR): the
1024^2 x 500 trajectory and the 1024^2 9-mu sweep (config2_1024's unit), one
warm-up, then reps timed launches each; one JSON line.

    python tools/probes/pair_ab.py [reps]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.config import get_snapshot_params  # noqa: E402
from finitedifference_amd.solver import FOMContext  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
N, T = 1024, 500
ctx = FOMContext(N, N)
g = np.linspace(0, 100, N + 1)
ctx.set_problem(g, g, 0.05, (5.19, 0.026))
ctx.upload(np.ones(ctx.m))
ctx.trajectory(T)
traj = [ctx.trajectory(T)["loop_ms"] for _ in range(reps)]
mus = get_snapshot_params()[:9]
ctx.sweep(mus, T, keep_snaps=False)
sw = [ctx.sweep(mus, T, keep_snaps=False)[1]["loop_ms"] for _ in range(reps)]
print(json.dumps({"BURG_PAIR": os.environ.get("BURG_PAIR", "default(1)"),
                  "trajectory_ms": [round(x, 3) for x in traj],
                  "trajectory_gcell": round(N * N * T / min(traj) / 1e6, 1),
                  "sweep9_ms": [round(x, 3) for x in sw],
                  "sweep9_gcell": round(9 * N * N * T / min(sw) / 1e6, 1)}), flush=True)
