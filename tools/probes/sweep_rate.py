"""Rate of the 1024^2 9-mu sweep (config2_1024's unit): python sweep_rate.py
[reps]; knobs (BURG_SWEEP_BATCH, BURG_PAIR) from the environment.  Checks
the last trajectory's final state against a second run with the knobs off
is left to the tests; this prints the launch times only."""
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
mus = get_snapshot_params()[:9]
ctx.sweep(mus, T, keep_snaps=False)
res = [ctx.sweep(mus, T, keep_snaps=False)[1] for _ in range(reps)]
sw = [r["loop_ms"] for r in res]
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("BURG_")},
                  "sweep9_ms": [round(x, 3) for x in sw],
                  "sweep9_gcell": round(9 * N * N * T / min(sw) / 1e6, 1),
                  "launches": res[-1].get("stream_launches"), "paired": res[-1].get("paired_launches"),
                  # compute-wave time spent waiting at block readiness (s_memtime:
                  # shader clock cycles, taken at the measured 2.176 GHz) over
                  # compute-wave time (one wave per tile)
                  "slow_blocks": res[-1].get("slow_diagonals"), "slow_ticks": res[-1].get("slow_ticks"),
                  "wait_frac": (round(res[-1]["slow_ticks"] / 2.176e9 / (sw[-1] * 1e-3 * res[-1]["stream_tiles"]), 4)
                                if res[-1].get("slow_ticks") else None)}),
      flush=True)
