"""The reference's own snapshot sweep (C/run_prom.py:59-71: 250^2, 9 training
mu, 500 steps, dt = 0.05) as one burg_sweep call, states left in HBM: best of
`reps` by HIP events; the A/B knobs (BURG_SWEEP_BATCH, BURG_SWEEP_BATCH_TILES)
come from the environment."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.config import get_snapshot_params  # noqa: E402
from finitedifference_amd.solver import FOMContext  # noqa: E402

N, T, reps = 250, 500, int(os.environ.get("AB_REPS", "4"))
ctx = FOMContext(N, N)
g = np.linspace(0, 100, N + 1)
ctx.set_problem(g, g, 0.05, (5.19, 0.026))
ctx.upload(np.ones(ctx.m))
mus = get_snapshot_params()[:9]
ctx.sweep(mus, T, keep_snaps=False)
sts = [ctx.sweep(mus, T, keep_snaps=False)[1] for _ in range(reps)]
ms = [s["loop_ms"] for s in sts]
print(json.dumps({"grid": "250x250", "mu": 9, "steps": T, "kernel_ms": [round(x, 3) for x in ms],
                  "best_ms": round(min(ms), 3), "W": sts[-1]["stream_w"],
                  "tiles": sts[-1]["stream_tiles"], "launches": sts[-1]["stream_launches"],
                  "gcell_per_s": round(N * N * T * 9 / min(ms) / 1e6, 2),
                  "checksum": float(np.sum(ctx.download())),
                  "env": {k: v for k, v in os.environ.items() if k.startswith("BURG_SWEEP")}}),
      flush=True)
