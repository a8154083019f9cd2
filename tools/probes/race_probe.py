"""Find where a wide-tile march first departs from the CPU oracle (race
hunting): python race_probe.py NX NY W T -> the first mismatching (step,
row, column, component), GPU and oracle values, and the count per step.
The library comes from BURG_LIB (e.g. a priority-changed A/B build)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle as orc  # noqa: E402  (test infrastructure: the checker)
from test_gpu_regime import _ctx, _problem  # noqa: E402

nx, ny, W, T = (int(x) for x in sys.argv[1:5])
dt = 0.05 * 1024 / nx
P = _problem(orc, nx, ny, dt=dt)
ref, _, _ = P.fom(np.ones(P.m), T)
ctx = _ctx(nx, ny, dt=dt, engine="pipe", stream_w=W)
out = {"grid": f"{nx}x{ny}", "W": W, "T": T}
try:
    snaps, st, _, _ = ctx.run(np.ones(P.m), T)
    out["stream_w"] = st["stream_w"]
except Exception as e:  # noqa: BLE001
    out["error"] = str(e)[:300]
    print(json.dumps(out), flush=True)
    sys.exit(0)
n = nx * ny
per = []
first = None
for j in range(1, T + 1):
    g, r = snaps[:, j], ref[j]
    bad = np.flatnonzero(~((g == r) | (np.isnan(g) & np.isnan(r))))
    per.append(int(bad.size))
    if bad.size and first is None:
        i = int(bad[0])
        comp, cell = divmod(i, n)
        row, col = divmod(cell, nx)
        rows = sorted(set((int(b) % n) // nx for b in bad[:2000]))
        cols = sorted(set((int(b) % n) % nx for b in bad[:2000]))
        first = {"step": j, "row": row, "col": col, "comp": "uv"[comp], "gpu": float(g[i]), "ref": float(r[i]),
                 "rows_sample": rows[:20], "cols_sample": cols[:20], "tile_col": col // W, "tile_row": row // 64}
out["mismatches_per_step"] = per
out["first"] = first
if first is not None and os.environ.get("RACE_SAVE"):
    j = first["step"]
    np.savez_compressed(os.environ["RACE_SAVE"], gpu=snaps[:, j], ref_prev=ref[j - 1], ref=ref[j],
                        gpu_prev=snaps[:, j - 1])
print(json.dumps(out), flush=True)
