"""Wall clock of burg_run_npy (run_fom.main's timed region: march + D2H +
.npy file) at 1024^2 x 500: python npy_rate.py [reps]; the writer-pool knobs
(BURG_NPY_WRITERS, BURG_NPY_FSYNC) are environment variables.  Checks the
file's last column against the context's final state."""
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.solver import FOMContext  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
nx, T = 1024, 500
ctx = FOMContext(nx, nx, engine="pipe")
g = np.linspace(0, 100, nx + 1)
ctx.set_problem(g, g, 0.05, (5.19, 0.026))
d = tempfile.mkdtemp(prefix="burg_npy_")
path = os.path.join(d, "snaps.npy")
walls = []
for r in range(reps):
    t0 = time.perf_counter()
    st = ctx.run_to_npy(np.ones(ctx.m), T, path)
    walls.append(time.perf_counter() - t0)
    a = np.load(path, mmap_mode="r")
    ok = bool(np.array_equal(np.asarray(a[:, -1]), ctx.download()))
    del a
    os.remove(path)
    if not ok:
        print(json.dumps({"error": "last column != final state", "rep": r}), flush=True)
        sys.exit(1)
os.rmdir(d)
ctx.close()
print(json.dumps({"wall_s": [round(w, 3) for w in walls], "best_mcell_per_s": round(nx * nx * T / min(walls) / 1e6, 1),
                  "flush_ms": round(st["flush_ms"], 1), "loop_ms": round(st["loop_ms"], 3),
                  "tmpdir": tempfile.gettempdir(),
                  "env": {k: v for k, v in os.environ.items() if k.startswith("BURG_NPY")}}), flush=True)
