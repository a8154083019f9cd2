"""A/B of library builds (BURG_LIB) at 1024^2 (BASELINE configs[1]): the 9-mu
sweep (one burg_sweep launch) and one 500-step trajectory (run_fom.main's
unit), best of `reps` launches by HIP events, with the final states'
checksums (a build must not change the bits)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.config import get_snapshot_params  # noqa: E402
from finitedifference_amd.solver import FOMContext  # noqa: E402

reps = int(os.environ.get("AB_REPS", "4"))
nx = 1024
ctx = FOMContext(nx, nx, engine="pipe")
g = np.linspace(0, 100, nx + 1)
ctx.set_problem(g, g, 0.05, (5.19, 0.026))
ctx.upload(np.ones(ctx.m))
mus = get_snapshot_params()[:9]
ctx.sweep(mus, 500, keep_snaps=False)
sws = [ctx.sweep(mus, 500, keep_snaps=False)[1] for _ in range(reps)]
sw = [x["loop_ms"] for x in sws]
c1 = float(np.sum(ctx.download()))
ctx.trajectory(500)
trs = [ctx.trajectory(500) for _ in range(reps)]
tr = [x["loop_ms"] for x in trs]
c2 = float(np.sum(ctx.download()))
tag = os.environ.get("BURG_LIB", "default").split("/")[-1]
print(f"{tag}: 1024^2 sweep {min(sw):.2f} ms ({nx*nx*4500/min(sw)/1e6:.1f} Gcell/s) | single traj "
      f"{min(tr):.3f} ms ({nx*nx*500/min(tr)/1e6:.1f} Gcell/s) | checksums {c1:.17g} {c2:.17g} | ieee "
      f"{sws[-1]['ieee_diagonals']} {trs[-1]['ieee_diagonals']} blocked {sws[-1]['slow_diagonals']} "
      f"{trs[-1]['slow_diagonals']}",
      flush=True)
