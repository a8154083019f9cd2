"""A/B timing of library builds (BURG_LIB=...): the 1024^2 9-mu sweep and a
4096^2 trajectory, device time per launch (HIP events)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.config import get_snapshot_params  # noqa: E402
from finitedifference_amd.solver import FOMContext  # noqa: E402


def run(nx, dt, mus, T, reps):
    ctx = FOMContext(nx, nx, engine="pipe",
                     tiles_target=int(os.environ.get("AB_TILES", "0")) if nx > 1024 else 0)
    g = np.linspace(0, 100, nx + 1)
    ctx.set_problem(g, g, dt, (5.19, 0.026))
    ctx.upload(np.ones(ctx.m))
    f = (lambda: ctx.sweep(mus, T, keep_snaps=False)[1]) if len(mus) > 1 else (lambda: ctx.trajectory(T))
    f()
    ms = []
    for _ in range(reps):
        st = f()
        ms.append(st["loop_ms"])
    ctx.close()
    return min(ms), st


tag = os.environ.get("BURG_LIB", "default").split("/")[-1]
a, st = run(1024, 0.05, get_snapshot_params()[:9], 500, 3)
b, st2 = run(4096, 0.0125, [(5.19, 0.026)], 500, 2)
print(f"{tag}: 1024^2 sweep {a:.2f} ms ({1024*1024*4500/a/1e6:.0f} Gcell/s)  blocked {st['slow_diagonals']} "
      f"polls {st['comm_polls']} | 4096^2 traj {b:.2f} ms ({4096*4096*500/b/1e6:.0f} Gcell/s) "
      f"blocked {st2['slow_diagonals']} wait {st2['slow_ticks']/max(1,st2['slow_diagonals']):.0f}clk polls {st2['comm_polls']} W {st2['stream_w']} tiles {st2['stream_tiles']}", flush=True)
