"""Pipe-engine timing sweep (diagnostics): device time of one trajectory
launch for several lengths T and tile widths W; the slope over T is the
per-step (W diagonals) cost, the intercept the pipeline ramp."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from finitedifference_amd.solver import FOMContext  # noqa: E402

nx = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
engine = os.environ.get("ENGINE", "pipe")
for W in (16, 8):
    c = FOMContext(nx, nx, engine=engine, stream_w=W)
    g = np.linspace(0, 100, nx + 1)
    c.set_problem(g, g, 0.05, (5.19, 0.026))
    c.upload(np.ones(2 * nx * nx))
    c.trajectory(50)
    res = []
    for T in (100, 250, 500, 1000):
        ts = []
        for _ in range(3):
            st = c.trajectory(T)
            ts.append(st["loop_ms"])
        t = float(np.median(ts))
        res.append((T, t))
        print(f"{engine} nx={nx} W={W} tiles={st['stream_tiles']} T={T}: {t:.3f} ms "
              f"{nx * nx * T / t / 1e6:.1f} Gcell/s blocked={st['slow_diagonals']} "
              f"spins={st['stall_spins']} ieee={st['ieee_diagonals']} polls={st['comm_polls']}",
              flush=True)
    T = np.array([r[0] for r in res], float)
    t = np.array([r[1] for r in res])
    b, a = np.polyfit(T, t, 1)
    print(f"  fit: {a:.3f} ms + {b * 1e3:.3f} us/step -> {b * 1e3 / W * 1e3:.0f} ns/diagonal, "
          f"ramp {a / (b / W):.0f} diagonals", flush=True)
    c.close()
