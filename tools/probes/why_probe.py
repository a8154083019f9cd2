"""Wait reasons of the pipe kernel on one shape (BURG_STREAM_DEBUG=8 prints
them, and with the BURG_PIPE_PROF library the compute waves' readiness-wait
share): python tools/probes/why_probe.py NX ROWS"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.solver import FOMContext  # noqa: E402

nx, rows = int(sys.argv[1]), int(sys.argv[2])
ctx = FOMContext(nx, rows, engine="pipe")
g = np.linspace(0, 100, nx + 1)
gy = np.linspace(0, 100.0 * rows / nx, rows + 1)
ctx.set_problem(g, gy, 0.05 * 1024 / nx, (5.19, 0.026), allow_nonsquare=(nx != rows))
ctx.upload(np.ones(ctx.m))
ctx.trajectory(500)
st = ctx.trajectory(500)
print(f"{nx}x{rows}: {st['loop_ms']:.2f} ms W {st['stream_w']} blocked {st['slow_diagonals']} "
      f"spins {st['stall_spins']} wait ticks {st['slow_ticks']}", flush=True)
