"""Per-diagonal time of the pipe kernel in small grids (diagnostics): one
strip of 64 rows with 1..4 tiles of width W (one workgroup, no cross-CU
traffic) against the full grid, to separate the compute waves' own
instruction stream from contention.

    python tools/probes/iso_bench.py [W] [T] [NXxNY,...]

Per diagonal = loop time / (T W + nx + ny): the wavefront's own length plus
its fill (the last tile starts nx + ny diagonals after the first).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.solver import FOMContext  # noqa: E402


def run(nx, ny, W, T, dt):
    ctx = FOMContext(nx, ny, engine="pipe", stream_w=W)
    gx = np.linspace(0, 100, nx + 1)
    gy = np.linspace(0, 100.0 * ny / nx, ny + 1)
    ctx.set_problem(gx, gy, dt, (5.19, 0.026), allow_nonsquare=nx != ny)
    ctx.upload(np.ones(ctx.m))
    ctx.trajectory(T)
    best = min(ctx.trajectory(T)["loop_ms"] for _ in range(3))
    ctx.close()
    diag = T * W + nx + ny
    return best, best * 1e6 / diag


W = int(sys.argv[1]) if len(sys.argv) > 1 else 256
T = int(sys.argv[2]) if len(sys.argv) > 2 else 200
shapes = ([tuple(int(v) for v in x.split("x")) for x in sys.argv[3].split(",")]
          if len(sys.argv) > 3 else [(W, 64), (4 * W, 64), (4 * W, 256), (4096, 4096)])
for nx, ny in shapes:
    ms, ns = run(nx, ny, W, T, 0.05 * 1024 / max(nx, ny))
    print(f"{nx}x{ny} W={W}: {ms:.2f} ms, {ns:.1f} ns per diagonal ({ns * 2.4:.0f} cycles at 2.4 GHz)",
          flush=True)
