"""Where does the wide-tile pipe engine differ from the oracle? (debug aid)
    BURG_ALLOW_NONFINITE=1 python tools/probes/wide_diff.py NX NY W T"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.solver import FOMContext  # noqa: E402
from oracle import oracle  # noqa: E402

nx, ny, W, T = (int(x) for x in sys.argv[1:5])
P = oracle.Problem(nx, ny, Ly=100.0 * ny / nx, allow_nonsquare=(nx != ny))
w0 = np.ones(P.m)
ctx = FOMContext(nx, ny, engine="pipe", stream_w=W)
ctx.set_problem(P.grid_x, P.grid_y, P.dt, P.mu, allow_nonsquare=(nx != ny))
snaps, st, _, _ = ctx.run(w0, T)
ref, _, _ = P.fom(w0, T)
print(f"{nx}x{ny} W={st['stream_w']} tiles={st['stream_tiles']} nonfinite={st['nonfinite_diagonals']}")
for j in range(1, T + 1):
    u = (snaps[:, j] != ref[j])[:nx * ny].reshape(ny, nx)
    bad_tiles = sorted({(r // 64, c // W) for r, c in zip(*np.nonzero(u))})
    print(f"  step {j}: {int(u.sum())} u cells differ, tiles (ti, tj) {bad_tiles[:12]}")
    if u.sum():
        r, c = [int(x[0]) for x in np.nonzero(u)]
        print(f"    first ({r},{c}) gpu {snaps[r * nx + c, j]!r} ref {ref[j][r * nx + c]!r}")
