"""Debug aid: window-vs-ring check of the wide pipe engine (BURG_PIPE_DEBUG=1)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finitedifference_amd.solver import FOMContext  # noqa: E402

N, W = int(sys.argv[1]), int(sys.argv[2])
ctx = FOMContext(N, 64, engine="pipe", stream_w=W)
g = np.linspace(0, 100, N + 1)
ctx.set_problem(g, np.linspace(0, 100 * 64 / N, 65), 0.05, (5.19, 0.026), allow_nonsquare=True)
ctx.upload(np.ones(2 * 64 * N))
try:
    st = ctx.advance(2)
    print({k: st[k] for k in ("stall_spins", "slow_diagonals", "ieee_diagonals", "nonfinite_diagonals")})
except Exception as ex:
    print("failed:", ex)
