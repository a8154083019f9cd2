"""Per-diagonal cost at 1024^2 under diagnostic variants (BURG_STREAM_DEBUG bits:
1 = tiles ignore their neighbours, 2 = deeper prefetch)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from finitedifference_amd.solver import FOMContext
nx = ny = 1024
for flags in ("8",):
  for R in ("8", "32", "128"):
    os.environ["BURG_STREAM_R"] = R
    os.environ["BURG_STREAM_DEBUG"] = flags
    for W in (16, 32):
        c = FOMContext(nx, ny, stream_w=W)
        c.set_problem(np.linspace(0, 100, nx + 1), np.linspace(0, 100, ny + 1), 0.05, (5.19, 0.026))
        c.upload(np.ones(2 * nx * ny))
        c.advance(2)
        t1 = c.advance(50)["loop_ms"]
        st = c.advance(550)
        t2 = st["loop_ms"]
        print(f"R={R} flags={flags} W={W} per-diag {(t2-t1)*1e6/(500*W):.0f} ns  t550 {t2:.3f} ms  "
              f"spins {st['stall_spins']} slow {st['slow_diagonals']} slow_ms/wave {st['slow_ticks']/max(1,st['stream_tiles'])/2.1e6:.3f}", flush=True)
