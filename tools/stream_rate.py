"""Per-diagonal cost of the streaming engine for a few tilings (diagnostics):
time advance(K) for two K and report the incremental time per diagonal."""
import sys, os, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from finitedifference_amd.solver import FOMContext

def ctx_for(nx, ny, **kw):
    c = FOMContext(nx, ny, **kw)
    c.set_problem(np.linspace(0, 100, nx + 1), np.linspace(0, 100.0 * ny / nx, ny + 1), 0.05,
                  (5.19, 0.026), allow_nonsquare=(nx != ny))
    return c

cases = [(16, 64, 16), (32, 64, 16), (16, 128, 16), (256, 64, 16), (1024, 1024, 16),
         (1024, 1024, 8), (1024, 1024, 32), (64, 64, 64), (2048, 2048, 32)]
for nx, ny, W in cases:
    c = ctx_for(nx, ny, stream_w=W)
    c.upload(np.ones(2 * nx * ny))
    c.advance(2)
    K1, K2 = 50, 550
    t1 = c.advance(K1)["loop_ms"]
    st = c.advance(K2)
    t2 = st["loop_ms"]
    per_diag_us = (t2 - t1) * 1e3 / ((K2 - K1) * W)
    cells = nx * ny
    print(f"{nx}x{ny} W={W} tiles={st['stream_tiles']} t({K1})={t1:.3f}ms t({K2})={t2:.3f}ms "
          f"per-diag {per_diag_us*1e3:.0f} ns  steady {cells/((t2-t1)*1e-3/(K2-K1))/1e9:.1f} Gcell/s "
          f"spins {st['stall_spins']}", flush=True)
