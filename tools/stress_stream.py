"""Stress driver for the streaming engine's edge protocol (diagnostics only)."""
import sys, os, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from finitedifference_amd.solver import FOMContext
from finitedifference_amd._lib import BurgersError
from oracle import oracle

def ctx_for(N, **kw):
    c = FOMContext(N, N, **kw)
    c.set_problem(np.linspace(0, 100, N + 1), np.linspace(0, 100, N + 1), 0.05, (5.19, 0.026))
    return c

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
fails = 0
t0 = time.time()
for N, W in [(200, 8), (200, 16), (333, 32), (1024, 16)]:
    P = oracle.Problem(N)
    ref, _, _ = P.fom(np.ones(P.m), 9)
    c = ctx_for(N, stream_w=W)
    nf = nm = 0
    spins = []
    for it in range(iters):
        try:
            c.upload(np.ones(P.m))
            for k in (2, 3, 4):
                st = c.advance(k)
                spins.append(st["stall_spins"])
            if not np.array_equal(c.download(), ref[9]):
                nm += 1
        except BurgersError as e:
            nf += 1
            if nf <= 3:
                print("  ", N, W, it, e, flush=True)
    print(N, W, "iters", iters, "timeouts", nf, "mismatches", nm, "spins med/max",
          int(np.median(spins)), max(spins), f"{time.time()-t0:.1f}s", flush=True)
