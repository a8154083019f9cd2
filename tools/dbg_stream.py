"""Debug driver for the streaming engine (not part of the product or tests)."""
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

for N, W in [(200, 8), (200, 16), (130, 8), (64, 8)]:
    P = oracle.Problem(N)
    ref, _, _ = P.fom(np.ones(P.m), 6)
    for mode in ("run", "adv"):
        c = ctx_for(N, stream_w=W)
        try:
            t0 = time.time()
            if mode == "run":
                s, st, _, _ = c.run(np.ones(P.m), 3)
                ok = np.array_equal(s[:, 3], ref[3])
            else:
                c.upload(np.ones(P.m))
                st = c.advance(2)
                ok2 = np.array_equal(c.download(), ref[2])
                st = c.advance(1)
                ok = ok2 and np.array_equal(c.download(), ref[3])
            print(N, W, mode, "ok" if ok else "MISMATCH", "spins", st["stall_spins"], "slow", st["slow_diagonals"], "tiles", st["stream_tiles"], f"{time.time()-t0:.2f}s", flush=True)
        except BurgersError as e:
            print(N, W, mode, "ERROR", e, f"{time.time()-t0:.2f}s", flush=True)
