"""1024^2 9-mu sweep (BASELINE configs[1]) at narrow tile widths 8 and 16:
W = 8 puts two compute waves on each SIMD (2048 tiles, two workgroups per
CU), W = 16 one.  Prints ms per sweep launch and Gcell-updates/s."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from finitedifference_amd.config import get_snapshot_params
    from finitedifference_amd.solver import FOMContext
    nx, T = 1024, 500
    mus = get_snapshot_params()[:9]
    g = np.linspace(0, 100, nx + 1)
    for W in (16, 8, 16, 8):
        ctx = FOMContext(nx, nx, engine="pipe", stream_w=W)
        ctx.set_problem(g, g, 0.05, mus[0])
        ctx.upload(np.ones(ctx.m))
        st = ctx.sweep(mus, T, keep_snaps=False)[1]
        t0 = time.perf_counter()
        ms = 0.0
        for _ in range(3):
            st = ctx.sweep(mus, T, keep_snaps=False)[1]
            ms += st["loop_ms"]
        el = time.perf_counter() - t0
        ctx.close()
        print(f"W={st['stream_w']} tiles={st['stream_tiles']} launch_ms={ms / 3:.2f} "
              f"Gcell/s={nx * nx * T * 9 * 3 / el / 1e9:.1f} launches={st['stream_launches']}", flush=True)


if __name__ == "__main__":
    main()
