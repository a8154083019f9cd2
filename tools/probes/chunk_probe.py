"""Which snapshot columns of a chunked burg_run differ from the oracle, and
where (first differing cell).  python tools/probes/chunk_probe.py nx ny W T chunk every [traj_first]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    nx, ny, W, T, chunk, every = (int(x) for x in sys.argv[1:7])
    traj_first = len(sys.argv) > 7 and sys.argv[7] == "1"
    if chunk > 0:
        os.environ["BURG_STREAM_CHUNK"] = str(chunk)
    from oracle import oracle
    from finitedifference_amd.solver import FOMContext
    dt = 0.05 * 1024 / max(nx, 1024)
    P = oracle.Problem(nx, ny, dt=dt, Ly=100.0 * ny / nx, allow_nonsquare=nx != ny)
    ref = P.march_traj(np.ones(P.m), T, every)
    ctx = FOMContext(nx, ny, engine="pipe", stream_w=W)
    ctx.set_problem(P.grid_x, P.grid_y, dt, P.mu, allow_nonsquare=nx != ny)
    if traj_first:
        ctx.upload(np.ones(P.m))
        ctx.trajectory(T)
    snaps, st, _, _ = ctx.run(np.ones(P.m), T, snap_every=every)
    print(f"{nx}x{ny} W={st['stream_w']} T={T} chunk={chunk} every={every} traj_first={traj_first} "
          f"launches={st['stream_launches']}")
    n = nx * ny
    for j in range(T // every + 1):
        d = np.nonzero(snaps[:, j] != ref[j])[0]
        if d.size:
            e = d[0]
            pl, cell = divmod(e, n)
            r, c = divmod(cell, nx)
            print(f"  col {j} (step {j * every}): {d.size} cells differ; first plane {pl} row {r} "
                  f"col {c} tile ({r // 64},{c // W}) lane {r % 64} cl {c % W}: "
                  f"{snaps[e, j]!r} vs {ref[j][e]!r}")
    print("done")


if __name__ == "__main__":
    main()
