"""One rank of the multi-GPU drop-in tests in tests/test_gpu_job.py (not a
test module): the REFERENCE API under a multi-process job, every rank on the
box's one GPU -- run_fom.main (or load_or_compute_snaps on a non-square
grid), exactly as a user's script would call it under torchrun.

    job_worker.py OUTDIR fine750|slab16384 ...
    env: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT (as torchrun sets them)
Writes OUTDIR/rank{r}.json: shape, a digest of the returned matrix, the
elapsed time, whether it is a copy-on-write map.
"""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def digest(a):
    h = hashlib.sha256()
    for j in range(0, a.shape[0], 1 << 16):
        h.update(np.ascontiguousarray(a[j:j + (1 << 16)]).tobytes())
    return h.hexdigest()[:16]


def main():
    out, case = sys.argv[1], sys.argv[2]
    rank = int(os.environ["RANK"])
    os.chdir(out)  # run_fom.main saves hdm_snaps_*.npy into the working directory
    if case == "fine750":
        # BurgersFD_CleanFine/run_fom.py:28 -- 750^2, 500 steps, every state
        from finitedifference_amd import run_fom
        el, snaps = run_fom.main(5.19, 0.026, save_snaps=False, num_cells=750,
                                 snap_folder=os.path.join(out, "param_snaps"), device=0)
    else:
        # 16384 x 2048 (configs[4]'s per-GPU row length), T steps, every 10th state
        from finitedifference_amd import hypernet2D as H
        import time
        T = int(sys.argv[3])
        nx, ny = 16384, 2048
        gx = np.linspace(0, 100, nx + 1)
        gy = np.linspace(0, 100.0 * ny / nx, ny + 1)
        t0 = time.time()
        snaps = H.load_or_compute_snaps((5.19, 0.026), gx, gy, np.ones(2 * nx * ny), 0.05 * 1024 / nx,
                                        T, snap_folder=os.path.join(out, "param_snaps"),
                                        snap_every=10, allow_nonsquare=True, device=0,
                                        stream_w=1024)
        el = time.time() - t0
    info = {"rank": rank, "shape": list(snaps.shape), "digest": digest(snaps), "elapsed": el,
            "memmap": isinstance(snaps, np.memmap), "writeable": bool(snaps.flags.writeable)}
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump(info, f)


if __name__ == "__main__":
    main()
