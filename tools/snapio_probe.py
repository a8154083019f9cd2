"""Snapshot I/O probe: end-to-end time of computing a
trajectory AND caching it as the reference's .npy file, two ways --
  reference flow: snapshot matrix in host memory, then np.save
                  (C/hypernet2D.py:3141-3143, C/run_fom.py:41-43)
  streamed:       load_or_compute_snaps(stream=True): the library writes the
                  snapshots into a memory map of the cache file
(both without fsync, as np.save; the fsync'd times are reported too).

    python tools/snapio_probe.py [N] [T] [dir]
"""
import json
import os
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    d = sys.argv[3] if len(sys.argv) > 3 else "/tmp/snapio"
    from finitedifference_amd import hypernet2D as H
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    w0 = np.ones(2 * N * N)
    mu = (5.19, 0.026)
    H.inviscid_burgers_implicit2D(gx, gy, w0, 0.05, 2, mu, verbose=0)  # warm-up
    out = {"N": N, "T": T, "file_bytes": 2 * N * N * (T + 1) * 8}
    for mode in ("reference", "streamed"):
        shutil.rmtree(d, ignore_errors=True)
        os.makedirs(d)
        t0 = time.time()
        if mode == "reference":
            s = H.inviscid_burgers_implicit2D(gx, gy, w0, 0.05, T, mu, verbose=0)
            t1 = time.time()
            np.save(H.param_to_snap_fn(mu, d), s)
        else:
            s = H.load_or_compute_snaps(mu, gx, gy, w0, 0.05, T, snap_folder=d, stream=True,
                                        mmap=True)
            t1 = time.time()
        t2 = time.time()
        os.sync()
        t3 = time.time()
        out[mode] = {"compute_s": t1 - t0, "total_s": t2 - t0, "total_fsync_s": t3 - t0,
                     "GBps_to_file": out["file_bytes"] / (t2 - t0) / 1e9}
        del s
    shutil.rmtree(d, ignore_errors=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
