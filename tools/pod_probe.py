"""POD timing probe (burg_pod): POD of the 250^2 training
snapshot set -- the 9 get_snapshot_params trajectories of 500 steps
(C/run_prom.py:58-86), computed on the GPU by one sweep -- 125000 x 4509.

    python tools/pod_probe.py [N] [T] [nmu]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MUS = [(4.25, 0.015), (4.25, 0.0225), (4.25, 0.03), (4.875, 0.015), (4.875, 0.0225),
       (4.875, 0.03), (5.5, 0.015), (5.5, 0.0225), (5.5, 0.03)]


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 250
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    nmu = int(sys.argv[3]) if len(sys.argv) > 3 else 9
    from finitedifference_amd import hypernet2D as H
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    t = time.time()
    sn = H.inviscid_burgers_implicit2D_sweep(gx, gy, np.ones(2 * N * N), 0.05, T, MUS[:nmu],
                                             verbose=0)
    S = np.hstack(sn)
    del sn
    t_fom = time.time() - t
    H.POD(S[:, :64], method="svd")  # warm-up (rocBLAS/rocSOLVER init)
    t = time.time()
    u, s, ms = H.POD(S, num_modes=95, method="rsvd", return_ms=True)
    t_pod = time.time() - t
    m, ns = S.shape
    print(json.dumps({"N": N, "T": T, "nmu": nmu, "shape": [m, ns], "fom_sweep_s": t_fom,
                      "pod_wall_s": t_pod, "pod_device_ms": ms,
                      "qr_tflops_equiv": 2.0 * m * ns * ns / (ms / 1e3) / 1e12,
                      "s0": float(s[0]), "s94_rel": float(s[94] / s[0])}))


if __name__ == "__main__":
    main()
