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
    H.POD(S[:, :64], num_modes=8, method="rsvd", random_state=0)
    m, ns = S.shape
    out = {"N": N, "T": T, "nmu": nmu, "shape": [m, ns], "fom_sweep_s": t_fom}
    t = time.time()
    u, s, ms_first = H.POD(S, num_modes=95, method="rsvd", random_state=0, return_ms=True)
    wall_first = time.time() - t
    t = time.time()  # again: the first call also pays the libraries' lazy code loading
    u, s, ms = H.POD(S, num_modes=95, method="rsvd", random_state=0, return_ms=True)
    r = 105
    flops = 2.0 * m * ns * r * (2 + 2 * 7) + 2.0 * m * ns * r  # S.Omega, 7 x (S^T.Q, S.Z), Q^T.S
    out["rsvd"] = {"wall_s": time.time() - t, "device_ms": ms, "wall_s_first": wall_first,
                   "device_ms_first": ms_first, "gemm_flops": flops,
                   "gemm_TFLOPs_equiv": flops / (ms / 1e3) / 1e12,
                   "s0": float(s[0]), "s94_rel": float(s[94] / s[0])}
    if os.environ.get("POD_PROBE_RSVD_ONLY"):
        print(json.dumps(out))
        return
    t = time.time()
    ue, se, mse = H.POD(S, method="svd", return_ms=True)
    out["svd"] = {"wall_s": time.time() - t, "device_ms": mse,
                  "rsvd_vs_exact_s_maxrel": float(np.max(np.abs(s / se[:95] - 1))),
                  "rsvd_vs_exact_min_abs_cos_top50": float(np.min(np.abs(np.sum(u[:, :50] * ue[:, :50], axis=0))))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
