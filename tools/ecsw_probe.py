"""ECSW training-matrix assembly (compute_ECSW_training_matrix_2D,
C/hypernet2D.py:2719-2740) on the GPU at the reference driver's size:
250^2, n_pod = 95 (C/run_HPROM_ecsw_joshua_.py:33), one mu block of 50
snapshots (snaps[:, 3:500:10], :81-84).  Prints one JSON line: kernel time per
snapshot and its HBM rate on algorithmic bytes (read w, wp: 32 B/cell; read
the basis: 16 B x n_pod per cell; write C: 8 B x n_pod per cell), and the D2H
time of C (PCIe-bound: C is n_pod x n doubles per snapshot).

    python tools/ecsw_probe.py [N] [npod] [nsnaps]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from finitedifference_amd.solver import FOMContext  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 250
npod = int(sys.argv[2]) if len(sys.argv) > 2 else 95
ns = int(sys.argv[3]) if len(sys.argv) > 3 else 50
rng = np.random.default_rng(1234557)
m = 2 * N * N
snaps = rng.uniform(1.0, 6.0, (m, ns))
prev = rng.uniform(1.0, 6.0, (m, ns))
basis = np.linalg.qr(rng.standard_normal((m, npod)))[0]
ctx = FOMContext(N, N)
g = np.linspace(0, 100, N + 1)
ctx.set_problem(g, g, 0.05, (5.19, 0.026))
ctx.ecsw_matrix(snaps[:, :2], prev[:, :2], basis)  # warm
t0 = time.perf_counter()
C, st = ctx.ecsw_matrix(snaps, prev, basis, return_stats=True)
wall = time.perf_counter() - t0
per_kern = st["loop_ms"] / ns
alg = (32 + 24 * npod) * N * N
print(json.dumps({
    "kernel": "ecsw_kernel", "grid": f"{N}x{N}", "n_pod": npod, "n_snaps": ns,
    "kernel_ms_per_snapshot": round(per_kern, 5),
    "alg_bytes_per_snapshot": alg, "achieved_GBs": round(alg / (per_kern * 1e-3) / 1e9, 1),
    "frac_of_8TBs": round(alg / (per_kern * 1e-3) / 8e12, 4),
    "d2h_ms_per_snapshot": round(st["flush_ms"] / ns, 4),
    "wall_s": round(wall, 3), "C_shape": list(C.shape)}), flush=True)
