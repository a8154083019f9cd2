"""LSPG PROM timing probe (burg_lspg): T steps of the
ROM at N^2 with an npod-vector basis (columns: the first FOM states of a
training trajectory, computed on the GPU, orthonormalised on the host), and
the fused J.basis + Gram kernel's achieved HBM rate on its algorithmic bytes
(2 * 2n * npod * 8 B of basis planes -- straight and transposed -- plus
4 * 2n * 8 B of state, its transpose and the residual, per launch).

    python tools/lspg_probe.py [N] [npod] [T]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 250
    npod = int(sys.argv[2]) if len(sys.argv) > 2 else 95
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    from finitedifference_amd.solver import FOMContext
    gx = np.linspace(0, 100, N + 1)
    m = 2 * N * N
    train = FOMContext(N, N)
    train.set_problem(gx, gx, 0.05, (4.25, 0.015))
    t = time.time()
    S, *_ = train.run(np.ones(m), 5 * npod, snap_every=5)
    t_fom = time.time() - t
    t = time.time()
    B = np.linalg.qr(S[:, 1:npod + 1])[0]
    t_qr = time.time() - t
    ctx = FOMContext(N, N)
    ctx.set_problem(gx, gx, 0.05, (4.75, 0.02))
    ctx.lspg(np.ones(m), 1, B, keep_snaps=False)  # warm-up
    snaps, red, its, rels, times, st = ctx.lspg(np.ones(m), T, B, keep_snaps=False)
    upd = st["newton_updates"]
    gram_ms = times[0] / max(upd, 1)
    alg = 2 * m * npod * 8 + 4 * m * 8
    out = {"N": N, "npod": npod, "steps": T, "gn_updates": upd, "its_per_step": its.tolist(),
           "loop_ms": st["loop_ms"], "ms_per_step": st["loop_ms"] / T,
           "gram_ms_per_launch": gram_ms, "res_ms_total": times[1], "ls_ms_total": times[2],
           "gram_alg_bytes": alg, "gram_GBps": alg / gram_ms / 1e6,
           "gram_frac_hbm": alg / gram_ms / 1e6 / 8000.0,
           "gram_gflops": 2 * m * (32 * ((npod + 32) // 32)) ** 2 / gram_ms / 1e6,
           "setup_fom_s": t_fom, "setup_qr_s": t_qr}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
