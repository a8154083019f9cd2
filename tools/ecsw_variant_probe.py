"""ECSW decoder variants (ecsw.py; C/hypernet2D.py:2785-2860 / 2862-2958 /
2960-3072) on the GPU at the reference driver's shape: 250^2, one mu block of
50 snapshots (snaps[:, 1::10], C/run_POD_RBF_HPROM_ecsw_joshua.py:41-47),
U_p 10 primary and U_s 140 secondary modes, 25 neighbours.  Inputs are
synthetic: the build's own 250^2 trajectories at three training mus (POD of
them gives U_p, U_s and the training coordinates), the test mu's snapshots
for C.  Prints one JSON line per variant: wall time per snapshot, the
kernel's share, Gauss-Newton counts are the reference's loop.

    python tools/ecsw_variant_probe.py [N] [rp] [rs] [nsnaps]
"""
import contextlib
import io
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ecsw_models as em  # noqa: E402
from finitedifference_amd import hypernet2D as H  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 250
rp = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rs = int(sys.argv[3]) if len(sys.argv) > 3 else 140
ns = int(sys.argv[4]) if len(sys.argv) > 4 else 50
T, dt = 500, 0.05
gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
w0 = np.ones(2 * N * N)
with contextlib.redirect_stdout(io.StringIO()):
    S = np.hstack([H.inviscid_burgers_implicit2D(gx, gy, w0, dt, T, mu, verbose=0)[:, ::5]
                   for mu in ((4.25, 0.015), (5.5, 0.03), (4.875, 0.0225))])
    test = H.inviscid_burgers_implicit2D(gx, gy, w0, dt, T, (4.56, 0.019), verbose=0)
U, _ = H.POD(S)
Up, Us = U[:, :rp], U[:, rp:rp + rs]
qp_raw, Q = (Up.T @ S).T, (Us.T @ S).T
scaler = em.scaler_of(qp_raw)
P = scaler.transform(qp_raw)
tree = em.kdtree_of(P)
snaps, prev = test[:, 1::10][:, :ns], test[:, :-1:10][:, :ns]
mu = (4.56, 0.019)
eps, k = 1.0, 25
from scipy.spatial.distance import pdist, squareform  # noqa: E402
Wg = np.linalg.solve(np.exp(-(eps * squareform(pdist(P))) ** 2) + 1e-8 * np.eye(P.shape[0]), Q)
gp = em.gp_of(P, Q, 1.5, 0.6, 1e-8)
cases = {
    "rbf_nearest_neighbors": lambda: H.compute_ECSW_training_matrix_2D_rbf_nearest_neighbors(
        snaps, prev, Up, Us, eps, k, tree, P, Q, None, None, gx, gy, dt, mu, scaler, "gaussian",
        verbose=False),
    "rbf_global": lambda: H.compute_ECSW_training_matrix_2D_rbf_global(
        snaps, prev, Up, Us, Wg, P, Q, None, None, gx, gy, dt, mu, scaler, eps, "gaussian",
        verbose=False),
    "gp": lambda: H.compute_ECSW_training_matrix_2D_gp(
        snaps, prev, Up, Us, gp, None, None, gx, gy, dt, mu, scaler, verbose=False),
}
for name, fn in cases.items():
    fn()  # warm (rocBLAS handles, allocations)
    t0 = time.perf_counter()
    if os.environ.get("PROBE_PROFILE"):  # host-side profile of the timed call -> stderr
        import cProfile
        import pstats
        pr = cProfile.Profile()
        C = pr.runcall(fn)
        pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(20)
    else:
        C = fn()
    wall = time.perf_counter() - t0
    print(json.dumps({"variant": name, "grid": f"{N}x{N}", "r_p": rp, "r_s": rs, "n_snaps": ns,
                      "C_shape": list(C.shape), "wall_s": round(wall, 4),
                      "ms_per_snapshot": round(1e3 * wall / ns, 3)}), flush=True)
