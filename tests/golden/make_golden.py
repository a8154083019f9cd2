"""Generate the golden fixtures in tests/golden/ from the Python reference.

Runs ONLY in the build container, where /root/reference exists; the fixtures
(small .npz/.json files: inputs and reference outputs, no reference source)
are committed and travel to the GPU box instead of the reference.

Recipe: PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg
OPENBLAS_NUM_THREADS=1, reference on sys.path, scratch cwd (the reference's
load_or_compute_snaps writes param_snaps/ into the cwd).

    python tests/golden/make_golden.py [--skip-750] [--coarse-npy PATH]

Fixtures written
  ref_small.npz      full reference trajectories (inviscid_burgers_implicit2D,
                     C/hypernet2D.py:72) at small square grids + Newton
                     update counts and printed relative residuals per step
  ref_ops.npz        single-call residual (res2D_alt, :2512), Jacobian action
                     (exact_jac2D @ x, :2627) and spsolve(J, r) (:1854) at
                     random states, seed 1234557 (C/config.py:12)
  ref_coarse250.npz  C/run_fom.py:main() defaults (250^2, 500 steps,
                     mu=(5.19, 0.026)): slices, column norms/sums, full
                     states at steps 1/100/500, Newton counts
  ref_fine750.npz    F/ grid 750^2, first 2 steps at mu=(5.19, 0.026)
  author_pickles.npz HDM mid-line slices byte-scanned (never unpickled) from
                     the author's C/ and F/ predict_mu_5.19e+00_2.60e-02_hprom.pickle
  ref_ecsw.npz       compute_ECSW_training_matrix_2D (:2719-2740) with the
                     reference's own callbacks (res2D, exact_jac2D) on
                     reference snapshots, the driver's 3-step offset sampling
                     (C/run_HPROM_ecsw_joshua_.py:81-84) and a POD basis
  ref_ecsw_variants.npz  the decoder variants compute_ECSW_training_matrix_2D_rnm /
                     _rbf_nearest_neighbors / _rbf_global / _gp (:2742-3072) and
                     their decoders (decode_* / jac_*, :1279-1808) on
                     reference snapshots with fixed latent models
                     (tests/ecsw_models.py)
  ref_lspg.npz       inviscid_burgers_implicit2D_LSPG (:133-200) + gauss_newton_LSPG
                     (:1859-1929) trajectories with POD bases of reference
                     snapshots at training mu, per-step Gauss-Newton counts
                     (from its printed 'iteration i' lines), and the LSPG
                     Jacobian (row-only JDyec permutation, :165-167) times the
                     basis at a random state
  ref_pod.npz        POD (:2670-2695) of reference snapshot sets: method 'svd'
                     (u, s) and method 'rsvd' with random_state=0 (10 modes)
  author_logs.json   Newton counts/residuals from the author's SLURM log
                     F/output_55034725.log (750^2)
"""
import argparse
import contextlib
import io
import json
import os
import pickletools
import re
import sys
import tempfile
import time

import numpy as np

REF = "/root/reference"
COARSE = os.path.join(REF, "BurgersFD_CleanCoarse")
FINE = os.path.join(REF, "BurgersFD_CleanFine")
HERE = os.path.dirname(os.path.abspath(__file__))
NEWTON_RE = re.compile(r"^(\d+): ([0-9.eE+-]+)\s*$")
SEED = 1234557  # C/config.py:12


def _import_reference():
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    sys.path.insert(0, COARSE)
    import hypernet2D  # noqa: E402  (reference module, build container only)
    return hypernet2D


def _newton_log(text):
    its, rel = [], []
    for line in text.splitlines():
        m = NEWTON_RE.match(line.strip())
        if m:
            its.append(int(m.group(1)))
            rel.append(float(m.group(2)))
    return np.array(its, dtype=np.int32), np.array(rel)


def run_reference(hn, N, T, mu, dt=0.05):
    gx, gy = hn.make_2D_grid(0, 100, 0, 100, N, N)
    w0 = np.ones(2 * N * N)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        snaps = hn.inviscid_burgers_implicit2D(gx, gy, w0, dt, T, list(mu))
    its, rel = _newton_log(buf.getvalue())
    assert its.size == T, (its.size, T)
    return snaps, its, rel


def make_small(hn):
    out = {}
    cases = [  # (tag, N, T, mu)
        ("n8", 8, 500, (5.19, 0.026)),
        ("n13", 13, 40, (5.19, 0.026)),
        ("n16", 16, 100, (5.19, 0.026)),
        ("n16b", 16, 60, (4.56, 0.019)),
        ("n50", 50, 20, (4.75, 0.02)),
        ("n100", 100, 6, (5.19, 0.026)),
    ]
    for tag, N, T, mu in cases:
        t = time.time()
        snaps, its, rel = run_reference(hn, N, T, mu)
        out[f"{tag}_snaps"] = snaps
        out[f"{tag}_its"] = its
        out[f"{tag}_rel"] = rel
        out[f"{tag}_meta"] = np.array([N, T, mu[0], mu[1], 0.05])
        print(f"small {tag}: N={N} T={T} {time.time() - t:.1f}s its={its[:6]}")
    np.savez_compressed(os.path.join(HERE, "ref_small.npz"), **out)


def make_ops(hn):
    import scipy.sparse.linalg as spla
    rng = np.random.default_rng(SEED)
    out = {}
    for N in (16, 64, 250):
        gx, gy = hn.make_2D_grid(0, 100, 0, 100, N, N)
        _, _, JDxec, JDyec, Eye = hn.get_ops(gx, gy)
        mu = [4.25 + 1.25 * rng.random(), 0.015 + 0.015 * rng.random()]
        dt = 0.05
        w = rng.uniform(1.0, 6.0, 2 * N * N)
        wp = rng.uniform(1.0, 6.0, 2 * N * N)
        x = rng.standard_normal(2 * N * N)
        r = hn.inviscid_burgers_res2D_alt(w, gx, gy, dt, wp, mu, JDxec, JDyec)
        J = hn.inviscid_burgers_exact_jac2D(w, dt, JDxec, JDyec, Eye)
        jx = J @ x
        r1 = hn.inviscid_burgers_res2D(w, gx, gy, dt, wp, mu,
                                       hn.make_ddx(gx), hn.make_ddx(gy))
        tag = f"n{N}"
        out[f"{tag}_mu"] = np.array(mu)
        if N <= 64:
            d = spla.spsolve(J.tocsc(), r)
            out.update({f"{tag}_w": w, f"{tag}_wp": wp, f"{tag}_x": x,
                        f"{tag}_res": r, f"{tag}_res1d": r1, f"{tag}_jx": jx,
                        f"{tag}_solve": d})
        else:  # 250^2: regenerate inputs from the seed in the test; keep summaries
            idx = rng.choice(2 * N * N, 512, replace=False)
            out.update({f"{tag}_w": w, f"{tag}_wp": wp, f"{tag}_x": x,
                        f"{tag}_res_norm": np.linalg.norm(r),
                        f"{tag}_res_idx": idx, f"{tag}_res_at": r[idx],
                        f"{tag}_jx_norm": np.linalg.norm(jx), f"{tag}_jx_at": jx[idx]})
        print(f"ops N={N} done")
    np.savez_compressed(os.path.join(HERE, "ref_ops.npz"), **out)


def make_ecsw(hn):
    out = {}
    for tag, N, T, mu, npod, f in (("n16", 16, 14, (4.56, 0.019), 6, 2),
                                   ("n24", 24, 10, (5.19, 0.026), 5, 3)):
        gx, gy = hn.make_2D_grid(0, 100, 0, 100, N, N)
        snaps, _, _ = run_reference(hn, N, T, mu)
        basis = np.linalg.svd(snaps, full_matrices=False)[0][:, :npod]
        s_use, s_prev = snaps[:, 3:T:f], snaps[:, 0:T - 3:f]
        C = hn.compute_ECSW_training_matrix_2D(s_use, s_prev, basis, hn.inviscid_burgers_res2D,
                                               hn.inviscid_burgers_exact_jac2D, gx, gy, 0.05,
                                               list(mu))
        out.update({f"{tag}_snaps": snaps, f"{tag}_basis": basis, f"{tag}_C": C,
                    f"{tag}_meta": np.array([N, T, mu[0], mu[1], 0.05, npod, f])})
        print(f"ecsw {tag}: C {C.shape}")
    np.savez_compressed(os.path.join(HERE, "ref_ecsw.npz"), **out)


RESID_RE = re.compile(r"^(Initial|Final)( reconstruction)? residual: ([0-9.eE+-]+)\s*$")


def make_ecsw_variants(hn):
    """ref_ecsw_variants.npz: the decoder variants of the ECSW training matrix
    (C/hypernet2D.py:2742-3072) on reference snapshots at 16^2, with POD
    primary/secondary bases of a 2-mu training set, a MinMaxScaler, a KD-tree,
    global RBF weights per kernel, a fixed-hyper-parameter Matern(1.5) GP and
    a float32 torch decoder for rnm (tests/ecsw_models.py rebuilds the same
    objects from the stored arrays); plus the decoders' own outputs
    (decode_* / jac_*, :1279-1808) at one reduced point, and the residuals
    the variants print per snapshot."""
    import torch
    from scipy.spatial.distance import pdist, squareform
    sys.path.insert(0, os.path.dirname(HERE))
    import ecsw_models as em
    from rbf_utils import RBFUtils  # reference module (build container only)
    N, T, dt, rp, rs, eps, k = 16, 14, 0.05, 4, 8, 1.0, 6
    mu = (4.56, 0.019)
    gx, gy = hn.make_2D_grid(0, 100, 0, 100, N, N)
    S = np.hstack([run_reference(hn, N, T, m)[0] for m in ((4.25, 0.015), (5.5, 0.03))])
    snaps = run_reference(hn, N, T, mu)[0]
    U = np.linalg.svd(S, full_matrices=False)[0]
    basis, basis2 = U[:, :rp], U[:, rp:rp + rs]
    qp_raw, Q = (basis.T @ S).T, (basis2.T @ S).T
    scaler = em.scaler_of(qp_raw)
    P = scaler.transform(qp_raw)
    kdtree = em.kdtree_of(P)
    s_use, s_prev = snaps[:, 3:T:3], snaps[:, 0:T - 3:3]
    y_probe = basis.T @ s_use[:, 1]
    res, jac = hn.inviscid_burgers_res2D, hn.inviscid_burgers_exact_jac2D
    out = dict(meta=np.array([N, T, mu[0], mu[1], dt, rp, rs, eps, k]), snaps=snaps, basis=basis,
               basis2=basis2, qp_raw=qp_raw, P=P, Q=Q, y_probe=y_probe)

    def run(tag, fn, *args):
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            C = fn(*args)
        resid = [float(m.group(3)) for m in map(RESID_RE.match, buf.getvalue().splitlines()) if m]
        assert len(resid) == 2 * s_use.shape[1], buf.getvalue()
        out[f"{tag}_C"], out[f"{tag}_resid"] = C, np.array(resid)
        print(f"ecsw variant {tag}: C {C.shape}, final residuals {resid[1::2]}")

    phis = {"gaussian": RBFUtils.gaussian_rbf, "imq": RBFUtils.inverse_multiquadric_rbf,
            "linear": RBFUtils.linear_rbf, "multiquadric": RBFUtils.multiquadric_rbf,
            "matern": RBFUtils.matern_kernel}
    for kt in em.RBF_KERNELS_NN:
        run(f"nn_{kt}", hn.compute_ECSW_training_matrix_2D_rbf_nearest_neighbors, s_use, s_prev,
            basis, basis2, eps, k, kdtree, P, Q, res, jac, gx, gy, dt, list(mu), scaler, kt)
        out[f"nn_{kt}_dec"] = hn.decode_rbf_nearest_neighbors(y_probe, eps, k, kdtree, P, Q, basis,
                                                              basis2, scaler, kt)
        out[f"nn_{kt}_jac"] = hn.jac_rbf_nearest_neighbors(y_probe, kdtree, P, Q, basis, basis2,
                                                           eps, k, scaler, kt)
    for kt in em.RBF_KERNELS_GLOBAL:
        W = np.linalg.solve(phis[kt](squareform(pdist(P)), eps) + 1e-8 * np.eye(P.shape[0]), Q)
        out[f"glob_{kt}_W"] = W
        run(f"glob_{kt}", hn.compute_ECSW_training_matrix_2D_rbf_global, s_use, s_prev, basis,
            basis2, W, P, Q, res, jac, gx, gy, dt, list(mu), scaler, eps, kt)
        out[f"glob_{kt}_dec"] = hn.decode_rbf_global(y_probe, W, P, basis, basis2, eps, scaler, kt)
        out[f"glob_{kt}_jac"] = hn.jac_rbf_global(y_probe, W, P, Q, basis, basis2, eps, scaler, kt)
    gp_par = np.array([1.5, 0.6, 1e-8])  # ConstantKernel value, Matern length scale, alpha
    gp = em.gp_of(P, Q, *gp_par)
    out["gp_par"] = gp_par
    run("gp", hn.compute_ECSW_training_matrix_2D_gp, s_use, s_prev, basis, basis2, gp, res, jac,
        gx, gy, dt, list(mu), scaler)
    out["gp_dec"] = hn.decode_gp(y_probe, gp, basis, basis2, scaler)
    out["gp_jac"] = hn.jac_gp(y_probe, gp, basis, basis2, scaler)
    rng = np.random.default_rng(SEED)
    A, b = 0.05 * rng.standard_normal((rs, rp)), 0.1 * rng.standard_normal(rs)
    approx, jacfwd = em.nn_decoder_of(basis, basis2, A, b)
    out["rnm_A"], out["rnm_b"] = A, b
    run("rnm", hn.compute_ECSW_training_matrix_2D_rnm, s_use, s_prev, basis, approx, jacfwd, res,
        jac, gx, gy, dt, list(mu))
    assert torch.get_default_dtype() == torch.float32
    np.savez_compressed(os.path.join(HERE, "ref_ecsw_variants.npz"), **out)


GN_RE = re.compile(r"^iteration (\d+): relative norm ([0-9.eE+-]+)\s*$")


def make_lspg(hn):
    import scipy.sparse as sp
    rng = np.random.default_rng(SEED)
    out = {}
    # (tag, N, T, training mus, npod, rom mu)
    for tag, N, T, train, npod, mu in (
            ("n16", 16, 30, ((4.25, 0.015), (5.5, 0.03)), 6, (4.75, 0.02)),
            ("n24", 24, 20, ((4.25, 0.015), (5.5, 0.03), (5.19, 0.026)), 12, (4.56, 0.019)),
            ("n32", 32, 12, ((4.25, 0.03), (5.5, 0.015)), 20, (5.19, 0.026))):
        gx, gy = hn.make_2D_grid(0, 100, 0, 100, N, N)
        S = np.hstack([run_reference(hn, N, T, m)[0] for m in train])
        basis = np.linalg.svd(S, full_matrices=False)[0][:, :npod]
        w0 = np.ones(2 * N * N)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            snaps, stats = hn.inviscid_burgers_implicit2D_LSPG(gx, gy, w0, 0.05, T, list(mu), basis)
        gn = [GN_RE.match(l.strip()) for l in buf.getvalue().splitlines()]
        its = np.array([int(m.group(1)) + 1 for m in gn if m], dtype=np.int32)
        rel = np.array([float(m.group(2)) for m in gn if m])
        assert its.size == T and its.sum() == stats[0], (its, stats)
        # the LSPG Jacobian (JDyec rows permuted only, :165-167) times the basis
        Dxec, Dyec = hn.make_ddx(gx), hn.make_ddx(gy)
        JDxec = sp.kron(sp.eye(N), Dxec)
        JDyec = sp.kron(sp.eye(N), Dyec)
        JDyec = JDyec.tocsr()[np.arange(N * N).reshape(N, -1).T.flatten(), :]
        Eye = sp.eye(2 * N * N)
        w = rng.uniform(1.0, 6.0, 2 * N * N)
        JV = hn.inviscid_burgers_exact_jac2D(w, 0.05, JDxec, JDyec, Eye).dot(basis)
        out.update({f"{tag}_snaps": snaps, f"{tag}_basis": basis, f"{tag}_its": its,
                    f"{tag}_rel": rel, f"{tag}_w": w, f"{tag}_JV": JV,
                    f"{tag}_meta": np.array([N, T, mu[0], mu[1], 0.05, npod])})
        print(f"lspg {tag}: its {its.tolist()}")
    np.savez_compressed(os.path.join(HERE, "ref_lspg.npz"), **out)


def make_pod(hn):
    out = {}
    for tag, N, T, mus in (("n16", 16, 30, ((4.25, 0.015), (5.5, 0.03))),
                           ("n24", 24, 20, ((4.25, 0.015), (5.5, 0.03), (5.19, 0.026)))):
        S = np.hstack([run_reference(hn, N, T, m)[0] for m in mus])
        u, s = hn.POD(S, method="svd")
        ur, sr = hn.POD(S, num_modes=10, method="rsvd", random_state=0)
        out.update({f"{tag}_S": S, f"{tag}_u": u, f"{tag}_s": s, f"{tag}_ur": ur,
                    f"{tag}_sr": sr})
        print(f"pod {tag}: S {S.shape}, s[0] {s[0]:.6e}, s[-1] {s[-1]:.3e}")
    np.savez_compressed(os.path.join(HERE, "ref_pod.npz"), **out)


def _summaries(snaps, N, steps_full):
    n = N * N
    T1 = snaps.shape[1]
    mid = N // 2
    every = np.arange(0, T1, 10)
    U = snaps[:n, every].reshape(N, N, -1)
    V = snaps[n:, every].reshape(N, N, -1)
    out = {
        "slice_steps": every,
        "u_row": U[mid, :, :].T.copy(), "u_col": U[:, mid, :].T.copy(),
        "v_row": V[mid, :, :].T.copy(), "v_col": V[:, mid, :].T.copy(),
        "col_norm": np.sqrt(np.square(snaps).sum(axis=0)),
        "col_sum": snaps.sum(axis=0),
    }
    for j in steps_full:
        if j < T1:
            out[f"state_{j}"] = snaps[:, j].copy()
    return out


def make_coarse250(hn, coarse_npy=None, coarse_log=None):
    N, T = 250, 500
    if coarse_npy and os.path.exists(coarse_npy):
        # cached output of this same recipe (C/run_fom.py main(), 623 s here)
        snaps = np.load(coarse_npy, mmap_mode="r")
        its, rel = _newton_log(open(coarse_log).read())
        print("coarse250: using cached reference trajectory", coarse_npy)
    else:
        t = time.time()
        snaps, its, rel = run_reference(hn, N, T, (5.19, 0.026))
        print(f"coarse250: reference run {time.time() - t:.0f}s")
    out = _summaries(np.asarray(snaps), N, (1, 2, 100, 500))
    out["its"], out["rel"] = its, rel
    np.savez_compressed(os.path.join(HERE, "ref_coarse250.npz"), **out)


def make_fine750(hn):
    N, T = 750, 2
    t = time.time()
    snaps, its, rel = run_reference(hn, N, T, (5.19, 0.026))
    print(f"fine750: {time.time() - t:.0f}s its={its} rel={rel}")
    out = _summaries(snaps, N, ())
    out["its"], out["rel"] = its, rel
    mid = N // 2
    out["u_row_all"] = snaps[:N * N].reshape(N, N, -1)[mid, :, :].T.copy()
    out["v_col_all"] = snaps[N * N:].reshape(N, N, -1)[:, mid, :].T.copy()
    np.savez_compressed(os.path.join(HERE, "ref_fine750.npz"), **out)


def scan_pickle(path, N):
    """HDM slices from the author's pickled Figure, by scanning byte payloads
    with pickletools.genops (nothing is unpickled or executed)."""
    data = open(path, "rb").read()
    arrs = []
    for op, arg, _pos in pickletools.genops(io.BytesIO(data)):
        if op.name in ("SHORT_BINBYTES", "BINBYTES", "BINBYTES8") and len(arg) == 8 * N:
            arrs.append(np.frombuffer(arg, dtype="<f8").copy())
    g = np.linspace(0, 100, N + 1)
    xc = (g[1:] + g[:-1]) / 2
    ys = [a for a in arrs if not np.array_equal(a, xc)]
    # each line is stored twice (_xorig/_x paths): keep one of each pair
    ys = ys[::2]
    assert len(ys) == 24, len(ys)
    # order: axis-1 (row N//2) HDM x6, HPROM x6; axis-2 (column N//2) HDM x6, HPROM x6
    return np.stack(ys[0:6]), np.stack(ys[12:18])


def make_pickles():
    out = {}
    for tag, d, N in (("coarse", COARSE, 250), ("fine", FINE, 750)):
        row, col = scan_pickle(os.path.join(d, "predict_mu_5.19e+00_2.60e-02_hprom.pickle"), N)
        out[f"{tag}_u_row"] = row
        out[f"{tag}_u_col"] = col
        out[f"{tag}_steps"] = np.arange(0, 501, 100)
    np.savez_compressed(os.path.join(HERE, "author_pickles.npz"), **out)
    print("pickles done")


def make_logs():
    out = {}
    for name in ("output_55034725.log", "output_54767262.log"):
        text = open(os.path.join(FINE, name)).read()
        runs, cur, mu = [], None, None
        for line in text.splitlines():
            m = re.match(r"^Running HDM for mu1=([0-9.]+)", line)
            if m:
                cur = {"mu1": float(m.group(1)), "its": [], "rel": []}
                runs.append(cur)
                continue
            m = NEWTON_RE.match(line.strip())
            if m and cur is not None and len(cur["its"]) < 500:
                cur["its"].append(int(m.group(1)))
                cur["rel"].append(float(m.group(2)))
            m = re.match(r"^Elapsed time: ([0-9.e+]+)", line)
            if m and cur is not None and "elapsed_s" not in cur:
                cur["elapsed_s"] = float(m.group(1))
        out[name] = runs
    with open(os.path.join(HERE, "author_logs.json"), "w") as f:
        json.dump(out, f)
    print("logs done")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-750", action="store_true")
    ap.add_argument("--coarse-npy", default="/tmp/oracle_probe/hdm_snaps_mu1_5.19_mu2_0.026.npy")
    ap.add_argument("--coarse-log", default="/tmp/oracle_probe/coarse_full.log")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    only = set(args.only.split(",")) if args.only else None
    make_pickles() if not only or "pickles" in only else None
    make_logs() if not only or "logs" in only else None
    scratch = tempfile.mkdtemp(prefix="golden_")
    cwd = os.getcwd()
    os.chdir(scratch)
    try:
        hn = _import_reference()
        if not only or "small" in only:
            make_small(hn)
        if not only or "ops" in only:
            make_ops(hn)
        if not only or "ecsw" in only:
            make_ecsw(hn)
        if not only or "ecsw_variants" in only:
            make_ecsw_variants(hn)
        if not only or "pod" in only:
            make_pod(hn)
        if not only or "lspg" in only:
            make_lspg(hn)
        if not only or "coarse" in only:
            make_coarse250(hn, args.coarse_npy, args.coarse_log)
        if (not only or "fine" in only) and not args.skip_750:
            make_fine750(hn)
    finally:
        os.chdir(cwd)


if __name__ == "__main__":
    main()
