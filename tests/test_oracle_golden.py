"""Pin the CPU oracle to the reference (CPU only, no GPU).

The oracle (oracle/burgers_oracle.c) is the checker of every GPU parity test,
so it is checked here against every golden vector the reference provides:
fixtures made by importing the Python reference (tests/golden/make_golden.py),
the author's pickled HDM slices and the author's SLURM Newton logs.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(b))


# ---------------------------------------------------------- single calls ---
@pytest.mark.parametrize("N", [16, 64, 250])
def test_residual_vs_reference(orc, N):
    g = golden("ref_ops.npz")
    P = orc.Problem(N, mu=tuple(g[f"n{N}_mu"]))
    r = P.residual(g[f"n{N}_w"], g[f"n{N}_wp"])
    if N <= 64:
        assert rel(r, g[f"n{N}_res"]) <= 1e-15
        # res2D (1-D operator form, C/hypernet2D.py:2468) is the same residual
        assert rel(r, g[f"n{N}_res1d"]) <= 1e-15
    else:
        assert np.allclose(r[g["n250_res_idx"]], g["n250_res_at"], rtol=1e-14, atol=0)
        assert abs(np.linalg.norm(r) - g["n250_res_norm"]) <= 1e-13 * g["n250_res_norm"]


@pytest.mark.parametrize("N", [16, 64, 250])
def test_jvp_vs_reference(orc, N):
    g = golden("ref_ops.npz")
    P = orc.Problem(N, mu=tuple(g[f"n{N}_mu"]))
    y = P.jvp(g[f"n{N}_w"], g[f"n{N}_x"])
    if N <= 64:
        assert rel(y, g[f"n{N}_jx"]) <= 1e-14
    else:
        assert abs(np.linalg.norm(y) - g["n250_jx_norm"]) <= 1e-13 * g["n250_jx_norm"]


@pytest.mark.parametrize("N", [16, 64])
def test_block_solve_vs_spsolve(orc, N):
    g = golden("ref_ops.npz")
    P = orc.Problem(N, mu=tuple(g[f"n{N}_mu"]))
    d = P.block_solve(g[f"n{N}_w"], g[f"n{N}_res"])
    assert rel(d, g[f"n{N}_solve"]) <= 1e-13
    # and it is the inverse of the Jacobian action
    assert rel(P.jvp(g[f"n{N}_w"], d), g[f"n{N}_res"]) <= 1e-13


# ------------------------------------------------------ trajectories -------
@pytest.mark.parametrize("tag", ["n8", "n13", "n16", "n16b", "n50", "n100"])
def test_newton_fom_reproduces_reference(orc, tag):
    g = golden("ref_small.npz")
    N, T, mu1, mu2, dt = g[f"{tag}_meta"]
    N, T = int(N), int(T)
    P = orc.Problem(N, dt=dt, mu=(mu1, mu2))
    snaps, its, rl = P.fom(np.ones(2 * N * N), T, solver="newton")
    ref = g[f"{tag}_snaps"]
    assert np.array_equal(its, g[f"{tag}_its"])
    assert max(rel(snaps[j], ref[:, j]) for j in range(1, T + 1)) <= 1e-13


@pytest.mark.parametrize("tag", ["n8", "n13", "n16", "n16b", "n50", "n100"])
def test_march_fom_matches_reference(orc, tag):
    g = golden("ref_small.npz")
    N, T, mu1, mu2, dt = g[f"{tag}_meta"]
    N, T = int(N), int(T)
    P = orc.Problem(N, dt=dt, mu=(mu1, mu2))
    snaps, _, _ = P.fom(np.ones(2 * N * N), T, solver="march")
    ref = g[f"{tag}_snaps"]
    assert max(rel(snaps[j], ref[:, j]) for j in range(1, T + 1)) <= 1e-12


def test_coarse250_reference_run(orc):
    """C/run_fom.py defaults, all 500 steps, against the reference run."""
    g = golden("ref_coarse250.npz")
    N, T = 250, 500
    P = orc.Problem(N)
    snaps, _, _ = P.fom(np.ones(2 * N * N), T, solver="march")
    for j in (1, 2, 100, 500):
        assert rel(snaps[j], g[f"state_{j}"]) <= 1e-12
    assert np.allclose(np.sqrt(np.square(snaps).sum(axis=1)), g["col_norm"], rtol=1e-12, atol=0)
    assert np.allclose(snaps.sum(axis=1), g["col_sum"], rtol=1e-12, atol=0)
    n = N * N
    steps = g["slice_steps"]
    U = snaps[steps, :n].reshape(len(steps), N, N)
    V = snaps[steps, n:].reshape(len(steps), N, N)
    assert rel(U[:, N // 2, :], g["u_row"]) <= 1e-12
    assert rel(U[:, :, N // 2], g["u_col"]) <= 1e-12
    assert rel(V[:, N // 2, :], g["v_row"]) <= 1e-12
    assert rel(V[:, :, N // 2], g["v_col"]) <= 1e-12


def test_coarse250_newton_counts_vs_reference_log(orc):
    """Per-step Newton update counts of the reference's 250^2 run."""
    g = golden("ref_coarse250.npz")
    N, T = 250, 60
    P = orc.Problem(N)
    _, its, rl = P.fom(np.ones(2 * N * N), T, solver="newton")
    assert np.array_equal(its, g["its"][:T])
    # printed relative residuals agree to the printed precision (3 digits)
    assert np.allclose(rl, g["rel"][:T], rtol=1e-2, atol=0)


def test_author_pickle_coarse(orc):
    """The author's own pickled HDM slices (C/predict_mu_5.19e+00_2.60e-02_hprom.pickle)."""
    g = golden("author_pickles.npz")
    N, T = 250, 500
    P = orc.Problem(N)
    snaps, _, _ = P.fom(np.ones(2 * N * N), T, solver="march")
    n = N * N
    for k, j in enumerate(g["coarse_steps"]):
        u = snaps[j, :n].reshape(N, N)
        assert rel(u[N // 2, :], g["coarse_u_row"][k]) <= 1e-12
        assert rel(u[:, N // 2], g["coarse_u_col"][k]) <= 1e-12


@pytest.mark.slow
def test_author_pickle_fine750(orc):
    """F/ grid (750^2), 500 steps, against the author's pickled slices."""
    g = golden("author_pickles.npz")
    N = 750
    P = orc.Problem(N)
    w = np.ones(2 * N * N)
    n = N * N
    for step in range(501):
        if step % 100 == 0:
            k = step // 100
            u = w[:n].reshape(N, N)
            assert rel(u[N // 2, :], g["fine_u_row"][k]) <= 1e-12
            assert rel(u[:, N // 2], g["fine_u_col"][k]) <= 1e-12
        if step < 500:
            w = P.march_step(w)


def test_fine750_first_steps_and_author_log(orc):
    """750^2: reference run (2 steps) and the author's SLURM log
    F/output_55034725.log (Newton counts 5, 4, ... ; printed residuals)."""
    g = golden("ref_fine750.npz")
    logs = json.load(open(os.path.join(GOLDEN, "author_logs.json")))
    run = logs["output_55034725.log"][0]
    assert run["mu1"] == 5.19
    N = 750
    P = orc.Problem(N)
    w = np.ones(2 * N * N)
    w1, its1, rel1 = P.newton_step(w)
    w2, its2, rel2 = P.newton_step(w1)
    assert [its1, its2] == list(g["its"]) == run["its"][:2]
    assert f"{rel1:3.2e}" == f"{run['rel'][0]:3.2e}"  # "5.82e-16" in the author's log
    n = N * N
    assert rel(w2[:n].reshape(N, N)[N // 2, :], g["u_row_all"][2]) <= 1e-13
    assert rel(w2[n:].reshape(N, N)[:, N // 2], g["v_col_all"][2]) <= 1e-13
    m1 = P.march_step(w)
    assert rel(m1, w1) <= 1e-13
    assert np.all(np.asarray(run["its"][1:]) == 4)


# ------------------------------------------------- tile schedule (engine) --
@pytest.mark.parametrize("N,tw", [(13, 64), (130, 64), (250, 128)])
def test_tile_schedule_bitwise_at_tol0(orc, N, tw):
    P = orc.Problem(N)
    w = np.ones(2 * N * N)
    for _ in range(5):
        w = P.march_step(w)
    ws, k, done = P.march_tiled(w, tw=tw, tol=0.0)
    assert np.array_equal(ws, P.march_step(w))


def test_tile_schedule_converges_in_few_passes(orc):
    N = 512
    P = orc.Problem(N)
    w = np.ones(2 * N * N)
    for _ in range(30):
        w = P.march_step(w)
    ws, k, done = P.march_tiled(w, tw=64, tol=2.0 ** -50)
    assert k <= 6
    assert rel(ws, P.march_step(w)) <= 1e-15


def test_oracle_ecsw_matrix_vs_reference():
    """Oracle restatement of compute_ECSW_training_matrix_2D (C/hypernet2D.py:
    2719-2740) against the reference's own output (tests/golden/ref_ecsw.npz,
    generated by importing the reference: make_golden.py --only ecsw)."""
    from oracle import oracle
    g = golden("ref_ecsw.npz")
    for tag in ("n16", "n24"):
        N, T, m1, m2, dt, npod, f = g[f"{tag}_meta"]
        N, T, f = int(N), int(T), int(f)
        P = oracle.Problem(N, mu=(m1, m2), dt=dt)
        sn = g[f"{tag}_snaps"]
        C = P.ecsw_matrix(sn[:, 3:T:f], sn[:, 0:T - 3:f], g[f"{tag}_basis"])
        ref = g[f"{tag}_C"]
        assert C.shape == ref.shape == (int(npod) * len(range(3, T, f)), N * N)
        assert np.linalg.norm(C - ref) <= 1e-14 * np.linalg.norm(ref)


# ------------------------------------------------ LSPG PROM --
@pytest.mark.parametrize("tag", ["n16", "n24", "n32"])
def test_oracle_lspg_vs_reference(orc, tag):
    """oracle Problem.lspg_jvp / lspg (restating inviscid_burgers_implicit2D_LSPG,
    C/hypernet2D.py:133-200, and gauss_newton_LSPG, :1859-1929) against the
    reference's own outputs (tests/golden/ref_lspg.npz): the LSPG Jacobian with
    the row-only JDyec permutation times the basis, the ROM trajectory and the
    per-step Gauss-Newton counts (its printed 'iteration i' lines; the printed
    relative norm carries 3 significant digits)."""
    g = golden("ref_lspg.npz")
    N, T, m1, m2, dt, npod = g[f"{tag}_meta"]
    N, T, npod = int(N), int(T), int(npod)
    P = orc.Problem(N, dt=dt, mu=(m1, m2))
    B = g[f"{tag}_basis"]
    JV = np.stack([P.lspg_jvp(g[f"{tag}_w"], B[:, k]) for k in range(npod)], axis=1)
    assert orc.rel_l2(JV, g[f"{tag}_JV"]) < 1e-14
    snaps, its, rels = P.lspg(np.ones(2 * N * N), T, B)
    assert orc.rel_l2(snaps, g[f"{tag}_snaps"]) < 1e-13
    assert np.array_equal(its, g[f"{tag}_its"])
    assert np.allclose(rels, g[f"{tag}_rel"], rtol=1e-2)


# ------------------------------------------------------- POD --
@pytest.mark.parametrize("tag", ["n16", "n24"])
def test_oracle_pod_vs_reference(orc, tag):
    """oracle.pod_svd restates POD(method='svd') (C/hypernet2D.py:2670-2695);
    against the reference's own output (tests/golden/ref_pod.npz), signs
    normalised on both sides."""
    g = golden("ref_pod.npz")
    u, s = orc.pod_svd(g[f"{tag}_S"])
    assert np.allclose(s, g[f"{tag}_s"], rtol=0, atol=1e-12 * s[0])
    ur = orc.svd_flip_u(g[f"{tag}_u"])
    keep = s > 1e-6 * s[0]
    assert keep.sum() >= 8
    assert np.max(np.abs(u[:, keep] - ur[:, keep])) < 1e-8


def test_oracle_under_sanitizers():
    """Host sanitizers over the CPU oracle (AddressSanitizer +
    UndefinedBehaviorSanitizer, oracle/sanitize_check.c via `make -C oracle
    sanitize`): every entry point on a ragged 37 x 23 grid, Newton = march to
    1e-12, the tile schedule simulator bitwise = the march, the OpenMP sweep,
    and J x / block solve inverse to each other; any sanitizer report fails."""
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    odir = os.path.join(os.path.dirname(here), "oracle")
    b = subprocess.run(["make", "-s", "-C", odir, "sanitize"], capture_output=True, text=True)
    if b.returncode != 0 and "asan" in (b.stderr + b.stdout).lower():
        pytest.skip("no sanitizer runtime for this compiler: " + b.stderr[-200:])
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="2")
    r = subprocess.run([os.path.join(odir, "_san", "sanitize_check")], capture_output=True,
                       text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize_check ok" in r.stdout


@pytest.mark.parametrize("nx,ny,T,every,threads", [(37, 23, 5, 1, 3), (200, 130, 7, 2, 8),
                                                   (64, 64, 4, 4, 5), (130, 1, 3, 1, 4)])
def test_row_pipelined_march_is_the_serial_march(orc, nx, ny, T, every, threads):
    """orc_march_traj_par (rows pipelined over OpenMP threads; the checker of
    the bench-size GPU trajectories in tests/test_gpu_regime.py) equals
    orc_march_step's trajectory bit for bit, including tiny/subnormal states
    (the IEEE slow path's inputs)."""
    P = orc.Problem(nx, ny, Ly=100.0 * ny / nx, allow_nonsquare=nx != ny)
    w0 = np.ones(P.m)
    w0[nx * ny:][::7] = 5e-320
    ref, _, _ = P.fom(w0, T)
    out = P.march_traj(w0, T, every, threads=threads)
    assert out.shape == (T // every + 1, P.m)
    for j in range(out.shape[0]):
        assert np.array_equal(out[j], ref[j * every]), j
