"""Drop-in host API for the reference FOM hot path (MI355X-backed).

Same names, argument meaning, return layout and error behaviour as the
reference module ``hypernet2D`` for the FOM path (paths relative to
/root/reference, C/ = BurgersFD_CleanCoarse/):

  make_2D_grid                  C/hypernet2D.py:2425-2431
  make_ddx / get_ops            C/hypernet2D.py:2410-2416, 2433-2444 (scipy setup)
  inviscid_burgers_implicit2D   C/hypernet2D.py:72-131     -> burg_run (HIP)
  inviscid_burgers_res2D_alt    C/hypernet2D.py:2512-2570  -> burg_residual (HIP)
  inviscid_burgers_res2D        C/hypernet2D.py:2468-2510  -> burg_residual (HIP)
  plot_snaps                    C/hypernet2D.py:3147-3180  (matplotlib, host)
  inviscid_burgers_exact_jac2D  C/hypernet2D.py:2627-2656  -> JacobianOperator
                                (burg_jvp / burg_block_solve, HIP)
  newton_raphson                C/hypernet2D.py:1811-1857  (host control loop)
  compute_error                 C/hypernet2D.py:3074-3079
  param_to_snap_fn              C/hypernet2D.py:3081-3105
  get_saved_params              C/hypernet2D.py:3107-3109
  load_or_compute_snaps         C/hypernet2D.py:3111-3145
  compute_ECSW_training_matrix_2D (+ _rnm, _rbf_nearest_neighbors,
    _rbf_global, _gp)           C/hypernet2D.py:2719-3072 -> ecsw.py (HIP)
  decode_/jac_rbf_nearest_neighbors, decode_/jac_rbf_global, decode_gp,
    jac_gp, matern15_grad       C/hypernet2D.py:1279-1495, 1720-1808
                                -> rom_decoders.py (host model code)

The snapshot matrix is the reference's: float64, shape (2*nx*ny,
num_steps + 1), C-contiguous, column j = state after j steps, u rows then v
rows.  Extensions are keyword-only (solver, snap_every, device, tile_w, tol,
par_passes, verbose, allow_nonsquare) and default to reference behaviour.
"""
import ctypes
import glob
import os
import time

import numpy as np
import scipy.sparse as sp
from scipy.sparse.linalg import LinearOperator

from .dist import agree, job, job_context, job_device, shared_tmp_path, slabs_to_npy
from .grid import fom_coefficients, make_2D_grid  # noqa: F401  (re-export)
from .solver import DEFAULT_TOL, get_context
from .ecsw import (compute_ECSW_training_matrix_2D_gp,  # noqa: F401  (re-export)
                   compute_ECSW_training_matrix_2D_rbf_global,
                   compute_ECSW_training_matrix_2D_rbf_nearest_neighbors,
                   compute_ECSW_training_matrix_2D_rnm)
from .rom_decoders import (decode_gp, decode_rbf_global,  # noqa: F401  (re-export)
                           decode_rbf_nearest_neighbors, jac_gp, jac_rbf_global,
                           jac_rbf_nearest_neighbors, matern15_grad)


def make_ddx(grid_x):
    """Backward-difference operator (C/hypernet2D.py:2410-2416); setup only."""
    dx = grid_x[1:] - grid_x[:-1]
    return sp.spdiags([-np.ones(grid_x.size - 1) / dx, np.ones(grid_x.size - 1) / dx],
                      [-1, 0], grid_x.size - 1, grid_x.size - 1, "lil")


def get_ops(grid_x, grid_y):
    """(Dxec, Dyec, JDxec, JDyec, Eye) as the reference builds them
    (C/hypernet2D.py:2433-2444).  Only needed by callers that pass operators
    around; the HIP path computes the stencil from the grid directly."""
    Dxec = make_ddx(grid_x)
    Dyec = make_ddx(grid_y)
    JDxec = sp.kron(sp.eye(grid_y.size - 1, grid_y.size - 1), Dxec)
    JDyec = sp.kron(sp.eye(grid_x.size - 1, grid_x.size - 1), Dyec)
    JDyec = JDyec.tocsr()
    idx = np.arange((grid_y.size - 1) * (grid_x.size - 1)).reshape(
        (grid_y.size - 1, grid_x.size - 1)).T.ravel()
    JDyec = JDyec[idx, :]
    JDyec = JDyec[:, idx]
    Eye = sp.identity(2 * (grid_x.size - 1) * (grid_y.size - 1))
    return Dxec, Dyec, JDxec, JDyec, Eye


def _ctx_for(grid_x, grid_y, dt, mu, device=0, allow_nonsquare=False, **opts):
    nx, ny = np.asarray(grid_x).size - 1, np.asarray(grid_y).size - 1
    ctx = get_context(nx, ny, job_device(device), **opts)
    ctx.set_problem(grid_x, grid_y, dt, mu, allow_nonsquare)
    return ctx


def inviscid_burgers_implicit2D(grid_x, grid_y, w0, dt, num_steps, mu, *, solver="march",
                                snap_every=1, device=None, engine="pipe", tile_w=64,
                                tol=DEFAULT_TOL, par_passes=0, verbose=1, allow_nonsquare=False,
                                newton_max_its=100, newton_rtol=1e-12, return_stats=False,
                                out=None, stream_w=0, tiles_target=0):
    """Implicit (trapezoidal-flux) time stepping of the 2D inviscid Burgers FOM
    (C/hypernet2D.py:72-131) on an MI355X.

    solver="march" (default) solves each implicit step exactly with the
    closed-form upwind march, by default on the pipe engine (engine="pipe":
    all steps in one pipelined launch, bitwise the sequential march;
    engine="stream" the streaming engine it grew from, engine="tiles" the
    per-step block-Jacobi tile engine, tuned by tile_w / tol / par_passes);
    solver="newton" runs the reference algorithm
    (newton_raphson, max_its=100, relnorm_cutoff=1e-12, exact block solve).
    Both return the reference's snapshot matrix.  verbose=1 (default) prints
    what the reference prints, unchanged: the header line, then per step
    " ... Working on timestep i" (C/hypernet2D.py:122) and, for the newton
    solver, Newton's "k: rel" line (:1844) -- after the run, since the whole
    time loop is one launch.  The march solver runs no Newton iteration, so
    it prints no Newton line (it does not emulate one); verbose=0 prints
    nothing.  out: an existing
    (2n, num_steps//snap_every + 1) C-contiguous float64 array (e.g. a .npy
    memmap) the snapshots are written into and returned.

    Multi-GPU (launched under torchrun, one process per GPU, WORLD_SIZE > 1):
    every rank calls this with the same arguments -- the whole grid and w0, as
    the reference -- and gets the whole snapshot matrix back.  Rank k marches
    its row slab on GPU `device` (default LOCAL_RANK) with the one-way halo
    streamed from rank k-1 during the launch, and writes
    its u rows and v rows straight into one shared .npy file of the whole
    matrix (BURG_SNAP_DIR or the temporary directory; burg_run_npy_ex), which
    every rank then maps copy-on-write (np.load(mmap_mode="c"): the values of
    the single-GPU run, bit for bit, writable, one copy in host memory for
    the whole node) before the file is unlinked.  The march solver only;
    stream_w / tiles_target: the slabs' pipe tiling (default: planned)."""
    d, rank, world = job()
    if world > 1:
        return _implicit2D_job(d, rank, world, grid_x, grid_y, w0, dt, num_steps, mu,
                               solver=solver, snap_every=snap_every, device=device,
                               engine=engine, verbose=verbose, allow_nonsquare=allow_nonsquare,
                               return_stats=return_stats, out=out, stream_w=stream_w,
                               tiles_target=tiles_target)
    if verbose:
        print("Running HDM for mu1={}".format(mu[0]))
    ctx = _ctx_for(grid_x, grid_y, dt, mu, device, allow_nonsquare, tile_w=tile_w,
                   par_passes=par_passes, tol=tol, engine=engine, stream_w=stream_w,
                   tiles_target=tiles_target)
    snaps, stats, its, rel = ctx.run(np.asarray(w0, dtype=np.float64).ravel(), int(num_steps),
                                     solver, newton_max_its, newton_rtol, int(snap_every),
                                     out=out)
    if verbose:
        lines = []
        for i in range(int(num_steps)):
            lines.append(" ... Working on timestep {}".format(i))
            if solver == "newton":
                lines.append("{}: {:3.2e}".format(its[i], rel[i]))
        if lines:
            print("\n".join(lines))
    if return_stats:
        stats = dict(stats, step_iters=its, step_rel=rel)
        return snaps, stats
    return snaps


def _job_ctx(d, rank, world, grid_x, grid_y, dt, mu, device, engine, allow_nonsquare, stream_w,
             tiles_target):
    nx, ny = np.asarray(grid_x).size - 1, np.asarray(grid_y).size - 1
    if engine != "pipe":
        raise ValueError("multi-GPU slabs run on the pipe engine")
    ctx = job_context(nx, ny, job_device(device), d, rank, world, engine="pipe",
                      stream_w=int(stream_w), tiles_target=int(tiles_target))
    ctx.set_problem(grid_x, grid_y, dt, mu, allow_nonsquare)
    return ctx


def _job_check(solver, out):
    if solver != "march":
        raise ValueError("multi-GPU slabs run the march solver (solver='march')")
    if out is not None:
        raise ValueError("out= is not supported on a multi-GPU job (every rank gets the "
                         "whole matrix as a copy-on-write map)")


def _implicit2D_job(d, rank, world, grid_x, grid_y, w0, dt, num_steps, mu, *, solver,
                    snap_every, device, engine, verbose, allow_nonsquare, return_stats, out,
                    stream_w, tiles_target):
    """inviscid_burgers_implicit2D on a multi-GPU job (its docstring)."""
    _job_check(solver, out)
    if verbose and rank == 0:
        print("Running HDM for mu1={}".format(mu[0]))
    ctx = _job_ctx(d, rank, world, grid_x, grid_y, dt, mu, device, engine, allow_nonsquare,
                   stream_w, tiles_target)
    path = shared_tmp_path(d, rank)
    st = slabs_to_npy(ctx, np.asarray(w0, dtype=np.float64).ravel(), int(num_steps), path,
                      int(snap_every), d, rank, world)
    snaps, err = None, None
    try:
        snaps = np.load(path, mmap_mode="c")
    except Exception as e:  # noqa: BLE001  (agreed on below: no rank waits for one that failed)
        err = e
    bad = agree(d, err)  # every rank holds its map (or all raise): the name can go
    if rank == 0:
        os.remove(path)
    if bad:
        raise RuntimeError(f"multi-GPU snapshot matrix {path}: {bad}")
    if verbose and rank == 0:
        print("\n".join(" ... Working on timestep {}".format(i) for i in range(int(num_steps))))
    if return_stats:
        its = np.ones(int(num_steps), dtype=np.int32)
        return snaps, dict(st, step_iters=its, step_rel=np.zeros(int(num_steps)), rank=rank,
                           world=world)
    return snaps


def inviscid_burgers_implicit2D_sweep(grid_x, grid_y, w0, dt, num_steps, mus, *, snap_every=1,
                                      device=0, verbose=1, allow_nonsquare=False,
                                      return_stats=False, outs=None, on_device=False):
    """inviscid_burgers_implicit2D (C/hypernet2D.py:72-131) for a LIST of mu at
    once -- what the reference's drivers do one call at a time when they fill
    a snapshot set (C/run_prom.py:59-71 over the 9 get_snapshot_params,
    C/run_tests.py:38-49 over 3 test mu).  All trajectories start from w0 and
    run in one pipelined launch per group on the GPU (burg_sweep): back to
    back in time, or -- grids that leave most of the chip idle, such as the
    reference's own 250^2 -- side by side as separate domains; each is
    bit-identical to inviscid_burgers_implicit2D(..., mu) with the march
    solver.  Returns a list of snapshot matrices, one per mu; on_device=True
    returns ONE float64 CUDA tensor, the np.hstack of those matrices
    (C/run_prom.py:59-71's snapshot set) left in HBM (burg_sweep_device), which
    POD(...) factorises in place."""
    mus = [tuple(mu) for mu in mus]
    if verbose:
        for mu in mus:
            print("Running HDM for mu1={}".format(mu[0]))
    ctx = _ctx_for(grid_x, grid_y, dt, mus[0], device, allow_nonsquare, engine="pipe")
    if on_device:
        S, stats = ctx.sweep_device(mus, int(num_steps), w0=np.asarray(w0, dtype=np.float64).ravel(),
                                    snap_every=int(snap_every))
        return (S, stats) if return_stats else S
    snaps, stats = ctx.sweep(mus, int(num_steps), w0=np.asarray(w0, dtype=np.float64).ravel(),
                             snap_every=int(snap_every), outs=outs)
    if return_stats:
        return snaps, stats
    return snaps


def inviscid_burgers_res2D_alt(w, grid_x, grid_y, dt, wp, mu, JDxec=None, JDyec=None, *,
                               device=0):
    """FOM residual R(w; wp, mu) (C/hypernet2D.py:2512-2570), computed on the GPU.
    JDxec/JDyec are accepted for signature compatibility and ignored."""
    ctx = _ctx_for(grid_x, grid_y, dt, mu, device)
    r, _ = ctx.residual(w, wp)
    return r


def inviscid_burgers_res2D(w, grid_x, grid_y, dt, wp, mu, Dxec=None, Dyec=None, *, device=0):
    """The same residual through the reference's 1-D operators
    (C/hypernet2D.py:2468-2510), the callback the ECSW / LSPG drivers pass
    around (C/run_HPROM_ecsw_joshua_.py:19-21,83).  Computed on the GPU by the
    res2D_alt stencil: the two reference forms differ only in the order of
    the per-cell sums (<= 4.4e-16 relative).
    Dxec/Dyec are accepted for signature compatibility and ignored."""
    return inviscid_burgers_res2D_alt(w, grid_x, grid_y, dt, wp, mu, device=device)


class JacobianOperator(LinearOperator):
    """J(w) of inviscid_burgers_exact_jac2D (C/hypernet2D.py:2627-2656) as a
    matrix-free operator: ``J @ x`` runs the HIP Jacobian-vector kernel and
    ``J.solve(b)`` the exact block forward substitution (what spsolve(J, b)
    computes at :1854)."""

    def __init__(self, ctx, w):
        self._ctx = ctx
        self._w = np.ascontiguousarray(np.asarray(w, dtype=np.float64).ravel())
        super().__init__(dtype=np.float64, shape=(ctx.m, ctx.m))

    def _matvec(self, x):
        return self._ctx.jvp(self._w, np.asarray(x, dtype=np.float64).ravel())

    def solve(self, b):
        return self._ctx.block_solve(self._w, np.asarray(b, dtype=np.float64).ravel())


def _grid_from_ops(JDxec, JDyec, n):
    nx = int(round(np.sqrt(n)))
    if nx * nx != n:
        raise ValueError("pass grid_x/grid_y for a non-square grid")
    inv_dx = np.asarray(JDxec.diagonal()[:nx], dtype=np.float64)
    inv_dy = np.asarray(JDyec.diagonal()[::nx][:nx], dtype=np.float64)
    gx = np.concatenate(([0.0], np.cumsum(1.0 / inv_dx)))
    gy = np.concatenate(([0.0], np.cumsum(1.0 / inv_dy)))
    return gx, gy


def inviscid_burgers_exact_jac2D(w, dt, JDxec=None, JDyec=None, Eye=None, *, grid_x=None,
                                 grid_y=None, device=0):
    """Exact FOM Jacobian at w (C/hypernet2D.py:2627-2656) as a JacobianOperator.
    The grid comes from grid_x/grid_y, or is recovered from JDxec/JDyec."""
    w = np.asarray(w, dtype=np.float64).ravel()
    if grid_x is None or grid_y is None:
        grid_x, grid_y = _grid_from_ops(JDxec, JDyec, w.size // 2)
    # the Jacobian does not depend on mu or the source: any mu is fine here
    ctx = _ctx_for(grid_x, grid_y, dt, (1.0, 0.0), device)
    return JacobianOperator(ctx, w)


def newton_raphson(func, jac, x0, max_its=20, relnorm_cutoff=1e-12):
    """newton_raphson (C/hypernet2D.py:1811-1857) with the reference's control
    flow and print line.  The linear solve uses J.solve(f) when J is a
    JacobianOperator (HIP exact block solve), else scipy's spsolve as the
    reference does."""
    x = np.array(x0, dtype=np.float64, copy=True)
    init_norm = np.linalg.norm(func(x0))
    resnorms = []
    for i in range(max_its):
        resnorm = np.linalg.norm(func(x))
        resnorms.append(resnorm)
        if resnorm / init_norm < relnorm_cutoff:
            print("{}: {:3.2e}".format(i, resnorm / init_norm))
            break
        J = jac(x)
        f = func(x)
        if hasattr(J, "solve"):
            x -= J.solve(f)
        else:
            x -= sp.linalg.spsolve(J, f)
    return x, resnorms


def compute_ECSW_training_matrix_2D(snaps, prev_snaps, basis, res=None, jac=None, grid_x=None,
                                    grid_y=None, dt=None, mu=None, *, device=0):
    """ECSW hyper-reduction training matrix (C/hypernet2D.py:2719-2740), same
    signature and (n_pod*n_snaps, n_hdm) result, assembled on the GPU in one
    kernel per snapshot (residual + J(snap) @ basis + the per-node products).
    `res` / `jac` are accepted for call compatibility: the reference passes
    inviscid_burgers_res2D and inviscid_burgers_exact_jac2D, which the kernel
    computes (the residual in res2D_alt's op order, equal to res2D's to
    round-off)."""
    if grid_x is None or grid_y is None or dt is None or mu is None:
        raise ValueError("grid_x, grid_y, dt and mu are required")
    ctx = _ctx_for(grid_x, grid_y, dt, mu, device)
    return ctx.ecsw_matrix(snaps, prev_snaps, basis)


def inviscid_burgers_implicit2D_LSPG(grid_x, grid_y, w0, dt, num_steps, mu, basis, *, device=0,
                                     max_its=20, relnorm_cutoff=1e-5, min_delta=0.1,
                                     verbose=True, return_coords=False):
    """LSPG PROM time loop (C/hypernet2D.py:133-200) with its Gauss-Newton
    solver (gauss_newton_LSPG, :1859-1929; max_its / relnorm_cutoff /
    min_delta are its defaults), on the GPU (burg_lspg).  Same call and
    result: (snaps (2n, T+1), (num_its, jac_time, res_time, ls_time)), snaps
    column j = basis @ y_j.  The LSPG Jacobian keeps the reference's row-only
    JDyec permutation (:165-167; its y-derivative reads the transposed field,
    lspg.hip), so nx == ny is required, as in the reference.  Each
    Gauss-Newton update solves the least-squares problem by the normal
    equations of J.basis (Cholesky) where the reference calls
    np.linalg.lstsq; the two agree to round-off for a full-rank J.basis.
    jac_time is the fused J.basis + Gram kernel, res_time the residual
    kernel, ls_time the solve and the basis expansion (seconds, HIP events).
    return_coords=True appends the reduced coordinates (npod, T+1)."""
    if verbose:
        print(f"Running ROM of size {np.shape(basis)[1]} for mu1={mu[0]}, mu2={mu[1]}")
    ctx = _ctx_for(grid_x, grid_y, dt, mu, device)
    snaps, red, its, rel, times, _ = ctx.lspg(w0, num_steps, basis, max_its=max_its,
                                             relnorm_cutoff=relnorm_cutoff, min_delta=min_delta)
    if verbose:
        for i in range(int(num_steps)):
            print(f" ... Working on timestep {i}")
            print("iteration {}: relative norm {:3.2e}".format(int(its[i]) - 1, rel[i]))
    out = (snaps, (int(its.sum()), times[0] / 1e3, times[1] / 1e3, times[2] / 1e3))
    return out + (red,) if return_coords else out


def POD(snaps, num_modes=None, method="svd", random_state=None, *, device=0, return_ms=False):
    """POD of a snapshot matrix (C/hypernet2D.py:2670-2695) on the GPU.
    Returns (u, s) as the reference:
      method 'svd'  -> all min(m, ns) modes of the exact thin SVD
                       (np.linalg.svd(snaps, full_matrices=False); num_modes
                       unused, as there): burg_pod, rocSOLVER Householder QR of
                       the tall matrix + SVD of R (backward stable like LAPACK);
      method 'rsvd' -> num_modes modes (default all) by sklearn's
                       randomized_svd algorithm (10 oversamples, n_iter 7 if
                       num_modes < 0.1 min(m, ns) else 4, Gaussian test matrix
                       drawn from check_random_state(random_state) exactly as
                       sklearn draws it): burg_pod_rsvd, the products with S
                       on fp64 MFMA kernels, CholeskyQR3 and a Jacobi small
                       SVD on the device.  The power iterations are
                       normalised by QR (sklearn's 'auto' uses LU: same
                       subspace).
    Column signs follow sklearn's svd_flip rule on u (largest-magnitude entry
    positive); np.linalg.svd's are arbitrary."""
    if method not in ("svd", "rsvd"):
        raise ValueError("Unknown method '{}' for POD. Use 'svd' or 'rsvd'.".format(method))
    from . import _lib
    on_dev = type(snaps).__module__.startswith("torch")
    if on_dev:
        # a device-resident snapshot matrix (e.g. inviscid_burgers_implicit2D_sweep(...,
        # on_device=True)): factorised in place, no host round trip
        import torch
        if (snaps.dtype != torch.float64 or snaps.dim() != 2 or not snaps.is_contiguous()
                or snaps.device.type != "cuda"):
            raise ValueError("a device snapshot matrix must be a contiguous 2-D float64 CUDA tensor")
        device = snaps.device.index if snaps.device.index is not None else 0
        torch.cuda.synchronize(snaps.device)
        S = snaps
    else:
        S = np.ascontiguousarray(np.asarray(snaps, dtype=np.float64))
        if S.ndim != 2:
            raise ValueError("snaps must be a 2-D (dofs, snapshots) matrix")
    m, ns = S.shape
    if m < ns:
        raise ValueError("POD on the GPU needs at least as many rows as snapshots")
    k = min(m, ns) if (method == "svd" or num_modes is None) else int(num_modes)
    u = np.zeros((m, k))
    sv = np.zeros(k)
    ms = ctypes.c_double(0.0)
    L = _lib.load()
    if method == "svd":
        if on_dev:
            _lib.check(L.burg_pod_rsvd_device(int(device), m, ns, S.data_ptr(), k, 0, 0, None,
                                              _lib.dptr(u), _lib.dptr(sv), ctypes.byref(ms)))
        else:
            _lib.check(L.burg_pod(int(device), m, ns, _lib.dptr(S), k, _lib.dptr(u), _lib.dptr(sv),
                                  ctypes.byref(ms)))
    else:
        if random_state is None:
            rng = np.random.mtrand._rand
        elif isinstance(random_state, (int, np.integer)):
            rng = np.random.RandomState(random_state)
        else:
            rng = random_state
        # sklearn draws the full (ns, k + 10) Gaussian test matrix whatever k
        # is; draw exactly that, so later draws from the same RNG match the
        # reference run, and keep at most ns columns (they already span the
        # whole column space of S)
        n_iter = 7 if k < 0.1 * min(m, ns) else 4
        omega = rng.normal(size=(ns, k + 10))
        nrand = min(k + 10, ns)
        omega_cm = np.ascontiguousarray(omega[:, :nrand].T)  # column-major (ns x nrand)
        if on_dev:
            _lib.check(L.burg_pod_rsvd_device(int(device), m, ns, S.data_ptr(), k, nrand, n_iter,
                                              _lib.dptr(omega_cm), _lib.dptr(u), _lib.dptr(sv),
                                              ctypes.byref(ms)))
        else:
            _lib.check(L.burg_pod_rsvd(int(device), m, ns, _lib.dptr(S), k, nrand, n_iter,
                                       _lib.dptr(omega_cm), _lib.dptr(u), _lib.dptr(sv),
                                       ctypes.byref(ms)))
    return (u, sv, ms.value) if return_ms else (u, sv)


def compute_error(rom_snaps, hdm_snaps):
    """Relative error at each time step (C/hypernet2D.py:3074-3079)."""
    sq_hdm = np.sqrt(np.square(rom_snaps).sum(axis=0))
    sq_err = np.sqrt(np.square(rom_snaps - hdm_snaps).sum(axis=0))
    rel_err = sq_err / sq_hdm
    return rel_err, rel_err.mean()


def plot_snaps(grid_x, grid_y, snaps, snaps_to_plot, linewidth=2, color="black",
               linestyle="solid", label=None, fig_ax=None):
    """Mid-line slices of u for the snapshot columns in snaps_to_plot
    (C/hypernet2D.py:3147-3180, the figures the author pickled): axis 1 shows
    u along the middle row y = y[ny // 2], axis 2 along the middle column
    x = x[nx // 2]; only the first line of a call carries `label`.  Returns
    (fig, ax1, ax2); pass them back as fig_ax to overlay further calls."""
    import matplotlib.pyplot as plt
    if fig_ax is None:
        fig, (ax1, ax2) = plt.subplots(2, 1)
    else:
        fig, ax1, ax2 = fig_ax
    gx, gy = np.asarray(grid_x), np.asarray(grid_y)
    xc, yc = 0.5 * (gx[1:] + gx[:-1]), 0.5 * (gy[1:] + gy[:-1])
    jx, jy = xc.size // 2, yc.size // 2
    n = xc.size * yc.size
    for k, col in enumerate(snaps_to_plot):
        u = np.asarray(snaps[:n, col]).reshape(yc.size, xc.size)
        lab = label if k == 0 else None
        style = dict(color=color, linestyle=linestyle, linewidth=linewidth, label=lab)
        ax1.plot(xc, u[jy, :], **style)
        ax1.set_xlabel("$x$")
        ax1.set_ylabel("$u_x(x,y={:0.1f})$".format(yc[jy]))
        ax1.grid()
        ax2.plot(yc, u[:, jx], **style)
        ax2.set_xlabel("$y$")
        ax2.set_ylabel("$u_x(x={:0.1f},y)$".format(xc[jx]))
        ax2.grid()
    return fig, ax1, ax2


def param_to_snap_fn(mu, snap_folder="param_snaps", suffix=".npy"):
    """'param_snaps/mu1_{mu1}+mu2_{mu2}.npy' (C/hypernet2D.py:3081-3105)."""
    snapfn = snap_folder + "/"
    for i in range(len(mu)):
        if i > 0:
            snapfn += "+"
        snapfn += "mu{}_{}".format(i + 1, mu[i])
    return snapfn + suffix


def get_saved_params(snap_folder="param_snaps"):
    """Set of cached snapshot files (C/hypernet2D.py:3107-3109)."""
    return set(glob.glob(snap_folder + "/*"))


def _open_cache(fn, m, ncols):
    """A .npy file of shape (m, ncols) float64 C-order (np.save's format),
    memory-mapped for writing under a temporary name; _commit_cache renames it
    once complete, so an interrupted run never leaves a truncated cache file
    that get_saved_params would then trust."""
    tmp = fn + ".partial.npy"
    return tmp, np.lib.format.open_memmap(tmp, mode="w+", dtype=np.float64, shape=(m, ncols))


def _commit_cache(tmp, fn, mm):
    mm.flush()
    del mm
    os.replace(tmp, fn)


def load_or_compute_snaps(mu, grid_x, grid_y, w0, dt, num_steps, snap_folder="param_snaps",
                          stream=False, mmap=False, direct=False, recompute_short=False,
                          **solver_kw):
    """Load cached snapshots for mu, or compute and cache them
    (C/hypernet2D.py:3111-3145; same file names and .npy format, so caches
    are interchangeable with the reference's).  solver_kw go to
    inviscid_burgers_implicit2D.

    stream=False (default): the reference's flow -- the snapshot matrix in
    host memory (filled by pinned DMA from HBM), then np.save.  stream=True:
    the library writes the snapshots straight into a memory map of the cache
    file, so the host never holds the matrix twice (for trajectories that do
    not fit host memory twice); the returned array is an in-memory copy
    unless mmap=True (then the file's read-only memory map).  Measured at
    1024^2 x 101 columns (1.7 GB, tools/snapio_probe.py):
    0.29 s default vs 0.52 s streamed -- file-backed pages cannot be pinned,
    so the streamed D2H runs at pageable speed.
    mmap=True on a cache hit: np.load(..., mmap_mode='r') instead of reading
    the whole file.  direct=True (march solver): the library writes the cache
    file itself (burg_run_npy: the trajectory stays in HBM, row blocks of the
    C-order matrix go through two pinned buffers to a writer thread), then
    the file is loaded (mmap=True: mapped).

    A cache file with fewer columns than asked for is returned as it is,
    truncated to what it holds (the reference's np.load(fn)[:, :num_steps+1]);
    recompute_short=True recomputes it instead and overwrites the file.

    Multi-GPU (torchrun, WORLD_SIZE > 1; inviscid_burgers_implicit2D): every
    rank calls this with the same arguments.  Rank 0 decides hit or miss; on
    a miss the ranks march their slabs and write their rows straight into the
    cache file (under its .partial name, renamed by rank 0 once every rank has
    written -- the same bytes as the single-GPU direct=True file); either way
    every rank returns the cache file's matrix as a copy-on-write map
    (np.load(mmap_mode="c"), or "r" with mmap=True), so the node holds one
    copy.  The march solver only."""
    d, rank, world = job()
    if world > 1:
        return _load_or_compute_job(d, rank, world, mu, grid_x, grid_y, w0, dt, num_steps,
                                    snap_folder, mmap, recompute_short, solver_kw)
    if not os.path.exists(snap_folder):
        os.makedirs(snap_folder)
    every = int(solver_kw.get("snap_every", 1))
    ncols = int(num_steps) // every + 1
    # a thinned matrix (snap_every > 1) must never pass for the reference's
    # per-step cache: it gets a name of its own
    snap_fn = param_to_snap_fn(mu, snap_folder=snap_folder,
                               suffix=".npy" if every == 1 else f"+every{every}.npy")
    if snap_fn in get_saved_params(snap_folder=snap_folder):
        cached = np.load(snap_fn, mmap_mode="r")
        if cached.shape[1] >= ncols or not recompute_short:
            print(f"Loading saved snaps for mu1={mu[0]}, mu2={mu[1]}")
            return cached[:, :ncols] if mmap else np.array(cached[:, :ncols])
        print(f"Saved snaps for mu1={mu[0]}, mu2={mu[1]} hold {cached.shape[1]} of the "
              f"{ncols} columns asked for: recomputing")
        del cached
    print(f"Computing new snaps for mu1={mu[0]}, mu2={mu[1]}")
    t0 = time.time()
    if direct:
        if solver_kw.get("solver", "march") != "march":
            raise ValueError("direct=True writes march trajectories")
        device = solver_kw.get("device", 0)
        ctx = _ctx_for(grid_x, grid_y, dt, mu, device, solver_kw.get("allow_nonsquare", False),
                       engine=solver_kw.get("engine", "pipe"))
        tmp = snap_fn + ".partial.npy"
        try:
            ctx.run_to_npy(np.asarray(w0, dtype=np.float64).ravel(), int(num_steps), tmp,
                           snap_every=every)
        except Exception:
            if os.path.exists(tmp):  # never leave a partial cache behind
                os.remove(tmp)
            raise
        os.replace(tmp, snap_fn)
        print("Elapsed time: {:3.3e}".format(time.time() - t0))
        return np.load(snap_fn, mmap_mode="r" if mmap else None)
    if not stream:
        snaps = inviscid_burgers_implicit2D(grid_x, grid_y, w0, dt, num_steps, mu, **solver_kw)
        print("Elapsed time: {:3.3e}".format(time.time() - t0))
        np.save(snap_fn, snaps)
        return snaps
    m = np.asarray(w0).size
    tmp, mm = _open_cache(snap_fn, m, ncols)
    inviscid_burgers_implicit2D(grid_x, grid_y, w0, dt, num_steps, mu, out=mm, **solver_kw)
    print("Elapsed time: {:3.3e}".format(time.time() - t0))
    snaps = None if mmap else np.array(mm)
    _commit_cache(tmp, snap_fn, mm)
    return np.load(snap_fn, mmap_mode="r") if mmap else snaps


def _load_or_compute_job(d, rank, world, mu, grid_x, grid_y, w0, dt, num_steps, snap_folder,
                         mmap, recompute_short, solver_kw):
    """load_or_compute_snaps on a multi-GPU job (its docstring)."""
    kw = dict(solver_kw)
    every = int(kw.pop("snap_every", 1))
    _job_check(kw.pop("solver", "march"), kw.pop("out", None))
    ncols = int(num_steps) // every + 1
    snap_fn = param_to_snap_fn(mu, snap_folder=snap_folder,
                               suffix=".npy" if every == 1 else f"+every{every}.npy")
    box = [None]
    if rank == 0:
        os.makedirs(snap_folder, exist_ok=True)
        hit = False
        if snap_fn in get_saved_params(snap_folder=snap_folder):
            hit = np.load(snap_fn, mmap_mode="r").shape[1] >= ncols or not recompute_short
        box[0] = hit
    d.broadcast_object_list(box, src=0)
    mode = "r" if mmap else "c"
    if box[0]:
        if rank == 0:
            print(f"Loading saved snaps for mu1={mu[0]}, mu2={mu[1]}")
        return np.load(snap_fn, mmap_mode=mode)[:, :ncols]
    if rank == 0:
        print(f"Computing new snaps for mu1={mu[0]}, mu2={mu[1]}")
    t0 = time.time()
    ctx = _job_ctx(d, rank, world, grid_x, grid_y, dt, mu, kw.pop("device", None),
                   kw.pop("engine", "pipe"), kw.pop("allow_nonsquare", False),
                   kw.pop("stream_w", 0), kw.pop("tiles_target", 0))
    tmp = snap_fn + ".partial.npy"
    slabs_to_npy(ctx, np.asarray(w0, dtype=np.float64).ravel(), int(num_steps), tmp, every, d,
                 rank, world)
    d.barrier()
    if rank == 0:
        os.replace(tmp, snap_fn)
        print("Elapsed time: {:3.3e}".format(time.time() - t0))
    d.barrier()
    return np.load(snap_fn, mmap_mode=mode)


def load_or_compute_snaps_sweep(mus, grid_x, grid_y, w0, dt, num_steps,
                                snap_folder="param_snaps", stream=False, mmap=False):
    """load_or_compute_snaps (C/hypernet2D.py:3111-3145) for a list of mu: the
    cached ones are loaded, all missing ones are computed in ONE GPU sweep
    (inviscid_burgers_implicit2D_sweep) and cached under the reference's file
    names (streamed into the files' memory maps with stream=True, as in
    load_or_compute_snaps).  Returns the list of snapshot matrices in the
    order of `mus`."""
    if not os.path.exists(snap_folder):
        os.makedirs(snap_folder)
    saved = get_saved_params(snap_folder=snap_folder)
    out = [None] * len(mus)
    todo = []
    for i, mu in enumerate(mus):
        fn = param_to_snap_fn(mu, snap_folder=snap_folder)
        if fn in saved:
            print(f"Loading saved snaps for mu1={mu[0]}, mu2={mu[1]}")
            out[i] = np.load(fn, mmap_mode="r" if mmap else None)[:, :num_steps + 1]
        else:
            todo.append(i)
    if todo:
        for i in todo:
            print(f"Computing new snaps for mu1={mus[i][0]}, mu2={mus[i][1]}")
        t0 = time.time()
        fns = [param_to_snap_fn(mus[i], snap_folder=snap_folder) for i in todo]
        caches = [_open_cache(fn, np.asarray(w0).size, int(num_steps) + 1) for fn in fns] \
            if stream else None
        snaps = inviscid_burgers_implicit2D_sweep(grid_x, grid_y, w0, dt, num_steps,
                                                  [mus[i] for i in todo], verbose=0,
                                                  outs=[c[1] for c in caches] if stream else None)
        print("Elapsed time: {:3.3e}".format(time.time() - t0))
        for k, (i, sn) in enumerate(zip(todo, snaps)):
            if stream:
                tmp, mm = caches[k]
                keep = None if mmap else np.array(mm)
                del sn
                _commit_cache(tmp, fns[k], mm)
                out[i] = np.load(fns[k], mmap_mode="r") if mmap else keep
            else:
                np.save(fns[k], sn)
                out[i] = sn
    return out
