"""ECSW training matrices of the manifold (decoder) ROMs on the GPU
(paths relative to /root/reference,
C/ = BurgersFD_CleanCoarse/):

  compute_ECSW_training_matrix_2D_rnm                    C/hypernet2D.py:2742-2783
  compute_ECSW_training_matrix_2D_rbf_nearest_neighbors  C/hypernet2D.py:2785-2860
  compute_ECSW_training_matrix_2D_rbf_global             C/hypernet2D.py:2862-2958
  compute_ECSW_training_matrix_2D_gp                     C/hypernet2D.py:2960-3072

Each snapshot i: start from y0 = U_p^T snap, refit the reconstruction
w(y) to the snapshot by Gauss-Newton on ||w(y) - snap|| (stop when it falls
below 1e-2 of its initial value, or after 10 updates), then assemble the
snapshot's n_pod rows of C from the HDM residual R(w; prev) and J(w) V with
V = dw/dy at the final y:
  C[i*n_pod + k, node] = R_u[node] (J V)_u[node, k] + R_v[node] (J V)_v[node, k].

The reference builds J as a CSR matrix, multiplies it into V and fills C in
a Python loop over every node; here the block is one HIP kernel
(burg_ecsw_block_device, ecsw.hip) on device-resident w, prev and V^T.  For
the POD-RBF / POD-GP variants the large products of the refit -- w = U_p y +
U_s q(y), V^T = U_p^T + (dq/dy)^T U_s^T and the Gauss-Newton normal
equations V^T V, V^T (w - snap) (one split-K Gram) -- run on the device too
(rocBLAS through torch), with U_p and U_s resident; only the small latent maps q, dq/dy
(rom_decoders.py) and the r_p x r_p least-squares solve stay on the host, as
np.linalg.lstsq, as in the reference.  The NN-decoder variant (rnm) keeps
the caller's torch functions exactly as the reference calls them (float32),
and only its C block runs here.

Extensions (keyword-only): device, verbose (the reference's per-snapshot
residual prints), return_coords (also return the refit reduced coordinates,
(n_pod, n_snaps)).

Precision: the reference evaluates the rnm variant's residual and Jacobian on
the decoder's float32 output (numpy keeps the float32 fluxes); the kernel
evaluates them in float64 on the same float32 values (tests/test_gpu_parity.py
states the tolerance).
"""
import numpy as np


def _device_ctx(grid_x, grid_y, dt, mu, device):
    from .hypernet2D import _ctx_for
    return _ctx_for(grid_x, grid_y, dt, mu, device)


def _check_shapes(snaps, prev_snaps, basis, m):
    snaps = np.asarray(snaps, dtype=np.float64)
    prev_snaps = np.asarray(prev_snaps, dtype=np.float64)
    if snaps.ndim != 2 or snaps.shape[0] != m or prev_snaps.shape != snaps.shape:
        raise ValueError("snaps / prev_snaps must be (2*nx*ny, n_snaps) and equal in shape")
    basis = np.asarray(basis, dtype=np.float64)
    if basis.ndim != 2 or basis.shape[0] != m:
        raise ValueError("basis must be (2*nx*ny, n_pod)")
    return snaps, prev_snaps, basis


class _Blocks:
    """Device buffers of one variant run and the C assembly."""

    def __init__(self, ctx, n_pod, n_snaps):
        import torch
        self.torch, self.ctx = torch, ctx
        self.dev = torch.device("cuda", ctx.device)
        self.n = ctx.m // 2
        self.n_pod = n_pod
        self.C = np.zeros((n_pod * n_snaps, self.n))
        self.coords = np.zeros((n_pod, n_snaps))
        self.cblk = torch.empty((n_pod, self.n), dtype=torch.float64, device=self.dev)
        self.kernel_ms = 0.0

    def vec(self, x):
        return self.torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device=self.dev)

    def assemble(self, isnap, y, w, prev, Vt):
        """C rows of snapshot isnap from device w, prev (2n,) and V^T (n_pod, 2n);
        y: the refit reduced coordinates."""
        self.coords[:, isnap] = np.asarray(y, dtype=np.float64).ravel()
        self.kernel_ms += self.ctx.ecsw_block_device(w, prev, Vt.contiguous(), self.cblk)
        self.C[isnap * self.n_pod:(isnap + 1) * self.n_pod] = self.cblk.cpu().numpy()


def _gram(M, parts=256):
    """M M^T of a short, very wide device matrix (r x 2n) as a split-K
    batched product: one dgemm with k = 2n runs on a handful of workgroups
    (~18 ms at 250^2); `parts` slices of k in one bmm fill the chip."""
    import torch
    r, K = M.shape
    kc = -(-K // parts)
    if kc * parts != K:
        M = torch.nn.functional.pad(M, (0, kc * parts - K))
    Mb = M.reshape(r, parts, kc).transpose(0, 1)
    return torch.bmm(Mb, Mb.transpose(1, 2)).sum(0)


def _refit_pod_manifold(snaps, prev_snaps, basis, basis2, qmap, grid_x, grid_y, dt, mu, device,
                        max_its, tol, messages, verbose, return_coords):
    """The POD-RBF / POD-GP variants: w(y) = U_p y + U_s q(y)."""
    import torch
    ctx = _device_ctx(grid_x, grid_y, dt, mu, device)
    snaps, prev_snaps, basis = _check_shapes(snaps, prev_snaps, basis, ctx.m)
    basis2 = np.asarray(basis2, dtype=np.float64)
    if basis2.ndim != 2 or basis2.shape[0] != ctx.m:
        raise ValueError("basis2 must be (2*nx*ny, n_secondary)")
    n_pod, ns = basis.shape[1], snaps.shape[1]
    out = _Blocks(ctx, n_pod, ns)
    Upt = out.vec(basis.T)    # (r_p, 2n), resident for the whole run
    Ust = out.vec(basis2.T)   # (r_s, 2n)
    first, last = messages

    def decode(y):
        return Upt.T @ out.vec(y) + Ust.T @ out.vec(qmap.q(y))

    def jac_t(y):  # V(y)^T
        return Upt + out.vec(qmap.dq(y)).T @ Ust

    for isnap in range(ns):
        snap = out.vec(snaps[:, isnap])
        prev = out.vec(prev_snaps[:, isnap])
        y = (Upt @ snap).cpu().numpy()
        snap_norm = torch.linalg.vector_norm(snap).item()
        w = decode(y)
        init_res = torch.linalg.vector_norm(w - snap).item()
        approx_res, num_it = init_res, 0
        if verbose:
            print(first.format(init_res / snap_norm))
        with np.errstate(divide="ignore", invalid="ignore"):
            while abs(np.float64(approx_res) / init_res) > tol and num_it < max_its:
                # (the reference decodes y again here; w already is w(y))
                # V^T V and V^T (w - snap) from one Gram of [V^T; (w - snap)^T]
                G = _gram(torch.cat([jac_t(y), (w - snap)[None, :]])).cpu().numpy()
                JJ, Jr = G[:n_pod, :n_pod], G[:n_pod, n_pod]
                dy = np.linalg.lstsq(JJ, Jr, rcond=None)[0]
                y = y - dy
                w = decode(y)
                approx_res = torch.linalg.vector_norm(w - snap).item()
                num_it += 1
        if verbose:
            print(last.format(torch.linalg.vector_norm(w - snap).item() / snap_norm))
        out.assemble(isnap, y, w, prev, jac_t(y))
    return (out.C, out.coords) if return_coords else out.C


def compute_ECSW_training_matrix_2D_rbf_nearest_neighbors(
        snaps, prev_snaps, basis, basis2, epsilon, neighbors, kdtree, q_p_train, q_s_train, res,
        jac, grid_x, grid_y, dt, mu, scaler, kernel_type="gaussian", *, device=0, verbose=True,
        return_coords=False):
    """C/hypernet2D.py:2785-2860 (POD-RBF, dynamic nearest-neighbour
    interpolant).  Same signature and (n_pod*n_snaps, n_hdm) result; res / jac
    are accepted for call compatibility (the kernel computes res2D and
    exact_jac2D)."""
    from .rom_decoders import RBFNearestNeighborsMap
    qmap = RBFNearestNeighborsMap(kdtree, q_p_train, q_s_train, epsilon, neighbors, scaler,
                                  kernel_type)
    return _refit_pod_manifold(snaps, prev_snaps, basis, basis2, qmap, grid_x, grid_y, dt, mu,
                               device, 10, 1e-2,
                               ("Initial residual: {:3.2e}", "Final residual: {:3.2e}"), verbose,
                               return_coords)


def compute_ECSW_training_matrix_2D_rbf_global(
        snaps, prev_snaps, basis, basis2, W_global, q_p_train, q_s_train, res, jac, grid_x,
        grid_y, dt, mu, scaler, epsilon, kernel_type="gaussian", *, device=0, verbose=True,
        return_coords=False):
    """C/hypernet2D.py:2862-2958 (POD-RBF, global interpolant with weights
    W_global)."""
    from .rom_decoders import RBFGlobalMap
    qmap = RBFGlobalMap(W_global, q_p_train, epsilon, scaler, kernel_type)
    return _refit_pod_manifold(snaps, prev_snaps, basis, basis2, qmap, grid_x, grid_y, dt, mu,
                               device, 10, 1e-2,
                               ("Initial residual: {:.2e}", "Final residual: {:.2e}"), verbose,
                               return_coords)


def compute_ECSW_training_matrix_2D_gp(snaps, prev_snaps, basis, basis2, gp_model, res, jac,
                                       grid_x, grid_y, dt, mu, scaler, max_local_its=10,
                                       local_tol=1e-2, *, device=0, verbose=True,
                                       return_coords=False):
    """C/hypernet2D.py:2960-3072 (POD-GP, ConstantKernel * Matern(1.5) GP
    from primary to secondary coordinates)."""
    from .rom_decoders import GPMap
    return _refit_pod_manifold(snaps, prev_snaps, basis, basis2, GPMap(gp_model, scaler),
                               grid_x, grid_y, dt, mu, device, max_local_its, local_tol,
                               ("Initial reconstruction residual: {:.2e}",
                                "Final reconstruction residual: {:.2e}"), verbose,
                               return_coords)


def compute_ECSW_training_matrix_2D_rnm(snaps, prev_snaps, basis, approx, jacfwdfunc, res, jac,
                                        grid_x, grid_y, dt, mu, *, device=0, verbose=True,
                                        return_coords=False):
    """C/hypernet2D.py:2742-2783 (NN manifold decoder).  approx(y) and
    jacfwdfunc(y) are the caller's torch functions of float32 reduced
    coordinates, called exactly as the reference calls them (the refit is
    the reference's float32 Gauss-Newton); the C block of each snapshot runs
    in the kernel on the decoded state and Jacobian, cast to float64."""
    import torch
    ctx = _device_ctx(grid_x, grid_y, dt, mu, device)
    snaps, prev_snaps, basis = _check_shapes(snaps, prev_snaps, basis, ctx.m)
    n_pod, ns = basis.shape[1], snaps.shape[1]
    out = _Blocks(ctx, n_pod, ns)

    def host(t):
        return t.squeeze().detach().cpu().numpy()

    for isnap in range(ns):
        snap = snaps[:, isnap]
        y0 = torch.tensor(basis.T @ snap, dtype=torch.float)
        init_res = np.linalg.norm(host(approx(y0)) - snap)
        approx_res, num_it = init_res, 0
        y = y0.detach()
        if verbose:
            print("Initial residual: {:3.2e}".format(init_res / np.linalg.norm(snap)))
        while abs(approx_res / init_res) > 1e-2 and num_it < 10:
            Jf = jacfwdfunc(y)
            JJ = Jf.T @ Jf
            Jr = Jf.T @ (approx(y) - torch.tensor(snap, dtype=torch.float))
            dy = np.linalg.lstsq(host(JJ), host(Jr), rcond=None)[0]
            y -= dy
            approx_res = np.linalg.norm(host(approx(y)) - snap)
            num_it += 1
        w = host(approx(y))
        if verbose:
            print("Final residual: {:3.2e}".format(np.linalg.norm(w - snap) / np.linalg.norm(snap)))
        V = host(jacfwdfunc(y))
        if V.shape != (ctx.m, n_pod):
            raise ValueError(f"jacfwdfunc(y) gives {V.shape}, expected {(ctx.m, n_pod)}")
        out.assemble(isnap, y.detach().cpu().numpy(), out.vec(w), out.vec(prev_snaps[:, isnap]),
                     out.vec(V.T))
    return (out.C, out.coords) if return_coords else out.C
