"""Secondary-mode closures of the POD-RBF and POD-GP manifold ROMs: the
reconstruction w(y) = U_p y + U_s q(y) and its Jacobian V(y) = U_p + U_s dq/dy
that the ECSW decoder variants refit per snapshot (ecsw.py).

Host-side model code, as in the reference (paths relative to /root/reference,
C/ = BurgersFD_CleanCoarse/): the maps q(y) are small (r_p -> r_s, evaluated
on a handful of training points), the products with U_p and U_s are the
large part, and the ECSW driver runs those on the GPU.  The drop-in functions
below keep the reference's names and signatures and compute everything in
numpy, for callers that use them directly:

  decode_rbf_nearest_neighbors  C/hypernet2D.py:1279-1314
  jac_rbf_nearest_neighbors     C/hypernet2D.py:1316-1350
  decode_rbf_global             C/hypernet2D.py:1352-1394
  jac_rbf_global                C/hypernet2D.py:1397-1445
  decode_gp                     C/hypernet2D.py:1447-1495
  matern15_grad / jac_gp        C/hypernet2D.py:1720-1808

The kernel formulas follow C/rbf_utils.py (RBFUtils), restated as one table
per kernel instead of one function per kernel and method:
  phi(r)       the radial function (rbf_utils.py:10-33)
  nn_weight    g(r) with dq/dx_norm = W^T (g(r) * (x_norm - p)) in the
               nearest-neighbour Jacobians (rbf_utils.py:36-378).  Two of them
               are not the derivative of phi and are kept as the reference
               has them (the Jacobian feeds parity): imq uses
               -eps^2 phi(r) (1+(eps r)^2)^(-3/2) (:121-200; the derivative has
               no phi factor) and multiquadric eps^2 phi(r)/sqrt(1+(eps r)^2)
               = eps^2 (:292-378; the derivative is eps^2/phi(r)).
  glob_weight  the same for the global Jacobians (rbf_utils.py:675-1270);
               linear is zero where r <= 1e-12 (:1090-1144).
'matern' exists only for the global method; the nearest-neighbour method
raises ValueError for it, as the reference does.
"""
import numpy as np
from scipy.spatial.distance import pdist, squareform

_SQRT3 = np.sqrt(3)


def _phi_gaussian(r, eps):
    return np.exp(-(eps * r) ** 2)


def _phi_imq(r, eps):
    return 1.0 / np.sqrt(1 + (eps * r) ** 2)


def _phi_linear(r, eps):
    return r


def _phi_mq(r, eps):
    return np.sqrt(1 + (eps * r) ** 2)


def _phi_matern(r, eps):
    return (1.0 + _SQRT3 * eps * r) * np.exp(-_SQRT3 * eps * r)


def _inv_or_zero(r, floor):
    out = np.zeros_like(r)
    nz = r > floor
    out[nz] = 1.0 / r[nz]
    return out


# kernel -> (phi, nn_weight(r, eps, phi_r) or None, glob_weight(r, eps, phi_r))
KERNELS = {
    "gaussian": (_phi_gaussian,
                 lambda r, e, p: -2 * e ** 2 * p,
                 lambda r, e, p: -2 * e ** 2 * p),
    "imq": (_phi_imq,
            lambda r, e, p: -e ** 2 * p * (1 + (e * r) ** 2) ** (-3 / 2),
            lambda r, e, p: -e ** 2 * p ** 3),
    "linear": (_phi_linear,
               lambda r, e, p: _inv_or_zero(r, 0.0),
               lambda r, e, p: _inv_or_zero(r, 1e-12)),
    "multiquadric": (_phi_mq,
                     lambda r, e, p: p * (e ** 2 / np.sqrt(1 + (e * r) ** 2)),
                     lambda r, e, p: e ** 2 / p),
    "matern": (_phi_matern,
               None,
               lambda r, e, p: -3.0 * e ** 2 * (p / (1.0 + _SQRT3 * e * r))),
}


def _kernel(kernel_type, method):
    spec = KERNELS.get(kernel_type)
    if spec is None or (method == "nn" and spec[1] is None):
        raise ValueError(f"Unsupported kernel type: {kernel_type}")
    return spec


class RBFNearestNeighborsMap:
    """q(y) and dq/dy of the dynamic nearest-neighbour RBF interpolant
    (rbf_utils.py:36-378, 381-672): the `neighbors` training points nearest
    to scaler.transform(y) in the KD-tree (q_p_train is the normalised
    training set the tree was built on), local weights from the regularised
    kernel matrix (+1e-8 I), dq/dy chained through the scaler's scale_."""

    def __init__(self, kdtree, q_p_train, q_s_train, epsilon, neighbors, scaler,
                 kernel_type="gaussian"):
        self.phi, self.weight, _ = _kernel(kernel_type, "nn")
        self.kdtree, self.P, self.Q = kdtree, q_p_train, q_s_train
        self.eps, self.k, self.scaler = epsilon, neighbors, scaler

    def _local(self, y):
        xs = self.scaler.transform(np.asarray(y).reshape(1, -1))
        dist, idx = self.kdtree.query(xs, k=self.k)
        P = self.P[idx].reshape(self.k, -1)
        Wn = np.linalg.solve(self.phi(squareform(pdist(P)), self.eps) + np.eye(self.k) * 1e-08,
                             self.Q[idx].reshape(self.k, -1))
        return xs, P, Wn, dist.flatten()

    def q(self, y):
        _, _, Wn, r = self._local(y)
        return self.phi(r, self.eps) @ Wn

    def dq(self, y):
        xs, P, Wn, r = self._local(y)
        g = self.weight(r, self.eps, self.phi(r, self.eps))
        return (Wn.T @ (g[:, None] * (xs.reshape(1, -1) - P))) * self.scaler.scale_[None, :]


class RBFGlobalMap:
    """q(y) and dq/dy of the global RBF interpolant with precomputed weights
    W_global over the normalised training set (rbf_utils.py:675-1270,
    1272-1660)."""

    def __init__(self, W_global, q_p_train, epsilon, scaler, kernel_type="gaussian"):
        self.phi, _, self.weight = _kernel(kernel_type, "global")
        self.W, self.P, self.eps, self.scaler = W_global, q_p_train, epsilon, scaler

    def _dist(self, y):
        xs = self.scaler.transform(np.asarray(y).reshape(1, -1))
        return xs, np.linalg.norm(self.P - xs, axis=1)

    def q(self, y):
        _, r = self._dist(y)
        return self.phi(r, self.eps) @ self.W

    def dq(self, y):
        xs, r = self._dist(y)
        g = self.weight(r, self.eps, self.phi(r, self.eps))
        return (self.W.T @ (g[:, None] * (xs - self.P))) * self.scaler.scale_[None, :]


def matern15_grad(x_scaled, X_train, length_scale, cval):
    """Gradient of c * Matern(nu=1.5, l) at x_scaled w.r.t. x_scaled, one row
    per training point, zero at coincident points (C/hypernet2D.py:1720-1752)."""
    diff = x_scaled[None, :] - X_train
    d = np.linalg.norm(diff, axis=1)
    grad = np.zeros_like(diff)
    keep = d > 1e-14
    e = np.exp(-np.sqrt(3.0) * (d / length_scale))
    grad[keep] = (-3.0 * cval / (length_scale ** 2)) * e[keep, None] * diff[keep]
    return grad


class GPMap:
    """q(y) and dq/dy of a fitted multi-output GaussianProcessRegressor with a
    ConstantKernel * Matern(nu=1.5) kernel (decode_gp / jac_gp,
    C/hypernet2D.py:1447-1495, 1754-1808): q = k(X_train, x_scaled) @ alpha_
    (the reference's custom predict; gp_model.predict with
    use_custom_predict=False), dq/dy = alpha_^T grad_k * scale_."""

    def __init__(self, gp_model, scaler, use_custom_predict=True):
        self.gp, self.scaler, self.custom = gp_model, scaler, use_custom_predict

    def q(self, y):
        xs = self.scaler.transform(np.asarray(y).reshape(1, -1))
        if not self.custom:
            return self.gp.predict(xs).ravel()
        return self.gp.kernel_(self.gp.X_train_, xs).ravel() @ self.gp.alpha_

    def dq(self, y):
        xs = self.scaler.transform(np.asarray(y).reshape(1, -1)).ravel()
        k = self.gp.kernel_
        g = matern15_grad(xs, self.gp.X_train_, k.k2.length_scale, k.k1.constant_value)
        return (self.gp.alpha_.T @ g) * self.scaler.scale_


# --- drop-in reference functions (numpy, host) ---------------------------------

def decode_rbf_nearest_neighbors(x, epsilon, neighbors, kdtree, q_p_train, q_s_train, basis,
                                 basis2, scaler, kernel_type="gaussian"):
    """C/hypernet2D.py:1279-1314."""
    qmap = RBFNearestNeighborsMap(kdtree, q_p_train, q_s_train, epsilon, neighbors, scaler,
                                  kernel_type)
    return basis @ x + basis2 @ qmap.q(x)


def jac_rbf_nearest_neighbors(x, kdtree, q_p_train, q_s_train, basis, basis2, epsilon, neighbors,
                              scaler, kernel_type="gaussian"):
    """C/hypernet2D.py:1316-1350."""
    qmap = RBFNearestNeighborsMap(kdtree, q_p_train, q_s_train, epsilon, neighbors, scaler,
                                  kernel_type)
    return basis + basis2 @ qmap.dq(x)


def decode_rbf_global(x, W_global, q_p_train, basis, basis2, epsilon, scaler,
                      kernel_type="gaussian", echo_level=0):
    """C/hypernet2D.py:1352-1394."""
    return basis @ x + basis2 @ RBFGlobalMap(W_global, q_p_train, epsilon, scaler,
                                             kernel_type).q(x)


def jac_rbf_global(x, W_global, q_p_train, q_s_train, basis, basis2, epsilon, scaler,
                   kernel_type="gaussian", echo_level=0):
    """C/hypernet2D.py:1397-1445."""
    return basis + basis2 @ RBFGlobalMap(W_global, q_p_train, epsilon, scaler,
                                         kernel_type).dq(x)


def decode_gp(x, gp_model, basis, basis2, scaler, use_custom_predict=True, echo_level=0):
    """C/hypernet2D.py:1447-1495."""
    return basis @ x + basis2 @ GPMap(gp_model, scaler, use_custom_predict).q(x)


def jac_gp(x, gp_model, basis, basis2, scaler, echo_level=0):
    """C/hypernet2D.py:1754-1808."""
    return basis + basis2 @ GPMap(gp_model, scaler).dq(x)
