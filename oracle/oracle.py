"""Python face of the CPU oracle (oracle/burgers_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker -- never by the product package.
Parity of this restatement with the reference is pinned by the fixtures in
tests/golden/ (made by importing the Python reference in the build container)
and by the author's pickled HDM slices and SLURM logs; see
tests/test_oracle_golden.py.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liborcl.so")
_D = ctypes.POINTER(ctypes.c_double)
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(
                os.path.join(HERE, "burgers_oracle.c")):
            build()
        L = ctypes.CDLL(LIB)
        L.orc_newton_step.restype = ctypes.c_int
        L.orc_fom.restype = ctypes.c_int
        L.orc_march_tiled_sim.restype = ctypes.c_int
        L.orc_march_tiled_sim.argtypes = [ctypes.c_int, ctypes.c_int, _D, _D, _D, _D,
                                          ctypes.c_double, _D, _D, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_double,
                                          ctypes.POINTER(ctypes.c_longlong)]
        _lib = L
    return _lib


def _p(a):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_D)


class Problem:
    """Coefficient vectors of one (grid, dt, mu), NumPy-rounded like the reference
    (same formulas as finitedifference_amd.grid.fom_coefficients, restated here
    so the checker does not import the product)."""

    def __init__(self, nx, ny=None, dt=0.05, mu=(5.19, 0.026), L=100.0, Ly=None,
                 allow_nonsquare=False):
        ny = nx if ny is None else ny
        gx = np.linspace(0, L, nx + 1)
        gy = np.linspace(0, L if Ly is None else Ly, ny + 1)
        dx, dy = gx[1:] - gx[:-1], gy[1:] - gy[:-1]
        xc = (gx[1:] + gx[:-1]) / 2
        self.nx, self.ny, self.dt, self.mu = nx, ny, float(dt), tuple(mu)
        self.grid_x, self.grid_y = gx, gy
        self.inv_dx = np.ascontiguousarray(np.ones(nx) / dx)
        self.inv_dy = np.ascontiguousarray(np.ones(ny) / dy)
        self.src = np.ascontiguousarray(dt * 0.02 * np.exp(mu[1] * xc))
        if nx == ny:
            self.lbc = np.ascontiguousarray(0.5 * dt * mu[0] ** 2 / dx)
        elif allow_nonsquare:
            self.lbc = np.full(ny, 0.5 * dt * mu[0] ** 2 / dx[0])
        else:
            raise ValueError("reference requires nx == ny")
        self.m = 2 * nx * ny

    def _c(self):
        return (self.nx, self.ny, _p(self.inv_dx), _p(self.inv_dy), _p(self.src), _p(self.lbc),
                ctypes.c_double(self.dt))

    def residual(self, w, wp):
        r = np.empty(self.m)
        lib().orc_residual(*self._c(), _p(np.ascontiguousarray(w, dtype=np.float64)),
                           _p(np.ascontiguousarray(wp, dtype=np.float64)), _p(r))
        return r

    def jvp(self, w, x):
        y = np.empty(self.m)
        lib().orc_jvp(self.nx, self.ny, _p(self.inv_dx), _p(self.inv_dy), ctypes.c_double(self.dt),
                      _p(np.ascontiguousarray(w, dtype=np.float64)),
                      _p(np.ascontiguousarray(x, dtype=np.float64)), _p(y))
        return y

    def block_solve(self, w, rhs):
        d = np.empty(self.m)
        lib().orc_block_solve(self.nx, self.ny, _p(self.inv_dx), _p(self.inv_dy),
                              ctypes.c_double(self.dt),
                              _p(np.ascontiguousarray(w, dtype=np.float64)),
                              _p(np.ascontiguousarray(rhs, dtype=np.float64)), _p(d))
        return d

    def march_step(self, wp):
        w = np.empty(self.m)
        lib().orc_march_step(*self._c(), _p(np.ascontiguousarray(wp, dtype=np.float64)), _p(w))
        return w

    def march_tiled(self, wp, tw=64, th=64, tol=2.0 ** -50, kmax=100000):
        w = np.empty(self.m)
        done = ctypes.c_longlong(0)
        k = lib().orc_march_tiled_sim(*self._c(), _p(np.ascontiguousarray(wp, dtype=np.float64)),
                                      _p(w), th, tw, kmax, tol, ctypes.byref(done))
        return w, k, done.value

    def newton_step(self, wp, max_its=100, cutoff=1e-12):
        w = np.empty(self.m)
        rel = ctypes.c_double()
        its = lib().orc_newton_step(*self._c(), _p(np.ascontiguousarray(wp, dtype=np.float64)),
                                    _p(w), max_its, ctypes.c_double(cutoff), ctypes.byref(rel))
        return w, its, rel.value

    def march_sweep(self, w0, mus, num_steps, threads):
        """CPU baseline: one march trajectory per mu (same grid and dt), one
        OpenMP thread each (orc_march_sweep); returns the threads used."""
        srcs, lbcs = [], []
        for mu in mus:
            q = Problem(self.nx, self.ny, self.dt, mu, Ly=self.grid_y[-1],
                        allow_nonsquare=self.nx != self.ny)
            srcs.append(q.src)
            lbcs.append(q.lbc)
        src_b = np.ascontiguousarray(np.stack(srcs))
        lbc_b = np.ascontiguousarray(np.stack(lbcs))
        return lib().orc_march_sweep(self.nx, self.ny, _p(self.inv_dx), _p(self.inv_dy),
                                     _p(src_b), _p(lbc_b), ctypes.c_double(self.dt),
                                     _p(np.ascontiguousarray(w0, dtype=np.float64)), len(mus),
                                     int(num_steps), int(threads))

    def march_traj(self, w0, num_steps, snap_every=1, threads=None):
        """orc_march_step's trajectory, rows pipelined over OpenMP threads
        (orc_march_traj_par: bit-identical, for the bench-size checks).
        Returns the step-major states after 0, snap_every, 2*snap_every, ...
        steps, shape (num_steps // snap_every + 1, m)."""
        if threads is None:
            n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 1
            omp = os.environ.get("OMP_NUM_THREADS", "")
            threads = max(1, min(n, int(omp))) if omp.isdigit() else n
        out = np.empty((num_steps // snap_every + 1, self.m))
        lib().orc_march_traj_par(*self._c(), _p(np.ascontiguousarray(w0, dtype=np.float64)),
                                 int(num_steps), int(snap_every), _p(out), int(threads))
        return out

    def fom(self, w0, num_steps, solver="march", max_its=100, cutoff=1e-12):
        """Step-major trajectory (num_steps+1, m) + Newton counts/rels."""
        snaps = np.empty((num_steps + 1, self.m))
        its = np.zeros(num_steps, dtype=np.int32)
        rel = np.zeros(num_steps)
        lib().orc_fom(*self._c(), _p(np.ascontiguousarray(w0, dtype=np.float64)), num_steps,
                      0 if solver == "newton" else 1, max_its, ctypes.c_double(cutoff),
                      _p(snaps), its.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), _p(rel))
        return snaps, its, rel

    def ecsw_matrix(self, snaps, prev_snaps, basis):
        """compute_ECSW_training_matrix_2D (C/hypernet2D.py:2719-2740) restated:
        per snapshot column, the residual R(snap; prev) and W = J(snap) @ basis
        column by column (orc_residual / orc_jvp), then
        C[isnap*npod + k, node] = R_u[node] W_u[node, k] + R_v[node] W_v[node, k]
        (the reference's inner loop, :2737-2738).  Column-major snapshots as in
        the reference; the residual follows res2D_alt's op order (the reference
        passes res2D, :2468-2510, equal to 4.4e-16)."""
        snaps = np.asarray(snaps, dtype=np.float64)
        prev_snaps = np.asarray(prev_snaps, dtype=np.float64)
        basis = np.asarray(basis, dtype=np.float64)
        m, ns = snaps.shape
        n = m // 2
        npod = basis.shape[1]
        C = np.zeros((npod * ns, n))
        for i in range(ns):
            r = self.residual(snaps[:, i], prev_snaps[:, i])
            Wi = np.stack([self.jvp(snaps[:, i], basis[:, k]) for k in range(npod)], axis=1)
            C[i * npod:(i + 1) * npod, :] = (r[:n, None] * Wi[:n] + r[n:, None] * Wi[n:]).T
        return C

    def lspg_jvp(self, w, x):
        """J_LSPG(w) @ x of inviscid_burgers_implicit2D_LSPG (C/hypernet2D.py:133-200):
        exact_jac2D (:2627-2656) with the driver's JDyec = kron(I, Dy)[perm, :]
        (rows permuted only, :165-167; the FOM permutes rows and columns,
        :98-106).  For nx == ny that operator is (Y f)[r, c] =
        f[c, r]/dy_r - f[c, r-1]/dy_{r-1}: the y-difference of the transposed
        field.  JDxec = kron(I, Dx) is the row-wise backward difference
        (make_ddx, :2410-2416)."""
        assert self.nx == self.ny, "the LSPG Jacobian is defined for square grids"
        N, n, a = self.nx, self.nx * self.nx, 0.5 * self.dt
        u, v = w[:n].reshape(N, N), w[n:].reshape(N, N)
        xu, xv = x[:n].reshape(N, N), x[n:].reshape(N, N)

        def Dx(f):
            g = f * self.inv_dx[None, :]
            out = g.copy()
            out[:, 1:] -= g[:, :-1]
            return out

        def Y(f):
            g = f.T * self.inv_dy[:, None]
            out = g.copy()
            out[1:, :] -= g[:-1, :]
            return out

        yu = xu + Dx(a * u * xu) + 0.5 * Y(a * v * xu) + 0.5 * Y(a * u * xv)
        yv = xv + 0.5 * Dx(a * v * xu) + Y(a * v * xv) + 0.5 * Dx(a * u * xv)
        return np.concatenate((yu.ravel(), yv.ravel()))

    def lspg(self, w0, num_steps, basis, max_its=20, relnorm_cutoff=1e-5, min_delta=0.1):
        """inviscid_burgers_implicit2D_LSPG (C/hypernet2D.py:133-200) with
        gauss_newton_LSPG (:1859-1929) restated: y0 = basis^T w0; per step
        Gauss-Newton from the previous y with np.linalg.lstsq(J basis, -R).
        The residual is orc_residual (res2D_alt op order; the reference's LSPG
        calls res2D, equal to round-off).  Returns (snaps (2n, T+1), its per
        step = len(resnorms), rel per step = the printed relative norm)."""
        basis = np.asarray(basis, dtype=np.float64)
        npod = basis.shape[1]
        y = basis.T.dot(w0)
        w = basis.dot(y)
        snaps = np.zeros((self.m, num_steps + 1))
        snaps[:, 0] = w
        its = np.zeros(num_steps, dtype=np.int32)
        rels = np.zeros(num_steps)
        for s in range(num_steps):
            wp = w.copy()
            init = np.linalg.norm(self.residual(w, wp))
            resnorms = []
            for i in range(max_its):
                f = self.residual(w, wp)
                rn = np.linalg.norm(f)
                resnorms.append(rn)
                if rn / init < relnorm_cutoff:
                    break
                if len(resnorms) > 1 and abs((resnorms[-2] - resnorms[-1]) / resnorms[-2]) < min_delta:
                    break
                JV = np.stack([self.lspg_jvp(w, basis[:, k]) for k in range(npod)], axis=1)
                dy = np.linalg.lstsq(JV, -f, rcond=None)[0]
                y = y + dy
                w = basis.dot(y)
            its[s], rels[s] = len(resnorms), rn / init
            snaps[:, s + 1] = w
        return snaps, its, rels


def svd_flip_u(u):
    """sklearn's svd_flip rule on u: each column's largest-|.| entry positive."""
    idx = np.argmax(np.abs(u), axis=0)
    sg = np.sign(u[idx, np.arange(u.shape[1])])
    sg[sg == 0] = 1.0
    return u * sg


def pod_svd(snaps):
    """POD(snaps, method='svd') (C/hypernet2D.py:2670-2695) restated: the thin
    SVD np.linalg.svd(snaps, full_matrices=False) -> (u, s), u's column signs
    normalised by svd_flip_u (LAPACK's are arbitrary)."""
    u, s, _ = np.linalg.svd(np.asarray(snaps, dtype=np.float64), full_matrices=False)
    return svd_flip_u(u), s


def rel_l2(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))
