"""Context object over libburgers_hip: one grid on one MI355X.

FOMContext owns a ``burg_ctx`` (device buffers, HIP stream).  It is the only
place the package calls into the C ABI; hypernet2D.py / run_fom.py build the
reference-compatible API on top of it.
"""
import ctypes
import threading
import warnings

import numpy as np

from . import _lib
from .grid import fom_coefficients

DEFAULT_TOL = 2.0 ** -50  # 4 ulp relative inflow motion
NPY_GLOBAL, NPY_EXISTING = 1, 2  # burg_run_npy_ex flags (include/burgers.h)


class FOMContext:
    """A grid (nx x ny) resident on one GPU."""

    def __init__(self, nx, ny, device=0, tile_w=64, par_passes=0, tol=DEFAULT_TOL,
                 profile=False, engine="pipe", stream_w=0, tiles_target=0, _slab=None):
        self._L = _lib.load()
        self.nx, self.ny, self.device = int(nx), int(ny), int(device)
        h = ctypes.c_void_p()
        if _slab is None:
            self.ny_total, self.row0, self.rank, self.world = self.ny, 0, 0, 1
            _lib.check(self._L.burg_ctx_create(self.device, self.nx, self.ny, ctypes.byref(h)))
        else:
            self.ny_total, self.row0, self.rank, self.world, name = _slab
            _lib.check(self._L.burg_ctx_create_slab(self.device, self.nx, self.ny_total, self.row0,
                                                    self.ny, self.rank, self.world,
                                                    name.encode(), ctypes.byref(h)))
        self._h = h
        self._problem = None
        self.set_options(tile_w, par_passes, tol, profile)
        self.set_engine(engine, stream_w, tiles_target)

    @classmethod
    def slab(cls, nx, ny_total, row0, rows, rank, world, halo_name, device=0, **opts):
        """Rank `rank`'s slab (global rows [row0, row0+rows)) of an nx x ny_total
        grid; call connect() once every rank has created its slab context."""
        return cls(nx, rows, device, _slab=(int(ny_total), int(row0), int(rank), int(world),
                                            str(halo_name)), **opts)

    def connect(self):
        _lib.check(self._L.burg_slab_connect(self._h))

    def verify(self):
        """Consumer-side self-test of a device halo ring (after a barrier that
        follows every rank's connect(); a barrier must follow it before the
        first launch).  A failed test moves the boundary to the host ring."""
        _lib.check(self._L.burg_slab_verify(self._h))

    def halo_note(self):
        """Why this slab's halo is not on a device ring ('' if it is)."""
        return (self._L.burg_slab_halo_note(self._h) or b"").decode()

    def halo_modes(self):
        """(in, out) halo ring placement of a slab context: 0 none (end rank),
        1 pinned host memory, 2 the consumer GPU's device memory (IPC).  The
        inbound mode is known once the rank below has connected."""
        a, b = ctypes.c_int(), ctypes.c_int()
        _lib.check(self._L.burg_slab_halo_mode(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    @property
    def m(self):
        return 2 * self.nx * self.ny

    def close(self):
        if getattr(self, "_h", None):
            self._L.burg_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_options(self, tile_w=64, par_passes=0, tol=DEFAULT_TOL, profile=False):
        _lib.check(self._L.burg_set_options(self._h, int(tile_w), int(par_passes), float(tol),
                                            1 if profile else 0))
        self.options = dict(tile_w=tile_w, par_passes=par_passes, tol=tol, profile=profile)

    def set_engine(self, engine="pipe", stream_w=0, tiles_target=0):
        """March engine: "pipe" (the default: exact pipelined march, one launch
        per run chunk, LDS edges and a comm wave per workgroup; falls back to
        "stream" on one GPU when the grid needs tiles wider than 16),
        "stream" (the same march, edges polled by the compute waves) or
        "tiles" (block-Jacobi tile passes per step, tuned by set_options)."""
        _lib.check(self._L.burg_set_engine(self._h, _lib.ENGINES[engine], int(stream_w),
                                           int(tiles_target)))
        self.engine = dict(engine=engine, stream_w=stream_w, tiles_target=tiles_target)

    def set_problem(self, grid_x, grid_y, dt, mu, allow_nonsquare=False):
        """Global grid arrays (a slab context picks its own rows)."""
        key = (np.asarray(grid_x).tobytes(), np.asarray(grid_y).tobytes(), float(dt),
               float(mu[0]), float(mu[1]), bool(allow_nonsquare))
        if key == self._problem:
            return
        ix, iy, src, lbc = fom_coefficients(grid_x, grid_y, dt, mu, allow_nonsquare)
        self._grid = (np.asarray(grid_x, dtype=np.float64), np.asarray(grid_y, dtype=np.float64),
                      float(dt), bool(allow_nonsquare))
        if ix.size != self.nx or iy.size != self.ny_total:
            raise ValueError("grid does not match the context shape")
        _lib.check(self._L.burg_set_problem(self._h, _lib.dptr(ix), _lib.dptr(iy),
                                            _lib.dptr(src), _lib.dptr(lbc), float(dt)))
        self._problem = key

    def _vec(self, a, name):
        a = np.ascontiguousarray(np.asarray(a, dtype=np.float64).ravel())
        if a.size != self.m:
            raise ValueError(f"{name} has {a.size} entries, expected {self.m}")
        return a

    # ---- parity hooks -----------------------------------------------------
    def residual(self, w, wp):
        w, wp = self._vec(w, "w"), self._vec(wp, "wp")
        r = np.empty(self.m)
        nrm = ctypes.c_double()
        _lib.check(self._L.burg_residual(self._h, _lib.dptr(w), _lib.dptr(wp), _lib.dptr(r),
                                         ctypes.byref(nrm)))
        return r, nrm.value

    def slab_residual(self, w, wp, halo_w=None, halo_wp=None):
        """This slab's rows of R(w; wp) (burg_slab_residual): w, wp are the
        slab's rows; halo_w / halo_wp = [u row | v row] of the global row just
        below the slab (None on the bottom slab).  Returns (r, sum of squares
        of r)."""
        w, wp = self._vec(w, "w"), self._vec(wp, "wp")
        hw = hwp = None
        if halo_w is not None or halo_wp is not None:
            hw = np.ascontiguousarray(np.asarray(halo_w, dtype=np.float64).ravel())
            hwp = np.ascontiguousarray(np.asarray(halo_wp, dtype=np.float64).ravel())
            if hw.size != 2 * self.nx or hwp.size != 2 * self.nx:
                raise ValueError(f"halo rows need 2*nx = {2 * self.nx} entries")
        r = np.empty(self.m)
        ss = ctypes.c_double()
        _lib.check(self._L.burg_slab_residual(self._h, _lib.dptr(w), _lib.dptr(wp), _lib.dptr(hw),
                                              _lib.dptr(hwp), _lib.dptr(r), ctypes.byref(ss)))
        return r, ss.value

    def jvp(self, w, x):
        w, x = self._vec(w, "w"), self._vec(x, "x")
        y = np.empty(self.m)
        _lib.check(self._L.burg_jvp(self._h, _lib.dptr(w), _lib.dptr(x), _lib.dptr(y)))
        return y

    def block_solve(self, w, rhs):
        w, rhs = self._vec(w, "w"), self._vec(rhs, "rhs")
        d = np.empty(self.m)
        _lib.check(self._L.burg_block_solve(self._h, _lib.dptr(w), _lib.dptr(rhs),
                                            _lib.dptr(d)))
        return d

    # ---- time loop --------------------------------------------------------
    def run(self, w0, num_steps, solver="march", newton_max_its=100, newton_rtol=1e-12,
            snap_every=1, keep_snaps=True, out=None):
        """Returns (snaps (m, num_steps//snap_every + 1) C-order or None,
        stats dict, per-step iterations int32[num_steps], per-step rel[num_steps]).
        out: an existing C-contiguous float64 (m, ncols) array to fill instead
        of a new one -- e.g. np.lib.format.open_memmap of the snapshot cache
        file, so the snapshots stream from HBM into the .npy file's pages."""
        w0 = self._vec(w0, "w0")
        ncols = num_steps // snap_every + 1
        snaps = _out_array(out, self.m, ncols) if keep_snaps else None
        its = np.zeros(num_steps, dtype=np.int32)
        rel = np.zeros(num_steps)
        st = _lib.BurgStats()
        code = self._L.burg_run(self._h, _lib.dptr(w0), int(num_steps), _lib.SOLVERS[solver],
                                int(newton_max_its), float(newton_rtol),
                                _lib.dptr(snaps), ncols, int(snap_every), ctypes.byref(st),
                                _lib.iptr(its), _lib.dptr(rel))
        _lib.check(code, allow=(_lib.BURG_ENOCONV,))
        if code == _lib.BURG_ENOCONV:
            warnings.warn(self._L.burg_last_error().decode(), _lib.NotConvergedWarning)
        return snaps, st.as_dict(), its, rel

    def run_to_npy(self, w0, num_steps, path, snap_every=1, flags=0):
        """One trajectory written straight into the .npy file `path`
        (burg_run_npy_ex: pinned buffers, pwrite writer thread); returns stats
        (loop_ms launch, flush_ms gathers + D2H, march_kernel_ms whole call).
        flags: NPY_GLOBAL -- a slab context writes its rows at their places in
        the whole grid's matrix; NPY_EXISTING -- into a file another rank made
        (write_npy_header) instead of creating it (include/burgers.h)."""
        w0 = self._vec(w0, "w0")
        st = _lib.BurgStats()
        _lib.check(self._L.burg_run_npy_ex(self._h, _lib.dptr(w0), int(num_steps), int(snap_every),
                                           str(path).encode(), int(flags), ctypes.byref(st)))
        return st.as_dict()

    def upload(self, w):
        w = self._vec(w, "w")
        _lib.check(self._L.burg_upload_state(self._h, _lib.dptr(w)))

    def download(self):
        w = np.empty(self.m)
        _lib.check(self._L.burg_download_state(self._h, _lib.dptr(w)))
        return w

    def reserve(self, num_steps, snap_every=1):
        """Allocate the tiling, mailboxes and HBM ring trajectory(num_steps,
        snap_every=...) needs, without launching (burg_reserve_trajectory_ex):
        multi-GPU ranks call it before the barrier that precedes their first
        launch."""
        _lib.check(self._L.burg_reserve_trajectory_ex(self._h, int(num_steps), int(snap_every)))

    def trajectory(self, num_steps, from_initial=True, snap_every=1):
        """num_steps steps in one launch from the uploaded initial state (or,
        from_initial=False, from the resident state); returns stats (loop_ms =
        the launch's device time).  The states kept in HBM
        (burg_trajectory_ex): snap_every=1 every state while they fit (a ring
        capped by free HBM keeps the last ones), snap_every=k states 0, k, 2k,
        ..., snap_every=0 auto (1 if the whole trajectory fits, else 10); see
        retained() and trajectory_snaps()."""
        st = _lib.BurgStats()
        _lib.check(self._L.burg_trajectory_ex(self._h, int(num_steps), int(snap_every),
                                              1 if from_initial else 0, ctypes.byref(st)))
        return st.as_dict()

    def trajectory_plan(self, num_steps, snap_every=1):
        """(resolved snap_every, retained states or -1 for a capped ring, ring
        bytes) of trajectory(num_steps, snap_every=...), without allocating."""
        k, n, b = ctypes.c_int(), ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self._L.burg_trajectory_plan(self._h, int(num_steps), int(snap_every),
                                                ctypes.byref(k), ctypes.byref(n), ctypes.byref(b)))
        return k.value, n.value, b.value

    def retained(self):
        """(first_state, count, stride): the states the last trajectory() keeps
        resident are first_state + j * stride, j < count."""
        f, n, k = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int()
        _lib.check(self._L.burg_trajectory_retained(self._h, ctypes.byref(f), ctypes.byref(n),
                                                    ctypes.byref(k)))
        return f.value, n.value, k.value

    def trajectory_snaps(self, col0=0, ncols=None, out=None):
        """Retained columns col0 .. col0 + ncols - 1 of the last trajectory()
        as a C-order (2n, ncols) snapshot matrix (the reference's layout,
        C/hypernet2D.py:89-90,126): a new numpy array, `out` (numpy, written
        in place), or a contiguous float64 torch tensor on this context's GPU
        (burg_trajectory_copy on the device, no host round trip)."""
        first, count, stride = self.retained()
        ncols = count - col0 if ncols is None else int(ncols)
        if out is not None and not isinstance(out, np.ndarray):
            import torch
            dev = torch.device("cuda", self.device)
            if (out.dtype != torch.float64 or out.device != dev or not out.is_contiguous()
                    or out.dim() != 2 or out.shape[0] != self.m or out.shape[1] < ncols):
                raise ValueError(f"out must be a contiguous float64 ({self.m}, >= {ncols}) tensor "
                                 f"on {dev}")
            torch.cuda.current_stream(dev).synchronize()
            _lib.check(self._L.burg_trajectory_copy(self._h, int(col0), ncols, out.data_ptr(),
                                                    int(out.shape[1]), 1))
            return out
        snaps = _out_array(out, self.m, ncols)
        _lib.check(self._L.burg_trajectory_copy(self._h, int(col0), ncols,
                                                snaps.ctypes.data_as(ctypes.c_void_p), ncols, 0))
        return snaps

    def sweep(self, mus, num_steps, w0=None, keep_snaps=True, snap_every=1, outs=None):
        """Parameter sweep (burg_sweep): one trajectory of num_steps steps per
        mu in `mus`, all from w0 (None: the state last passed to upload()),
        on the grid and dt of the last set_problem, back to back in one
        pipelined launch per group of trajectories.  Returns (list of snapshot
        matrices (m, num_steps//snap_every + 1), or None with
        keep_snaps=False -- then the states stay in HBM --, stats).  outs: a
        list of existing (m, ncols) C-contiguous float64 arrays (None entries:
        allocate) to fill, as run()'s out."""
        if getattr(self, "_grid", None) is None:
            raise RuntimeError("set_problem first")
        gx, gy, dt, nonsq = self._grid
        mus = [tuple(float(x) for x in mu) for mu in mus]
        if not mus:
            raise ValueError("empty mu list")
        src_b, lbc_b = [], []
        for mu in mus:
            _, _, src, lbc = fom_coefficients(gx, gy, dt, mu, nonsq)
            src_b.append(src)
            lbc_b.append(lbc)
        src_b = np.ascontiguousarray(np.stack(src_b))
        lbc_b = np.ascontiguousarray(np.stack(lbc_b))
        if w0 is not None:
            self.upload(w0)
        ncols = num_steps // snap_every + 1
        snaps = None
        ptrs = None
        if keep_snaps:
            outs = list(outs) if outs is not None else [None] * len(mus)
            if len(outs) != len(mus):
                raise ValueError("outs must have one entry per mu")
            snaps = [_out_array(o, self.m, ncols) for o in outs]
            ptrs = (_lib._D * len(mus))(*[_lib.dptr(a) for a in snaps])
        st = _lib.BurgStats()
        _lib.check(self._L.burg_sweep(self._h, len(mus), _lib.dptr(src_b), _lib.dptr(lbc_b),
                                      int(num_steps), ptrs, ncols, int(snap_every),
                                      ctypes.byref(st)))
        return snaps, st.as_dict()

    def _sweep_tables(self, mus):
        gx, gy, dt, nonsq = self._grid
        src_b, lbc_b = [], []
        for mu in mus:
            _, _, src, lbc = fom_coefficients(gx, gy, dt, mu, nonsq)
            src_b.append(src)
            lbc_b.append(lbc)
        return np.ascontiguousarray(np.stack(src_b)), np.ascontiguousarray(np.stack(lbc_b))

    def sweep_device(self, mus, num_steps, w0=None, snap_every=1, out=None):
        """sweep() with the snapshot set left in HBM (burg_sweep_device):
        returns (a float64 CUDA tensor (m, len(mus) * ncols) = np.hstack of the
        per-mu snapshot matrices -- `out` if given, written in place --,
        stats)."""
        import torch
        if getattr(self, "_grid", None) is None:
            raise RuntimeError("set_problem first")
        mus = [tuple(float(x) for x in mu) for mu in mus]
        if not mus:
            raise ValueError("empty mu list")
        src_b, lbc_b = self._sweep_tables(mus)
        if w0 is not None:
            self.upload(w0)
        ncols = num_steps // snap_every + 1
        dev = torch.device("cuda", self.device)
        if out is None:
            out = torch.empty((self.m, len(mus) * ncols), dtype=torch.float64, device=dev)
        elif (out.dtype != torch.float64 or out.device != dev or not out.is_contiguous()
              or out.dim() != 2 or out.shape[0] != self.m or out.shape[1] < len(mus) * ncols):
            raise ValueError(f"out must be a contiguous float64 ({self.m}, >= {len(mus) * ncols}) "
                             f"tensor on {dev}")
        torch.cuda.current_stream(dev).synchronize()
        st = _lib.BurgStats()
        _lib.check(self._L.burg_sweep_device(self._h, len(mus), _lib.dptr(src_b), _lib.dptr(lbc_b),
                                             int(num_steps), int(snap_every), out.data_ptr(),
                                             int(out.shape[1]), ctypes.byref(st)))
        return out, st.as_dict()

    def ecsw_matrix(self, snaps, prev_snaps, basis, return_stats=False):
        """ECSW training matrix (burg_ecsw_matrix) of snapshot columns
        snaps[:, i] with previous states prev_snaps[:, i] and a (2n, npod)
        basis, on the problem of the last set_problem: (npod*nsnaps, n)."""
        snaps = np.asarray(snaps, dtype=np.float64)
        prev_snaps = np.asarray(prev_snaps, dtype=np.float64)
        if snaps.ndim != 2 or snaps.shape[0] != self.m or prev_snaps.shape != snaps.shape:
            raise ValueError("snaps / prev_snaps must be (2*nx*ny, n_snaps) and equal in shape")
        basis = np.ascontiguousarray(np.asarray(basis, dtype=np.float64))
        if basis.ndim != 2 or basis.shape[0] != self.m:
            raise ValueError("basis must be (2*nx*ny, n_pod)")
        ns, npod = snaps.shape[1], basis.shape[1]
        states = np.ascontiguousarray(snaps.T)  # state-major: column i contiguous
        prev = np.ascontiguousarray(prev_snaps.T)
        C = np.zeros((npod * ns, self.m // 2))
        st = _lib.BurgStats()
        _lib.check(self._L.burg_ecsw_matrix(self._h, ns, _lib.dptr(states), _lib.dptr(prev), npod,
                                            _lib.dptr(basis), _lib.dptr(C), ctypes.byref(st)))
        return (C, st.as_dict()) if return_stats else C

    def ecsw_block_device(self, state, prev, basis_t, out):
        """One snapshot's ECSW block with its own basis, on device tensors
        (burg_ecsw_block_device; the decoder variants of
        compute_ECSW_training_matrix_2D, C/hypernet2D.py:2742-3072):
        state, prev (2n,) and basis_t (npod, 2n) = V^T, float64 on this
        context's GPU; out (npod, n) receives the block.  Returns the kernel
        time in ms."""
        import torch
        dev = torch.device("cuda", self.device)
        npod = basis_t.shape[0] if basis_t.dim() == 2 else -1
        for name, t, shape in (("state", state, (self.m,)), ("prev", prev, (self.m,)),
                               ("basis_t", basis_t, (npod, self.m)),
                               ("out", out, (npod, self.m // 2))):
            if t.dtype != torch.float64 or t.device != dev or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous float64 tensor on {dev}")
            if tuple(t.shape) != shape:
                raise ValueError(f"{name} has shape {tuple(t.shape)}, expected {shape}")
        torch.cuda.current_stream(dev).synchronize()  # inputs written on torch's stream
        ms = ctypes.c_float(0.0)
        _lib.check(self._L.burg_ecsw_block_device(self._h, state.data_ptr(), prev.data_ptr(),
                                                  int(npod), basis_t.data_ptr(), out.data_ptr(),
                                                  ctypes.byref(ms)))
        return ms.value

    def lspg(self, w0, num_steps, basis, max_its=20, relnorm_cutoff=1e-5, min_delta=0.1,
             keep_snaps=True, keep_coords=True):
        """LSPG PROM trajectory (burg_lspg; inviscid_burgers_implicit2D_LSPG,
        C/hypernet2D.py:133-200, gauss_newton_LSPG :1859-1929) on the problem of
        the last set_problem.  Returns (snaps (2n, T+1) or None, red_coords
        (npod, T+1) or None, its per step, rel per step, times_ms [jac, res,
        ls], stats)."""
        basis = np.ascontiguousarray(np.asarray(basis, dtype=np.float64))
        if basis.ndim != 2 or basis.shape[0] != self.m:
            raise ValueError("basis must be (2*nx*ny, n_pod)")
        w0 = np.ascontiguousarray(np.asarray(w0, dtype=np.float64).ravel())
        if w0.size != self.m:
            raise ValueError("w0 must have 2*nx*ny entries")
        T, npod = int(num_steps), basis.shape[1]
        snaps = np.zeros((self.m, T + 1)) if keep_snaps else None
        red = np.zeros((npod, T + 1)) if keep_coords else None
        its = np.zeros(T, dtype=np.int32)
        rel = np.zeros(T)
        times = np.zeros(3)
        st = _lib.BurgStats()
        _lib.check(self._L.burg_lspg(self._h, _lib.dptr(w0), T, npod, _lib.dptr(basis),
                                     int(max_its), float(relnorm_cutoff), float(min_delta),
                                     _lib.dptr(snaps), T + 1, _lib.dptr(red), T + 1,
                                     _lib.iptr(its), _lib.dptr(rel), _lib.dptr(times),
                                     ctypes.byref(st)))
        return snaps, red, its, rel, times, st.as_dict()

    def kernel_bench(self, kernel="residual", reps=20):
        """Mean device time (ms) of one launch of the residual or J.x stencil
        on device-resident operands (burg_kernel_bench; upload() first)."""
        ms = ctypes.c_double(0.0)
        _lib.check(self._L.burg_kernel_bench(self._h, _lib.KERNELS[kernel], int(reps),
                                             ctypes.byref(ms)))
        return ms.value

    def advance(self, num_steps, solver="march"):
        st = _lib.BurgStats()
        _lib.check(self._L.burg_advance(self._h, int(num_steps), _lib.SOLVERS[solver],
                                        ctypes.byref(st)), allow=())
        return st.as_dict()


def _out_array(out, m, ncols):
    if out is None:
        return np.zeros((m, ncols))
    if (not isinstance(out, np.ndarray) or out.dtype != np.float64 or out.shape != (m, ncols)
            or not out.flags.c_contiguous or not out.flags.writeable):
        raise ValueError(f"out must be a writeable C-contiguous float64 ({m}, {ncols}) array")
    return out


_cache = threading.local()


def get_context(nx, ny, device=0, **opts):
    """Per-thread cached context for (device, nx, ny); options re-applied."""
    d = getattr(_cache, "ctxs", None)
    if d is None:
        d = _cache.ctxs = {}
    key = (int(device), int(nx), int(ny))
    eopts = {k: opts.pop(k) for k in ("engine", "stream_w", "tiles_target") if k in opts}
    ctx = d.get(key)
    if ctx is None:
        ctx = d[key] = FOMContext(nx, ny, device, **opts, **eopts)
        return ctx
    if opts and any(ctx.options.get(k) != v for k, v in opts.items()):
        merged = dict(ctx.options)
        merged.update(opts)
        ctx.set_options(**merged)
    if eopts and any(ctx.engine.get(k) != v for k, v in eopts.items()):
        merged = dict(ctx.engine)
        merged.update(eopts)
        ctx.set_engine(**merged)
    return ctx
