/*
 * burgers.h -- C ABI of libburgers_hip.so, the MI355X (gfx950) implementation
 * of the SADPR/FiniteDifference full-order-model (FOM) hot path.
 *
 * Reference interfaces replaced (paths relative to /root/reference,
 * C/ = BurgersFD_CleanCoarse/).  The reference has no FFI: every entry point
 * below replaces a Python function and is bound with ctypes by
 * finitedifference_amd/_lib.py (binding stub in INTEGRATION.md).
 *
 *   burg_run            C/hypernet2D.py:72-131   inviscid_burgers_implicit2D
 *                       (time loop + snapshot matrix), including
 *                       C/hypernet2D.py:1811-1857 newton_raphson and
 *                       C/hypernet2D.py:1854      spsolve, which it replaces
 *   burg_residual       C/hypernet2D.py:2512-2570 inviscid_burgers_res2D_alt
 *                       (+ np.linalg.norm of it, :1831/:1839)
 *   burg_jvp            C/hypernet2D.py:2627-2656 inviscid_burgers_exact_jac2D(w) @ x
 *   burg_block_solve    C/hypernet2D.py:1854      spsolve(J(w), rhs)
 *   burg_run_npy        C/hypernet2D.py:3141-3143  inviscid_burgers_implicit2D + np.save
 *                       of the snapshot cache (load_or_compute_snaps)
 *   burg_sweep          a loop of inviscid_burgers_implicit2D over a mu set
 *                       (C/run_prom.py:59-71, C/run_tests.py:38-49)
 *   burg_ecsw_matrix    C/hypernet2D.py:2719-2740 compute_ECSW_training_matrix_2D
 *   burg_ecsw_block_device  one snapshot's C rows of the decoder variants
 *                       C/hypernet2D.py:2742-3072 compute_ECSW_training_matrix_2D_rnm /
 *                       _rbf_nearest_neighbors / _rbf_global / _gp (:2776-2781,
 *                       :2840-2858, :2938-2956, :3050-3070), device pointers
 *   burg_lspg           C/hypernet2D.py:133-200   inviscid_burgers_implicit2D_LSPG
 *                       with C/hypernet2D.py:1859-1929 gauss_newton_LSPG
 *   burg_pod            C/hypernet2D.py:2670-2695   POD(method='svd') (np.linalg.svd)
 *   burg_pod_rsvd       C/hypernet2D.py:2688-2692   POD(method='rsvd') (randomized_svd)
 *   burg_pod_rsvd_device  the same on a device-resident snapshot matrix
 *   burg_sweep_device   C/run_prom.py:59-71  the training snapshot set, left on the device
 *   burg_trajectory_ex  C/hypernet2D.py:72-131  the time loop, snapshots kept in HBM
 *   burg_set_problem    C/hypernet2D.py:2410-2416, 2425-2431, 2536-2554
 *                       (make_ddx / make_2D_grid spacings, source, inlet BC)
 *
 * Conventions
 *   - State w has 2*nx*ny doubles: [u.ravel(), v.ravel()], u row-major
 *     (ny, nx), cell (r, c) at r*nx + c (C/run_fom.py:33-35).
 *   - All pointers passed in are HOST pointers owned by the caller and
 *     borrowed for the duration of the call; the library keeps none of them
 *     (exception: burg_ecsw_block_device takes device pointers, checked).
 *   - Every function returns BURG_OK (0) or a negative BURG_E* code; the
 *     message of the last failure on the calling thread is burg_last_error().
 *   - One context per host thread; a context owns its device buffers,
 *     its HIP stream and (multi-GPU) its halo rings.
 */
#ifndef BURGERS_H
#define BURGERS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BURG_ABI_VERSION 15

enum burg_status {
    BURG_OK = 0,
    BURG_EINVAL = -1,   /* bad argument (null pointer, size, option) */
    BURG_ESHAPE = -2,   /* grid shape not supported (e.g. nx != ny in strict mode) */
    BURG_EHIP = -3,     /* HIP runtime error */
    BURG_EHALO = -4,    /* multi-GPU halo ring error (rendezvous object, device ring over IPC
                           or its pinned host fallback) */
    BURG_ENOMEM = -5,   /* device or pinned-host allocation failed */
    BURG_ENOCONV = -6,  /* solver hit its iteration cap (result still returned) */
    BURG_ENAN = -7,     /* non-finite residual or state */
    BURG_ESTATE = -8    /* call order error (e.g. run before set_problem) */
};

enum burg_solver {
    BURG_SOLVER_MARCH = 0,  /* closed-form upwind march (default, exact implicit step) */
    BURG_SOLVER_NEWTON = 1  /* newton_raphson + exact block solve (reference algorithm) */
};

enum burg_kernel {
    BURG_KERNEL_RESIDUAL = 0,  /* residual stencil + its norm reduction (burg_residual) */
    BURG_KERNEL_JVP = 1        /* Jacobian action J(w) x (burg_jvp) */
};

typedef struct burg_ctx burg_ctx;

typedef struct burg_stats {
    int64_t steps;              /* time steps advanced */
    int64_t tile_marches;       /* tiles marched (all Jacobi passes, all steps) */
    int64_t passes;             /* march launches that did work */
    int32_t max_passes;         /* most passes one step needed (incl. the confirming one) */
    int32_t unconverged_steps;  /* steps that hit the pass cap; 0 on success */
    int64_t newton_updates;     /* newton solver: total Newton updates */
    int32_t newton_max_updates; /* newton solver: most updates in one step */
    int32_t par_passes;         /* parallel passes launched per step (engine option) */
    double loop_ms;             /* device time of the time loop (HIP events) */
    double flush_ms;            /* device time of snapshot transpose + D2H */
    double march_kernel_ms;     /* profiling mode: summed march kernel time */
    int64_t march_launches;     /* profiling mode: march kernel launches timed */
    double last_rel;            /* newton solver: last step's final ||R||/||R0|| */
    int64_t tail_passes;        /* passes finished by the final kernel's last workgroup */
    int32_t engine;             /* march engine used: BURG_ENGINE_* */
    int32_t stream_w;           /* streaming engine: tile width (columns) */
    int64_t stream_tiles;       /* streaming engine: tiles (= wavefronts) per launch */
    int64_t stall_spins;        /* streaming engine: polls of not-yet-ready edge data */
    int64_t slow_diagonals;     /* streaming engine: diagonals that took the slow path */
    int64_t stream_launches;    /* streaming engine: launches (one per run chunk) */
    int64_t slow_ticks;         /* streaming engine: shader clocks spent on the slow path */
    int64_t ieee_diagonals;     /* stream/pipe: diagonals redone with IEEE sqrt/div (range) */
    int64_t comm_polls;         /* pipe engine: comm-wave polling rounds (all workgroups) */
    int64_t nonfinite_diagonals; /* stream/pipe: diagonals whose new state held a NaN/Inf
                                    (the call then returns BURG_ENAN) */
    int64_t paired_launches;    /* pipe engine: launches that ran the paired-halves W = 16
                                   kernel (two cells per lane and diagonal) */
    /* pipe engine, the LAST launch of the call (what a
     * multi-GPU bench line reports per rank): */
    double ramp_ms;             /* first workgroup entry -> the last compute wave's first
                                   block (the pipeline fill, incl. waiting for the rank below) */
    double halo_wait_ms;        /* first workgroup entry -> the first block of the strip fed by
                                   the inbound halo ring (-1: no inbound halo) */
    /* pipe engine, all launches of the call: blocks that waited for south
     * inflow and their summed waiting time (wave-ms), by where the inflow
     * comes from -- a strip of this GPU, or the inbound halo ring */
    int64_t south_waits_local;
    int64_t south_waits_halo;
    double south_wait_ms_local;
    double south_wait_ms_halo;
    /* the context's bounds guards (the flat-pointer ring / transpose kernels,
     * DESIGN.md section 6.1), over its lifetime: copy calls that checked the
     * guard, and how many found it set (each of those returned BURG_EHIP) */
    int64_t bounds_checks;
    int64_t bounds_hits;
} burg_stats;

enum burg_engine {
    BURG_ENGINE_STREAM = 0,  /* one launch for many steps: exact pipelined march, edges polled
                                by the compute waves (any tile width) */
    BURG_ENGINE_TILES = 1,   /* one step at a time: block-Jacobi tile passes (burg_set_options) */
    BURG_ENGINE_PIPE = 2     /* default: the streaming march with LDS edges inside a workgroup
                                and a comm wave per workgroup; narrow tiles (W = 8, 16) keep the
                                previous step in LDS, wide tiles (W = 32 ... 1024) stream it back
                                from the HBM ring through a loader wave; falls back to STREAM on
                                one GPU only when no width up to 1024 keeps every tile resident */
};

int burg_abi_version(void);
const char *burg_last_error(void);

/* Source id of this build: the first 16 hex digits of the SHA-256 of the
 * library's sources (finitedifference_amd/csrc/ *.h, *.hip in byte order, then
 * its Makefile and this header), fixed at compile time.  finitedifference_amd
 * ._lib.source_id() computes the same digest from a checkout, so a test run
 * can show that the shipped binary was built from the tree it runs in. */
const char *burg_build_id(void);
/* The compile flags of this build's objects that change what the kernels do
 * (HIPFLAGS and every -D knob of the Makefile's object rules), fixed at
 * compile time: an A/B or race-screen build (e.g. -DBURG_COMM_PRIO=2) reports
 * the same source id as the shipped one but different flags, so a test run
 * can show that it loaded the default build ("default" + the flags). */
const char *burg_build_flags(void);

/* Host-only audit of the pipe engine's trajectory ring (no GPU, no context):
 * replays, for tile width W, a num_steps trajectory keeping every
 * snap_every-th state (ring_cap > 0: a working ring of ring_cap W + 128
 * entries with retained windows, a plain ring of ring_cap steps without), the
 * ring entries that every kernel touching the ring forms -- the initial-state
 * load, the compute waves' store walk (RetCursor), the loader wave's read
 * walk, the snapshot extracts -- and checks them against the ring's entries
 * per tile and against ring_pos.  report[9]: accesses checked, largest entry,
 * entries per tile, out-of-range entries, walk/ring_pos mismatches, retained
 * cells overwritten before the trajectory ended, ring entries overwritten
 * before the loader read them, retained states, snap_every used.  Returns
 * BURG_OK when the plan exists (the counts say whether it is sound). */
int burg_ring_audit(int W, int num_steps, int snap_every, int ring_cap, int64_t *report);
/* The same with flags: BURG_AUDIT_PAIRED replays the paired-halves W = 16
 * kernel's store walk instead of the one-cell walk (two cells per lane and
 * diagonal: the A cell's entry +1 per diagonal, +9 past column 7, the B cell
 * 8 entries below with its own wrap, and the steady blocks' block-base
 * entries, checked against the per-diagonal walk and ring_pos; plain rings,
 * W = 16). */
#define BURG_AUDIT_PAIRED 1
/* BURG_AUDIT_PAIRED | BURG_AUDIT_PAIRED_LAYOUT: the paired kernel's store
 * wave in a burg_sweep launch (ring of num_steps W + 2 W + 128 entries, every
 * state kept): the halves of paired diagonal s at entries origin + 2 s and
 * + 1 (ring_pos_paired), checked cell by cell against the extraction's
 * mapping; the retained states are 1 .. num_steps (state 0: the uploaded w0). */
#define BURG_AUDIT_PAIRED_LAYOUT 2
int burg_ring_audit_ex(int W, int num_steps, int snap_every, int ring_cap, int flags,
                       int64_t *report);

/* Create a context on HIP device `device` for an nx x ny grid (single GPU). */
int burg_ctx_create(int device, int nx, int ny, burg_ctx **out);

/* Multi-GPU (one process per GPU): this rank owns global rows
 * [row0, row0 + nrows) of an nx x ny_total grid (rank 0 the bottom slab).
 * The slabs exchange the one-way halo (north outflow of a slab's top row ->
 * south inflow of the next slab) through a ring each GPU reads or writes
 * directly while the time loop runs: by default in the consumer's device
 * memory, opened by the producer over IPC (stores cross xGMI); pinned POSIX
 * shared host memory when that is unavailable or BURG_HALO=host.  The rings
 * are found through POSIX shared-memory objects named from `halo_name` (the
 * same job-unique string on every rank, 1-64 chars).  This call creates the
 * ring this rank consumes; after EVERY rank has created its context (a host
 * barrier), call burg_slab_connect to attach the ring this rank produces
 * into, then (second barrier) burg_slab_verify, and run a third barrier
 * before the first launch.  world == 1 behaves as burg_ctx_create. */
int burg_ctx_create_slab(int device, int nx, int ny_total, int row0, int nrows,
                         int rank, int world, const char *halo_name, burg_ctx **out);
int burg_slab_connect(burg_ctx *ctx);
/* Consumer-side check of a device-memory halo ring (no-op on rank 0 and on
 * host rings): the producer's probe store, made over the link in
 * burg_slab_connect, must have arrived; if not, the boundary moves to the
 * pinned host ring on both sides (the producer adopts that at its first
 * launch, so a barrier must separate this call from any launch).  The
 * producer's own check (it reads the consumer's probe back) runs inside
 * burg_slab_connect.  Replaces nothing in the reference (its FOM is one
 * process); it guards the rows-slab halo of SURVEY.md section 8(e). */
int burg_slab_verify(burg_ctx *ctx);
/* Why a slab context's halo is not on a device ring ("" when it is, or for
 * world == 1); valid until the next call on the context. */
const char *burg_slab_halo_note(burg_ctx *ctx);
/* Where the halo rings live: *in_mode for the ring this rank consumes,
 * *out_mode for the one it produces into: 0 none (end rank), 1 pinned host
 * memory, 2 the consumer GPU's device memory (IPC). */
int burg_slab_halo_mode(burg_ctx *ctx, int *in_mode, int *out_mode);

void burg_ctx_destroy(burg_ctx *ctx);

/* Problem data, computed by the caller exactly as NumPy does in the reference
 * (GLOBAL arrays; a slab context picks its rows):
 *   inv_dx[nx]        = 1/dx_c              (make_ddx, C/hypernet2D.py:2414)
 *   inv_dy[ny_total]  = 1/dy_r
 *   src[nx]           = dt*0.02*exp(mu2*xc) (:2550)
 *   lbc[ny_total]     = 0.5*dt*mu1**2/dx[r] (:2553-2554, row-indexed quirk)
 * BURG_EINVAL unless dt > 0 and every dt/4 * inv_dx[c], dt/4 * inv_dy[r] is in
 * (0, 2^100) (the march's fast path relies on it; any physical grid and dt
 * are far inside).  */
int burg_set_problem(burg_ctx *ctx, const double *inv_dx, const double *inv_dy,
                     const double *src, const double *lbc, double dt);

/* Engine options.  tile_w: tile width in cells (64 or 128; tile height is the
 * 64-lane wavefront).  par_passes: block-Jacobi passes launched over all
 * tiles per step before the final pass (<= 0: default 3); the final pass
 * always finishes the step at the fixed point, so this only trades launches
 * against tail work.  tol: relative inflow change below which a tile is not
 * re-marched (0 = bitwise fixed point = the sequential march).
 * profile: 1 = time every march launch with HIP events (burg_stats). */
int burg_set_options(burg_ctx *ctx, int tile_w, int par_passes, double tol, int profile);

/* March engine selection.  engine: BURG_ENGINE_*.  stream_w: streaming tile
 * width, a power of two in [8, 4096] (0: automatic, the narrowest width whose
 * tile count fits tiles_target; the pipe engine takes 8 or 16).  tiles_target: wavefronts to aim for
 * (0: 1024 = one per SIMD of the MI355X).  The tile count is always capped by
 * what the device keeps resident at once (the engine needs every tile live). */
int burg_set_engine(burg_ctx *ctx, int engine, int stream_w, int tiles_target);

/* Parity hooks (whole-grid host arrays; single-GPU contexts only). */
int burg_residual(burg_ctx *ctx, const double *w, const double *wp, double *r,
                  double *norm_out);
int burg_jvp(burg_ctx *ctx, const double *w, const double *x, double *y);
/* The residual of a slab context's rows (inviscid_burgers_res2D_alt,
 * C/hypernet2D.py:2512-2570, restricted to global rows [row0, row0+nrows)):
 * w, wp are this slab's rows (2*nx*nrows, as burg_run's w0); the south
 * neighbour terms of the slab's first row come from halo_w / halo_wp =
 * [u row | v row] (2*nx doubles) of global row row0-1 of w and wp (both NULL
 * on the bottom slab, required above it).  r: 2*nx*nrows; sumsq (may be
 * NULL): the sum of squares of r (the caller sums over ranks for ||R||).
 * Each entry equals burg_residual's on the whole grid bit for bit; the halo
 * rows come from the rank below (finitedifference_amd/dist.py, a
 * torch.distributed send/recv).  Any context (world == 1: halos NULL). */
int burg_slab_residual(burg_ctx *ctx, const double *w, const double *wp, const double *halo_w,
                       const double *halo_wp, double *r, double *sumsq);
int burg_block_solve(burg_ctx *ctx, const double *w, const double *rhs, double *delta);

/* Time loop (inviscid_burgers_implicit2D).  w0: this context's rows of the
 * initial state (2*nx*nrows).  snaps: C-order host matrix with leading
 * dimension ld_snaps (>= num_steps/snap_every + 1); column j receives the
 * state after j*snap_every steps, rows as in w (u rows then v rows of this
 * context).  snaps may be NULL (no snapshots kept).  solver: burg_solver.
 * newton_max_its / newton_rtol: newton_raphson's max_its / relnorm_cutoff.
 * step_iters[num_steps] / step_rel[num_steps] (each may be NULL): per step,
 * the Newton update count and final ||R||/||R(wp)|| (newton solver; the
 * numbers newton_raphson prints, C/hypernet2D.py:1844), or the march passes
 * and 0.0 (march solver). */
int burg_run(burg_ctx *ctx, const double *w0, int num_steps, int solver,
             int newton_max_its, double newton_rtol, double *snaps,
             int64_t ld_snaps, int snap_every, burg_stats *stats,
             int32_t *step_iters, double *step_rel);

/* Device-resident stepping for benchmarks: upload once, advance, download.
 * burg_advance keeps the state in HBM (no host traffic) and waits for the
 * device before returning; stats->loop_ms is its device time. */
int burg_upload_state(burg_ctx *ctx, const double *w);
int burg_advance(burg_ctx *ctx, int num_steps, int solver, burg_stats *stats);
int burg_download_state(burg_ctx *ctx, double *w);

/* Roofline probe of the HBM-bound stencils: runs
 * kernel `which` (burg_kernel) `reps` times on device-resident operands (the
 * last uploaded state as w, the resident state as wp / x; results discarded)
 * and returns the mean device time per launch (HIP events on the context's
 * stream).  Algorithmic bytes per launch: 48 B per cell (read u, v and
 * up, vp / xu, xv; write two planes).  Single-GPU contexts; call
 * burg_upload_state first. */
int burg_kernel_bench(burg_ctx *ctx, int which, int reps, double *avg_ms);

/* One device-resident trajectory (the benchmark's unit of work; replaces the
 * time loop of inviscid_burgers_implicit2D, C/hypernet2D.py:72-131, with the
 * snapshot matrix kept in HBM instead of host memory, :89-90,126): num_steps
 * march steps in ONE launch from the last uploaded state (from_initial = 1,
 * kept on the device by burg_upload_state) or from the resident state (0),
 * the final state left resident.  The states kept in HBM (the snapshot
 * matrix, in the engine's ring layout; see burg_trajectory_retained):
 *   snap_every = 1: every state while the whole trajectory fits in 85 % of
 *     free HBM; a larger one (8192 x 2048 and up x 500 steps) gets a ring
 *     capped by free HBM that wraps inside the launch and keeps the last
 *     states only;
 *   snap_every = k >= 2: states 0, k, 2k, ..., floor(num_steps / k) k, in
 *     retained windows of the ring at no extra HBM traffic (pipe engine;
 *     narrow tiles with k < 1 + 64 / W keep every state, which must fit);
 *   snap_every <= 0: 1 when the whole trajectory fits, else 10.
 * Stream/pipe engines; stats->loop_ms is the launch's device time (HIP events
 * on the context's stream).  burg_trajectory(ctx, T, f, st) is
 * burg_trajectory_ex(ctx, T, 1, f, st). */
int burg_trajectory_ex(burg_ctx *ctx, int num_steps, int snap_every, int from_initial,
                       burg_stats *stats);
int burg_trajectory(burg_ctx *ctx, int num_steps, int from_initial, burg_stats *stats);
/* Allocate (or keep) everything burg_trajectory_ex(ctx, num_steps,
 * snap_every, ...) needs -- the tiling, the edge mailboxes and the HBM ring of
 * the trajectory (up to 85 % of free HBM; 134 GB for 500 steps of 4096^2) --
 * without launching.  Multi-GPU slab ranks call it before the barrier that
 * precedes their first launch, so no rank's first launch waits for a
 * neighbour's allocation. */
int burg_reserve_trajectory_ex(burg_ctx *ctx, int num_steps, int snap_every);
int burg_reserve_trajectory(burg_ctx *ctx, int num_steps);
/* What burg_trajectory_ex(ctx, num_steps, snap_every) would keep, without
 * allocating: the resolved snap_every (auto -> 1 or 10), the number of
 * retained states (-1: a capped ring, known after the run) and the ring's
 * minimum bytes (0 when capped; a windowed ring's working part then grows to
 * the memory budget). */
int burg_trajectory_plan(burg_ctx *ctx, int num_steps, int snap_every, int *snap_every_out,
                         int64_t *retained_states, int64_t *ring_bytes);
/* The states the last burg_trajectory_ex keeps resident: first_state,
 * first_state + stride, ... (count of them; state q = after q steps).
 * BURG_ESTATE when another run has since reused the ring. */
int burg_trajectory_retained(burg_ctx *ctx, int64_t *first_state, int64_t *count, int *stride);
/* Copy retained columns col0 .. col0 + ncols - 1 (column j = state
 * first_state + j * stride) into the C-order (2n x ld_out) matrix `out`, at
 * its columns 0 .. ncols - 1 -- the reference's snapshot layout
 * (C/hypernet2D.py:89-90,126).  out_on_device = 0: host memory;
 * 1: device memory of the context's GPU (e.g. for burg_pod_rsvd_device). */
int burg_trajectory_copy(burg_ctx *ctx, int64_t col0, int64_t ncols, double *out, int64_t ld_out,
                         int out_on_device);

/* Parameter sweep (the reference's snapshot generation over a set of mu,
 * e.g. C/run_prom.py:59-71 over get_snapshot_params, C/run_tests.py:38-49):
 * nmu trajectories of num_steps march steps each, all from the uploaded
 * initial state (burg_upload_state; the reference's w0 is the same for every
 * mu, C/run_fom.py:33-35), trajectory j with its own coefficients
 *   src_b[j*nx + c]        = dt*0.02*exp(mu2_j*xc)   (burg_set_problem's src)
 *   lbc_b[j*ny_total + r]  = 0.5*dt*mu1_j**2/dx[r]   (burg_set_problem's lbc)
 * (global arrays; a slab context picks its rows).  The trajectories run back
 * to back in ONE pipelined launch (as many as a third of free HBM holds per
 * launch), so the pipeline fills once per sweep, not once per trajectory.
 * Each trajectory is bit-identical to burg_run with that mu.
 * snaps: NULL (states stay in HBM, benchmark) or nmu host matrices, each
 * C-order with leading dimension ld_snaps, laid out as burg_run's.  The last
 * trajectory's final state becomes the resident state.  Pipe engine only. */
int burg_sweep(burg_ctx *ctx, int nmu, const double *src_b, const double *lbc_b, int num_steps,
               double *const *snaps, int64_t ld_snaps, int snap_every, burg_stats *stats);
/* The same sweep with the snapshot set left on the device: d_out is a
 * C-order (2n x ld_out) matrix in device memory of the context's GPU, and
 * trajectory j's num_steps / snap_every + 1 columns land at columns
 * j * (num_steps / snap_every + 1) ... -- np.hstack of the per-mu matrices,
 * the matrix C/run_prom.py:59-71 hands to POD (burg_pod_rsvd_device), with no
 * host round trip.  Small grids run several trajectories side by side in one
 * launch (either entry point). */
int burg_sweep_device(burg_ctx *ctx, int nmu, const double *src_b, const double *lbc_b,
                      int num_steps, int snap_every, double *d_out, int64_t ld_out,
                      burg_stats *stats);

/* One trajectory straight into a snapshot-cache file (load_or_compute_snaps'
 * compute-then-np.save, C/hypernet2D.py:3141-3143): the
 * march runs in one launch with every state kept in HBM, then the C-order
 * (2n x num_steps/snap_every+1) snapshot matrix is written to `path` in
 * np.save's .npy format, row blocks gathered on the device and copied into
 * two pinned host buffers that a writer thread drains while the next block
 * is copied.  stats: loop_ms = launch time, flush_ms = device time of the
 * gathers + D2H copies, march_kernel_ms = wall time of the whole call.
 * Single-trajectory rings only (BURG_ENOMEM when it does not fit in HBM). */
int burg_run_npy(burg_ctx *ctx, const double *w0, int num_steps, int snap_every, const char *path,
                 burg_stats *stats);

/* burg_run_npy with flags -- the multi-GPU form of load_or_compute_snaps'
 * cache write (C/hypernet2D.py:3141-3143, BurgersFD_CleanFine/run_fom.py:28
 * at 750^2 over 8 GPUs):
 *   BURG_NPY_GLOBAL: the file holds the WHOLE grid's (2 nx ny_total, ncols)
 *     matrix and this slab context writes its u rows at global rows
 *     [row0 nx, (row0 + nrows) nx) and its v rows at nx ny_total + the same
 *     (without BURG_NPY_EXISTING the file is created with that header and
 *     size);
 *   BURG_NPY_EXISTING: the file already exists with exactly that .npy header
 *     and at least its size (made by one rank, e.g. rank 0, before a barrier;
 *     BURG_EINVAL otherwise) -- it is neither truncated nor re-headed, so
 *     every rank writes its rows into the one file during the same call.
 * Every rank of a slab job calls this together (the march's halo streams
 * between the ranks' launches).  flags = 0 is burg_run_npy. */
#define BURG_NPY_GLOBAL 1
#define BURG_NPY_EXISTING 2
int burg_run_npy_ex(burg_ctx *ctx, const double *w0, int num_steps, int snap_every,
                    const char *path, int flags, burg_stats *stats);

/* ECSW hyper-reduction training matrix (compute_ECSW_training_matrix_2D,
 * C/hypernet2D.py:2719-2740), with the context's problem (grid, dt, mu of
 * burg_set_problem):
 *   C[isnap*n_pod + k, node] = R_u[node] W_u[node,k] + R_v[node] W_v[node,k],
 *   R = residual(states[isnap]; prev_states[isnap]), W = J(states[isnap]) basis.
 * states, prev_states: n_snaps states of 2n doubles each, state-major (the
 * columns of the reference's snapshot blocks, contiguous); basis: (2n x n_pod)
 * C-order (the reference's basis array); C: (n_pod*n_snaps x n) C-order
 * output, n = nx*ny.  stats (may be NULL): loop_ms = kernel time, flush_ms =
 * D2H time of C, steps = n_snaps.  Single-GPU contexts. */
int burg_ecsw_matrix(burg_ctx *ctx, int n_snaps, const double *states, const double *prev_states,
                     int n_pod, const double *basis, double *C, burg_stats *stats);

/* One snapshot's block of the ECSW training matrix with a per-snapshot
 * basis: the decoder variants (compute_ECSW_training_matrix_2D_rnm,
 * _rbf_nearest_neighbors, _rbf_global, _gp; C/hypernet2D.py:2742-3072)
 * refit a reconstruction w(y) per snapshot and assemble C from
 * R(w; prev) and J(w) V with V = dw/dy, a different basis per snapshot.
 * All arrays are DEVICE memory of the context's GPU (the decoder's products
 * live there; a host pointer is refused with BURG_EINVAL):
 *   d_state, d_prev: 2n doubles; d_basis_t: (n_pod x 2n) C-order (V^T: the
 *   columns of V contiguous); d_C: (n_pod x n) C-order output,
 *   d_C[k*n + node] = R_u[node] (J V)_u[node,k] + R_v[node] (J V)_v[node,k].
 * Stream-ordered on the context's stream and complete on return (callers
 * producing the inputs on another stream synchronise it first).
 * kernel_ms (may be NULL): the kernel's time.  Single-GPU contexts. */
int burg_ecsw_block_device(burg_ctx *ctx, const double *d_state, const double *d_prev,
                           int n_pod, const double *d_basis_t, double *d_C, float *kernel_ms);

/* LSPG PROM time loop (inviscid_burgers_implicit2D_LSPG, C/hypernet2D.py:133-200,
 * with gauss_newton_LSPG, :1859-1929), with the context's problem (grid, dt,
 * mu of burg_set_problem); square single-GPU contexts (the reference's
 * row-only JDyec permutation, :165-167, is defined for nx == ny only).
 *   y0 = basis^T w0, w = basis y0; per step: Gauss-Newton from the previous
 *   y, stopping at ||R||/||R(w at entry)|| < relnorm_cutoff, or when the
 *   relative change of ||R|| is below min_delta, or after max_its norms;
 *   each update solves min ||J(w) basis dy + R|| (normal equations,
 *   Cholesky; the reference: np.linalg.lstsq).
 * basis: (2n x n_pod) C-order, 1 <= n_pod <= 127.  snaps (NULL: not kept):
 * (2n x ld_snaps) C-order, column j = basis y_j (j = 0..num_steps);
 * red_coords (NULL: not kept): (n_pod x ld_red) C-order, column j = y_j;
 * step_its (NULL ok): per step, len(resnorms) of the reference (its printed
 * 'iteration i' + 1); step_rel (NULL ok): the printed relative norm.
 * times_ms (NULL ok): [0] fused J.basis + Gram kernel time, [1] residual
 * time, [2] solve + basis expansion time (HIP events; the reference's
 * jac_time, res_time, ls_time).  stats: steps, newton_updates = total
 * Gauss-Newton updates, loop_ms = wall time, flush_ms = snapshot D2H.
 * Returns BURG_ENOCONV when J basis is rank-deficient (Cholesky pivot <= 0). */
int burg_lspg(burg_ctx *ctx, const double *w0, int num_steps, int n_pod, const double *basis,
              int max_its, double relnorm_cutoff, double min_delta, double *snaps,
              int64_t ld_snaps, double *red_coords, int64_t ld_red, int32_t *step_its,
              double *step_rel, double *times_ms, burg_stats *stats);

/* POD of a snapshot matrix (POD, C/hypernet2D.py:2670-2695, as run_prom.py:58-86
 * calls it): the exact thin SVD S = U diag(sigma) V^T by Householder QR of S
 * and an SVD of its R factor (rocSOLVER dgeqrf / dgesvd / dormqr on the
 * device).  snaps: (m x ns) C-order host matrix, m >= ns; U: (m x k) C-order
 * host output, the k leading left singular vectors, each column's
 * largest-magnitude entry made positive (sklearn's svd_flip rule); sigma: k
 * singular values, descending.  1 <= k <= ns.  ms (may be NULL): device time
 * of the factorisation (HIP events).  No context: runs on `device`. */
int burg_pod(int device, int64_t m, int ns, const double *snaps, int k, double *U, double *sigma,
             double *ms);

/* Randomized truncated SVD, the algorithm of sklearn's randomized_svd that
 * POD(method='rsvd') calls (C/hypernet2D.py:2688-2692): Y = S omega, n_iter
 * power iterations (CholeskyQR3-normalised), Q = orth(Y), SVD of Q^T S.
 * omega: (ns x nrand) COLUMN-major host matrix (the caller's Gaussian draw,
 * nrand = k + oversamples, k <= nrand <= ns); other arguments as burg_pod.
 * nrand <= 128: the products with S run on the library's fp64 MFMA kernels
 * (S read in place) and the small SVD is a one-workgroup Jacobi; above, or
 * with BURG_POD_GEMM=rocblas, rocBLAS dgemm and rocSOLVER dgesvd. */
int burg_pod_rsvd(int device, int64_t m, int ns, const double *snaps, int k, int nrand, int n_iter,
                  const double *omega, double *U, double *sigma, double *ms);
/* burg_pod_rsvd (omega != NULL) or burg_pod (omega == NULL) on a snapshot
 * matrix that is already in device memory of `device` (C-order m x ns, e.g.
 * burg_sweep_device's): no upload.  U, sigma, omega are host arrays. */
int burg_pod_rsvd_device(int device, int64_t m, int ns, const double *d_snaps, int k, int nrand,
                         int n_iter, const double *omega, double *U, double *sigma, double *ms);

#ifdef __cplusplus
}
#endif

#endif /* BURGERS_H */
