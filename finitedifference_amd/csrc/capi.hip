// capi.hip -- C ABI (include/burgers.h) of libburgers_hip.so: contexts, the
// time loop (inviscid_burgers_implicit2D, C/hypernet2D.py:72-131) and the
// parity hooks.  Host-side only; kernels live in march.hip / stencil.hip.
#include <rocprofiler-sdk-roctx/roctx.h>
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <algorithm>
#include <climits>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../include/burgers.h"
#include "burg_internal.h"
#include "build_id.h"  // (the object directory's, -I$(B): Makefile)

using namespace burg;

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(expr)                                                                    \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(BURG_EHIP, "%s:%d %s: %s", __FILE__, __LINE__, #expr,           \
                        hipGetErrorString(e_));                                         \
    } while (0)

#define CHK(expr)                                                                       \
    do {                                                                                \
        int c_ = (expr);                                                                \
        if (c_ != 0) {                                                                  \
            if (c_ == -3)                                                               \
                return fail(BURG_EHIP, "%s:%d kernel launch %s: %s", __FILE__, __LINE__, \
                            #expr, hipGetErrorString(hipGetLastError()));               \
            return c_;                                                                  \
        }                                                                               \
    } while (0)

template <class T>
int dalloc(T **p, size_t count)
{
    *p = nullptr;
    if (count == 0) return 0;
    hipError_t e = hipMalloc((void **)p, count * sizeof(T));
    if (e != hipSuccess)
        return fail(BURG_ENOMEM, "hipMalloc(%zu bytes): %s", count * sizeof(T),
                    hipGetErrorString(e));
    return 0;
}

template <class T>
void dfree(T *&p)
{
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}

}  // namespace

// ROCTx ranges around the ABI entry points and the march launches
// (rocprofv3 --marker-trace shows them on the timeline; without a profiler
// attached they cost a call each).
struct TraceRange {
    explicit TraceRange(const char *name) { roctxRangePushA(name); }
    ~TraceRange() { roctxRangePop(); }
    TraceRange(const TraceRange &) = delete;
    TraceRange &operator=(const TraceRange &) = delete;
};
#define BURG_TRACE(name) TraceRange burg_trace_range_(name)

// The ring layout of a trajectory launch (ring_pos, burg_internal.h): a plain
// ring of L entries from `origin`, or (k >= 2) a working ring of L entries plus
// n retained windows of W + 64 entries from entry `base`; Lt entries per tile.
struct TrajMap {
    long long L = 0, origin = 0, Lt = 0, base = 0;
    int k = 0, n = 0;
};

// What the last burg_trajectory_ex left resident (burg_trajectory_retained):
// states first, first + stride, ... (count of them), read through `map`
// (state q of the trajectory is state q - state0 of the map's launch); with
// ret0 the trajectory's initial state is the copy d_ret0.
struct TrajRecord {
    bool valid = false;
    TrajMap map;
    int64_t T = 0, state0 = 0, first = 0, count = 0;
    int stride = 1;
    bool ret0 = false;
};

struct burg_ctx {
    int device = 0;
    int nx = 0, ny_total = 0, row0 = 0, nrows = 0;
    int rank = 0, world = 1;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;

    // problem (global arrays on device; cf views this slab's rows)
    bool have_problem = false;
    double dt = 0.0;
    double *d_inv_dx = nullptr, *d_inv_dy = nullptr, *d_src = nullptr, *d_lbc = nullptr;
    Coeffs cf{};

    // engine
    int tw = 64, par_passes_opt = 0, profile = 0;
    double tol = 0x1p-50;  // 4 ulp relative
    Engine eg{};
    int par_passes = 3;  // parallel passes before the final pass
    double *d_edges = nullptr;
    int *d_counters = nullptr;
    DevStats *d_stats = nullptr, *d_stats_solve = nullptr;

    // states (ping-pong) and scratch
    double *d_state[2] = {nullptr, nullptr};
    int cur = 0;
    double *d_w0 = nullptr;  // last uploaded state (burg_trajectory from_initial)
    // d_w0 uniform (every u equal, every v equal; bitwise) and its {u0, v0}
    // bits: the paired sweep kernel restarts its trajectories from that
    // constant (pipe_args, PipeArgs::w0c)
    bool w0_uni = false;
    unsigned w0c[4] = {0u, 0u, 0u, 0u};
    int last_play = 0;  // the last pipe launch wrote the paired sweep layout (ring_pos_paired)
    double *d_r = nullptr, *d_d = nullptr, *d_x = nullptr, *d_partials = nullptr,
           *d_sumsq = nullptr;
    int npartials = 0;
    std::vector<hipEvent_t> prof_ev;

    // streaming engine (stream.hip)
    int engine = BURG_ENGINE_STREAM;
    int stream_w_opt = 0, tiles_target_opt = 0;
    StreamPlan sp{};
    bool sp_ready = false, colc_ready = false;
    d2 *d_colc = nullptr, *d_boxes = nullptr, *d_ring = nullptr;
    size_t box16 = 0, ring_entries = 0;
    bool ring_maxed = false;  // the ring was sized to the free-memory limit
    unsigned *d_err = nullptr;
    StreamStats *d_sstats = nullptr;
    // pipe engine (pipe.hip): effective engine of march runs, workgroups per
    // strip, absolute step counter mod 2*kPipeR (mailbox sentinel colour)
    int eng_eff = BURG_ENGINE_STREAM;
    int nwj = 0, qbase = 0;
    // parameter sweep of the next pipe launch (burg_sweep): steps per
    // trajectory and the per-trajectory coefficient tables (0/nullptr: none)
    int sw_T = 0;
    const d2 *sw_colc = nullptr;
    const double *sw_lbc = nullptr;
    // one-trajectory override of the column table / inlet terms (wide-tile
    // sweeps run one launch per mu)
    const d2 *ov_colc = nullptr;
    const double *ov_lbc = nullptr;
    long long spin_ticks = 500000000LL;  // 5 s of s_memrealtime (100 MHz)
    // multi-GPU halo rings: the consumer's device memory
    // over IPC (mode 2), or pinned shared host memory (mode 1)
    std::string halo_name;
    void *halo_in_host = nullptr, *halo_out_host = nullptr;  // shm objects (ring + control page)
    d2 *halo_in_hostdev = nullptr, *halo_out_hostdev = nullptr;  // their device mappings
    d2 *halo_in_ring = nullptr;   // consumer: its device ring (uncached, exported)
    void *halo_out_ipc = nullptr;  // producer: the neighbour's device ring, opened
    d2 *halo_in_dev = nullptr, *halo_out_dev = nullptr;  // what the kernel uses
    int halo_in_mode = 0, halo_out_mode = 0;             // 0 unknown, 1 host, 2 device
    size_t halo_bytes = 0;
    bool halo_connected = false;
    bool slab_failed = false;        // a launch failed: refuse further launches (BURG_ESTATE)
    int64_t launches = 0;            // march launches of this context (test hook)
    int64_t paired_launches = 0;     // since stream_stats_begin: launches of the paired kernel
    // side-by-side domains (an internal sweep context, burg_sweep): bat_nd
    // domains of bat_ny_d rows, each padded to whole strips; per-domain column
    // tables bat_colc_stride apart (ov_colc)
    int bat_nd = 1, bat_ny_d = 0;
    size_t bat_colc_stride = 0;
    burg_ctx *bat_child = nullptr;  // the parent's cached side-by-side sweep context
    int bat_child_G = 0;
    double *d_halo_rows = nullptr;   // burg_slab_residual: the south halo rows of w, wp (4 nx)
    TrajRecord tr;                   // the last trajectory's resident states
    double *d_ret0 = nullptr;        // its initial state (retained windows: the working ring
                                     // overwrites it)
    bool halo_out_resolved = false;  // producer: took the consumer's verdict (first launch)
    std::string halo_note;           // why a device ring was not used
    // the last pipe launch's diagnostics (burg_stats ramp_ms / halo_wait_ms)
    double last_ramp_ms = 0.0, last_halo_wait_ms = -1.0;
    int64_t bounds_checks = 0, bounds_hits = 0;  // check_bounds calls / hits (lifetime)

    size_t m() const { return 2 * (size_t)nx * nrows; }
    size_t n() const { return (size_t)nx * nrows; }
};

namespace {

int engine_alloc(burg_ctx *c)
{
    dfree(c->d_edges);
    dfree(c->d_counters);
    const int nti = (c->nrows + kWave - 1) / kWave;
    const int ntj = (c->nx + c->tw - 1) / c->tw;
    const size_t nt = (size_t)nti * ntj;
    const size_t per_e = 2 * (size_t)kWave, per_n = 2 * (size_t)c->tw;
    const size_t total = nt * (2 * per_e + 2 * per_n + per_e + per_n);
    if (int e = dalloc(&c->d_edges, total)) return e;
    HIPCHK(hipMemsetAsync(c->d_edges, 0, total * sizeof(double), c->stream));
    double *p = c->d_edges;
    c->eg.eb[0] = p;
    p += nt * per_e;
    c->eg.eb[1] = p;
    p += nt * per_e;
    c->eg.nb[0] = p;
    p += nt * per_n;
    c->eg.nb[1] = p;
    p += nt * per_n;
    c->eg.wused = p;
    p += nt * per_e;
    c->eg.sused = p;
    c->eg.nti = nti;
    c->eg.ntj = ntj;
    c->eg.tw = c->tw;
    c->eg.tol = c->tol;
    c->eg.halo_flux = nullptr;
    c->eg.halo_wp = nullptr;
    const int bound = nti + ntj;  // #anti-diagonals + 1 passes always reach the fixed point
    c->eg.kbound = bound;
    c->par_passes = c->par_passes_opt > 0 ? std::min(c->par_passes_opt, bound - 1) : std::min(3, bound - 1);
    if (int e = dalloc(&c->d_counters, (size_t)bound + 3)) return e;
    HIPCHK(hipMemsetAsync(c->d_counters, 0, sizeof(int) * (bound + 3), c->stream));
    c->eg.ticket = c->d_counters + bound + 2;
    c->eg.counters = c->d_counters;
    return 0;
}

int ensure_scratch(burg_ctx *c)
{
    if (c->d_r) return 0;
    if (int e = dalloc(&c->d_r, c->m())) return e;
    if (int e = dalloc(&c->d_d, c->m())) return e;
    if (int e = dalloc(&c->d_x, c->m())) return e;
    c->npartials = residual_partials_count(c->cf);
    if (int e = dalloc(&c->d_partials, (size_t)c->npartials)) return e;
    if (int e = dalloc(&c->d_sumsq, 1)) return e;
    return 0;
}

int check_ready(burg_ctx *c)
{
    if (!c) return fail(BURG_EINVAL, "null context");
    if (!c->have_problem) return fail(BURG_ESTATE, "burg_set_problem has not been called");
    HIPCHK(hipSetDevice(c->device));
    return 0;
}

// One implicit step wp -> w by the march engine: P parallel passes + final.
int march_step(burg_ctx *c, const double *wp, double *w)
{
    const int P = c->par_passes;
    for (int k = 1; k <= P + 1; ++k) {
        hipEvent_t a = nullptr, b = nullptr;
        if (c->profile) {
            HIPCHK(hipEventCreate(&a));
            HIPCHK(hipEventCreate(&b));
            HIPCHK(hipEventRecord(a, c->stream));
        }
        CHK(launch_march_pass(c->cf, c->eg, wp, w, k, k == P + 1, c->d_stats, c->stream));
        if (c->profile) {
            HIPCHK(hipEventRecord(b, c->stream));
            c->prof_ev.push_back(a);
            c->prof_ev.push_back(b);
        }
    }
    return 0;
}

// Exact linear solve J(w) delta = rhs with the SOLVE cell.
int block_solve(burg_ctx *c, const double *w, const double *rhs, double *delta)
{
    if (c->tw != 64)
        return fail(BURG_EINVAL, "the exact block solve (newton solver) needs tile_w = 64");
    const int P = c->par_passes;
    for (int k = 1; k <= P + 1; ++k)
        CHK(launch_solve_pass(c->cf, c->eg, w, rhs, delta, k, k == P + 1, c->d_stats_solve,
                              c->stream));
    return 0;
}

int residual_norm(burg_ctx *c, const double *w, const double *wp, double *r, double *norm)
{
    CHK(launch_residual(c->cf, w, wp, r, c->d_partials, c->d_sumsq, nullptr, nullptr,
                        c->stream));
    double s = 0.0;
    HIPCHK(hipMemcpyAsync(&s, c->d_sumsq, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    *norm = std::sqrt(s);
    return 0;
}

// newton_raphson (C/hypernet2D.py:1811-1857) for one step, on the device:
// x = wp; init = ||R(wp)||; loop: rn = ||R(x)||; stop if rn/init < rtol;
// x -= J(x)^{-1} R(x).  Returns the number of updates.
int newton_step(burg_ctx *c, const double *wp, double *w, int max_its, double rtol,
                int *its_out, double *rel_out)
{
    HIPCHK(hipMemcpyAsync(w, wp, c->m() * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    double init = 0.0, rn = 0.0, rel = NAN;
    if (int e = residual_norm(c, wp, wp, c->d_r, &init)) return e;
    int it = 0;
    for (it = 0; it < max_its; ++it) {
        if (int e = residual_norm(c, w, wp, c->d_r, &rn)) return e;
        rel = rn / init;
        if (!std::isfinite(rn)) return fail(BURG_ENAN, "non-finite residual norm in Newton");
        if (rel < rtol) break;
        if (int e = block_solve(c, w, c->d_r, c->d_d)) return e;
        CHK(launch_axpy_neg(w, c->d_d, c->m(), c->stream));
    }
    *its_out = it;
    *rel_out = rel;
    return 0;
}

void collect_profile(burg_ctx *c, burg_stats *st)
{
    if (c->prof_ev.empty()) return;
    (void)hipStreamSynchronize(c->stream);
    double ms = 0.0;
    for (size_t i = 0; i + 1 < c->prof_ev.size(); i += 2) {
        float t = 0.f;
        (void)hipEventElapsedTime(&t, c->prof_ev[i], c->prof_ev[i + 1]);
        ms += t;
        (void)hipEventDestroy(c->prof_ev[i]);
        (void)hipEventDestroy(c->prof_ev[i + 1]);
    }
    if (st) {
        st->march_kernel_ms += ms;
        st->march_launches += (int64_t)(c->prof_ev.size() / 2);
    }
    c->prof_ev.clear();
}

int read_stats(burg_ctx *c, burg_stats *st)
{
    DevStats ds{};
    HIPCHK(hipMemcpyAsync(&ds, c->d_stats, sizeof ds, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (st) {
        st->steps = ds.steps;
        st->tile_marches = ds.tile_marches;
        st->passes = ds.passes;
        st->max_passes = ds.max_passes;
        st->unconverged_steps = ds.unconverged_steps;
        st->tail_passes = ds.tail_passes;
        st->par_passes = c->par_passes;
        st->engine = BURG_ENGINE_TILES;
    }
    return 0;
}

int halo_resolve_in(burg_ctx *c);  // multi-GPU halo rings (below)
void halo_resolve_out(burg_ctx *c);

// ---- streaming engine -------------------------------------------------------
void stream_free(burg_ctx *c)
{
    dfree(c->d_colc);
    dfree(c->d_boxes);
    dfree(c->d_ring);
    dfree(c->d_err);
    dfree(c->d_sstats);
    c->ring_entries = 0;
    c->ring_maxed = false;
    c->sp_ready = c->colc_ready = false;
    c->tr.valid = false;  // the ring it described is gone
}

// err[5] of the context: the flat-pointer ring / transpose kernels' bounds
// flag (stream.hip ring_ok / out_ok, stencil.hip transpose_kernel)
unsigned *bflag(burg_ctx *c) { return c->d_err ? c->d_err + 5 : nullptr; }

// after a copy: did a bounds guard fire?  (the stream is synchronised)
int check_bounds(burg_ctx *c, const char *where)
{
    if (!c->d_err) return 0;
    unsigned f = 0;
    HIPCHK(hipMemcpyAsync(&f, c->d_err + 5, sizeof f, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    ++c->bounds_checks;
    if (!f) return 0;
    ++c->bounds_hits;
    (void)hipMemsetAsync(c->d_err + 5, 0, sizeof f, c->stream);
    (void)hipStreamSynchronize(c->stream);
    return fail(BURG_EHIP, "%s: internal bounds check failed (%s%s): a library bug -- please "
                "report the grid, tile width and snap_every", where,
                (f & 1) ? "ring entry outside the tile's ring" : "",
                (f & 2) ? ((f & 1) ? ", output index past the buffer" : "output index past the buffer")
                        : "");
}

// Pipe engine plan: the narrowest W in {8, 16, ..., 1024} whose tile count
// fits the target, every workgroup (4 tiles + comm wave, + loader wave for
// wide tiles) resident at once; W <= 16 keeps the previous states in LDS,
// wider tiles stream them from the HBM ring (pipe.hip).  Target (target <= 0:
// automatic): narrow tiles 1024 (one compute wave per SIMD); wide tiles as
// many as there are resident compute-wave slots (two per SIMD for W = 64,
// 128).
bool pipe_plan(burg_ctx *c, int target, StreamPlan *out, int *nwj)
{
    std::vector<int> Ws;
    if (c->stream_w_opt != 0) {
        if (!pipe_width_supported(c->stream_w_opt)) return false;
        Ws.push_back(c->stream_w_opt);
    } else {
        for (int W = 8; W <= 1024; W *= 2) Ws.push_back(W);
    }
    int fit = -1;
    StreamPlan pf{};
    int wf = 0;
    for (int W : Ws) {
        StreamPlan p = plan_stream(c->nx, c->nrows, 0, W);
        const int wj = (p.ntj + 3) / 4;
        const int cap = pipe_max_resident_blocks(W);
        if (cap < 0) return false;
        if (p.nti * wj > cap) continue;
        p.R = kPipeR;
        if (fit < 0) {
            fit = W;
            pf = p;
            wf = wj;
        }
        const int tgt = target > 0 ? target : W <= 16 ? 1024 : 4 * cap;
        if (p.ntiles <= tgt) {
            *out = p;
            *nwj = wj;
            return true;
        }
    }
    if (fit < 0) return false;
    *out = pf;
    *nwj = wf;
    return true;
}

// Plan the tiling (capped by residency: every tile's wavefront must be live
// at once), allocate the mailboxes (all sentinel) and the column table.
int stream_setup(burg_ctx *c)
{
    if (!c->sp_ready) {
        const int target = c->tiles_target_opt > 0 ? c->tiles_target_opt : 1024;
        StreamPlan pp{};
        int wj = 0;
        if (c->engine == BURG_ENGINE_PIPE && pipe_plan(c, c->tiles_target_opt, &pp, &wj)) {
            c->sp = pp;
            c->nwj = wj;
            c->eng_eff = BURG_ENGINE_PIPE;
            c->box16 = (size_t)pp.ntiles * kPipeR * (kWave + pp.W) * (kPipeGranuleStride / sizeof(d2));
            if (c->box16 * sizeof(d2) >= (1ull << 31))
                return fail(BURG_ESHAPE, "edge mailboxes exceed 2 GiB");
            if (int e = dalloc(&c->d_boxes, c->box16)) return e;
            if (int e = dalloc(&c->d_colc, (size_t)pp.ntj * pp.W)) return e;
            if (int e = dalloc(&c->d_err, 8)) return e;
            if (int e = dalloc(&c->d_sstats, 1)) return e;
            CHK(launch_pipe_fill(c->d_boxes, c->box16, 0, c->stream));
            HIPCHK(hipMemsetAsync(c->d_err, 0, 8 * sizeof(unsigned), c->stream));
            c->qbase = 0;
            c->sp_ready = true;
            c->colc_ready = false;
        } else {
            if (c->world > 1)
                return fail(BURG_ESHAPE,
                            "multi-GPU slabs need the pipe engine: a %d-row x %d slab does not fit "
                            "one resident workgroup per 4 tiles of width <= 1024",
                            c->nrows, c->nx);
            StreamPlan p = plan_stream(c->nx, c->nrows, target,
                                       c->engine == BURG_ENGINE_PIPE ? 0 : c->stream_w_opt);
            for (;;) {
                if (!stream_width_supported(p.W))
                    return fail(BURG_EINVAL, "stream tile width %d not supported (8..4096, power of 2)",
                                p.W);
                int per_cu = 0, cus = 0;
                const int cap = stream_max_resident_blocks(p.W, &per_cu, &cus);
                if (cap < 0) return fail(BURG_EHIP, "occupancy query failed");
                if (p.ntiles <= 4 * cap) break;
                if ((c->engine == BURG_ENGINE_STREAM && c->stream_w_opt > 0) || p.W >= 4096)
                    return fail(BURG_ESHAPE, "%d tiles of width %d exceed the %d resident wavefronts",
                                p.ntiles, p.W, 4 * cap);
                p = plan_stream(c->nx, c->nrows, 0, p.W * 2);
            }
            c->sp = p;
            c->eng_eff = BURG_ENGINE_STREAM;
            c->box16 = (size_t)p.ntiles * p.R * (kWave + p.W) * (kGranuleStride / sizeof(d2));
            if (c->box16 * sizeof(d2) >= (1ull << 31))
                return fail(BURG_ESHAPE, "edge mailboxes exceed 2 GiB (%d tiles of width %d)",
                            p.ntiles, p.W);
            if (int e = dalloc(&c->d_boxes, c->box16)) return e;
            if (int e = dalloc(&c->d_colc, (size_t)p.ntj * p.W)) return e;
            if (int e = dalloc(&c->d_err, 8)) return e;
            if (int e = dalloc(&c->d_sstats, 1)) return e;
            CHK(launch_fill_sentinel(c->d_boxes, c->box16, c->stream));
            HIPCHK(hipMemsetAsync(c->d_err, 0, 8 * sizeof(unsigned), c->stream));
            c->sp_ready = true;
            c->colc_ready = false;
        }
    }
    if (c->world > 1 && !c->halo_connected)
        return fail(BURG_ESTATE, "slab context not connected (burg_slab_connect) to its neighbours");
    if (c->world > 1) {
        CHK(halo_resolve_in(c));
        halo_resolve_out(c);
    }
    if (!c->colc_ready) {
        CHK(launch_colc(c->cf, c->sp.ntj * c->sp.W, c->d_colc, c->stream));
        c->colc_ready = true;
    }
    return 0;
}

int ensure_ring(burg_ctx *c, long long L)
{
    c->tr.valid = false;  // the caller overwrites the ring
    const size_t need = (size_t)c->sp.ntiles * (size_t)L * kWave;
    if (need <= c->ring_entries) return 0;
    dfree(c->d_ring);
    c->ring_entries = 0;
    c->ring_maxed = false;  // a ring sized for L, not to the memory limit
    if (int e = dalloc(&c->d_ring, need)) return e;
    c->ring_entries = need;
    return 0;
}

StreamArgs stream_args(burg_ctx *c, long long L, long long origin, int K, const TrajMap *mp = nullptr)
{
    StreamArgs a{};
    a.Lt = (mp && mp->Lt >= L) ? mp->Lt : L;
    if (mp && mp->k > 0) {
        a.ret_k = mp->k;
        a.ret_n = mp->n;
        a.ret_base = mp->base;
    }
    a.cf = c->cf;
    a.colc = c->d_colc;
    a.ring = c->d_ring;
    a.wbox = c->d_boxes;
    a.sbox = c->d_boxes + (size_t)c->sp.ntiles * c->sp.R * kWave * (kGranuleStride / sizeof(d2));
    a.wbox_bytes = (size_t)c->sp.ntiles * c->sp.R * kWave * kGranuleStride;
    a.sbox_bytes = (size_t)c->sp.ntiles * c->sp.R * c->sp.W * kGranuleStride;
    a.origin = origin;
    a.L = L;
    a.K = K;
    a.nti = c->sp.nti;
    a.ntj = c->sp.ntj;
    a.ntiles = c->sp.ntiles;
    a.R = c->sp.R;
    a.err = c->d_err;
    a.stats = c->d_sstats;
    if (const char *e = std::getenv("BURG_STREAM_DEBUG")) a.flags = std::atoi(e);  // diagnostics
    return a;
}

// max steps per launch: a tile's ring (L = K*W + W + 96 entries of 1 KB) must
// stay addressable by one buffer descriptor (< 2 GiB)
int stream_max_steps(const burg_ctx *c) { return ((1 << 21) - 4096) / c->sp.W - 1; }

PipeArgs pipe_args(burg_ctx *c, long long L, long long origin, int K, const TrajMap *mp = nullptr)
{
    PipeArgs a{};
    a.Lt = (mp && mp->Lt >= L) ? mp->Lt : L;
    if (mp && mp->k > 0) {
        a.ret_k = mp->k;
        a.ret_n = mp->n;
        a.ret_base = mp->base;
    }
    a.cf = c->cf;
    a.colc = c->d_colc;
    a.ring = c->d_ring;
    a.wbox = c->d_boxes;
    a.sbox = c->d_boxes + (size_t)c->sp.ntiles * kPipeR * kWave * (kPipeGranuleStride / sizeof(d2));
    a.wbox_bytes = (size_t)c->sp.ntiles * kPipeR * kWave * kPipeGranuleStride;
    a.sbox_bytes = (size_t)c->sp.ntiles * kPipeR * c->sp.W * kPipeGranuleStride;
    a.halo_in = c->halo_in_dev;
    a.halo_out = c->halo_out_dev;
    a.halo_bytes = c->halo_bytes;
    a.origin = origin;
    a.L = L;
    a.K = K;
    a.T = c->sw_T > 0 ? c->sw_T : K;
    a.colc_b = c->sw_T > 0 ? c->sw_colc : nullptr;
    a.lbc_b = c->sw_T > 0 ? c->sw_lbc : nullptr;
    a.qbase = c->qbase;
    a.nti = c->sp.nti;
    a.ntj = c->sp.ntj;
    a.ntiles = c->sp.ntiles;
    a.nwj = c->nwj;
    a.nd = 1;
    a.nti_d = c->sp.nti;
    a.ny_d = c->nrows;
    a.colc_dstride = 0;
    if (c->bat_nd > 1) {
        a.nd = c->bat_nd;
        a.nti_d = c->sp.nti / c->bat_nd;
        a.ny_d = c->bat_ny_d;
        a.colc_dstride = c->bat_colc_stride;
    }
    {
        // Column-major workgroup order where row-major would give each XCD
        // (the dispatcher deals workgroup i to XCD i mod 8) whole column groups
        // of tiles (nwj a multiple of 8): 8192 x 2048 slab 146 -> 169,
        // 16384 x 2048 137 -> 152 Gcell-updates/s, 1024^2 sweep / trajectory
        // +0.8 / +1.5 %; 4096^2 (nwj = 4) 0.4 % slower that way
        // (profiles/r03/ab/wg_order.txt).  BURG_WG_MAP=0/1 forces an order.
        const char *e = std::getenv("BURG_WG_MAP");
        a.wg_cm = e ? (std::atoi(e) != 0) : (c->nwj % 8 == 0);
    }
    // Paired halves (pipe.hip PAIR): the W = 16 kernel
    // marches the tile's two 8-column halves in the same lanes, one step
    // apart -- the per-diagonal control is shared by two cells (97.8 instead
    // of 108 instructions per cell), but a launch has half the diagonals for
    // the same pipeline fill (nx + ny diagonals).  So: on for sweeps (the
    // 1024^2 9-mu sweep 149 -> 172 Gcell-updates/s) and for trajectories
    // long enough to amortise the fill (K >= (nx + rows) / 2; the 1024^2 x
    // 500 trajectory stays one-cell: 110 vs 104, profiles/r05/ab/pair).
    // Plain rings only.  BURG_PAIR=0 / 1 forces it off / on (2: on without
    // its steady blocks, diagnostics).
    {
        const char *e = std::getenv("BURG_PAIR");
        int pair_opt = (e && *e) ? std::atoi(e) : -1;  // (set but empty: the default)
        if (pair_opt < 0) pair_opt = (a.T < K || 2LL * K >= (long long)c->nx + c->nrows) ? 1 : 0;
        a.pair = (pair_opt == 1 || pair_opt == 2) && c->sp.W == 16 && a.ret_k == 0 ? pair_opt : 0;
        // the paired sweep kernel (with its store wave) restarts trajectories
        // from a uniform initial state only -- the reference's w0 = 1
        // (C/run_fom.py:33-35); any other initial state sweeps one-cell
        if (a.pair && a.colc_b && a.T < K && pipe_pair_sweep_uniform_only() && !c->w0_uni) a.pair = 0;
        std::memcpy(a.w0c, c->w0c, sizeof a.w0c);
        // paired sweeps with a store wave write the paired layout
        // (ring_pos_paired: contiguous 1 KB entries; the sweep's extraction
        // reads it); BURG_PAIR_LAYOUT=0 keeps the standard one (A/B)
        const char *pl = std::getenv("BURG_PAIR_LAYOUT");
        a.play = (a.pair && a.colc_b && pipe_pair_sweep_uniform_only() && !(pl && *pl && std::atoi(pl) == 0)) ? 1 : 0;
    }
    a.spin_ticks = c->spin_ticks;
    a.census_ticks = std::min<long long>(c->spin_ticks, 100000000LL);  // <= 1 s
    a.err = c->d_err;
    a.census = c->d_err + 4;

    a.stats = c->d_sstats;
    if (c->ov_colc) a.colc = c->ov_colc;
    if (c->ov_lbc) a.cf.lbc = c->ov_lbc;
    return a;
}

int stream_launch(burg_ctx *c, long long L, long long origin, int K, float *ms,
                  const TrajMap *mp = nullptr)
{
    BURG_TRACE("march launch");
    const bool pipe = c->eng_eff == BURG_ENGINE_PIPE;
    if (c->slab_failed)
        return fail(BURG_ESTATE, "a launch of this slab context failed earlier: its halo rings hold "
                                 "stale step colours, so every rank must destroy and recreate its "
                                 "context");
    // test hook: a launch with a device-memory halo ring fails as a stalled
    // halo wait would, without launching -- exercises the bench's fall-back to
    // the host rings (tools/gpu_round.sh).  BURG_TEST_FAIL_DEVICE_HALO=1: every
    // such launch; =R:K: only rank R's launch number K (0-based, counted per
    // context) -- the other ranks then meet a neighbour that stopped, and
    // their bounded waits give up on their own (tools/gpu_r4.sh rehearsal)
    const int64_t launch_no = c->launches++;
    if (const char *e = std::getenv("BURG_TEST_FAIL_DEVICE_HALO")) {
        int hr = -1;
        long long hk = -1;
        const bool all = std::strcmp(e, "1") == 0;
        const bool one = !all && std::sscanf(e, "%d:%lld", &hr, &hk) == 2 && hr == c->rank &&
                         hk == launch_no;
        if ((all || one) && (c->halo_in_mode == 2 || c->halo_out_mode == 2)) {
            c->slab_failed = true;
            return fail(BURG_EHIP, "pipe engine: a wait timed out (test hook "
                                   "BURG_TEST_FAIL_DEVICE_HALO=%s: device halo ring)", e);
        }
    }
    // Every failure return from here on leaves a slab's halo rings (shared
    // with its neighbours) in an unknown colour state: a world > 1 context
    // then refuses further launches (not only on the kernel's own
    // error word, also on a failed launch, event or copy)
    struct SlabFailGuard {
        burg_ctx *c;
        bool ok = false;
        ~SlabFailGuard()
        {
            if (!ok && c->world > 1) c->slab_failed = true;
        }
    } guard{c};
    if (pipe) {
        // the launch diagnostics' timers: t_entry, t_halo_first start at ~0
        // (atomicMin), t_first_max at 0 (atomicMax)
        HIPCHK(hipMemsetAsync(&c->d_sstats->t_entry, 0xFF, 2 * sizeof(unsigned long long), c->stream));
        HIPCHK(hipMemsetAsync(&c->d_sstats->t_first_max, 0, sizeof(unsigned long long), c->stream));
    }
    HIPCHK(hipEventRecord(c->ev0, c->stream));
    if (pipe) {
        const PipeArgs pa = pipe_args(c, L, origin, K, mp);
        c->last_play = pa.play;
        CHK(launch_pipe(pa, c->sp.W, c->stream));
        if (pa.pair) ++c->paired_launches;
    } else {
        if (mp && mp->k > 0) return fail(BURG_EINVAL, "retained windows need the pipe engine");
        CHK(launch_stream(stream_args(c, L, origin, K), c->sp.W, c->stream));
    }
    HIPCHK(hipEventRecord(c->ev1, c->stream));
    HIPCHK(hipEventSynchronize(c->ev1));
    float t = 0.f;
    HIPCHK(hipEventElapsedTime(&t, c->ev0, c->ev1));
    *ms += t;
    unsigned err[4] = {0, 0, 0, 0};
    HIPCHK(hipMemcpy(err, c->d_err, sizeof err, hipMemcpyDeviceToHost));
    if (err[0]) {
        // a slab's halo rings (shared with its neighbours) cannot be reset by
        // one rank alone: the context refuses further launches (the guard)
        // leave the mailboxes clean for the next launch
        (void)hipMemsetAsync(c->d_err, 0, sizeof err, c->stream);
        if (pipe) {
            (void)launch_pipe_fill(c->d_boxes, c->box16, 0, c->stream);
            c->qbase = 0;
        } else {
            (void)launch_fill_sentinel(c->d_boxes, c->box16, c->stream);
        }
        (void)hipStreamSynchronize(c->stream);
        if (pipe && err[3] == 64u)
            return fail(BURG_EHIP,
                        "pipe engine: only %u of %d workgroups became resident together (W=%d); "
                        "the pipeline needs the whole grid on the GPU at once -- another kernel "
                        "or process holds CUs",
                        err[2], c->sp.nti * c->nwj, c->sp.W);
        if (pipe)
            return fail(BURG_EHIP,
                        "pipe engine: a wait timed out (workgroup tile %u of %d, step/diagonal %u, "
                        "wait %#x [16: comm wave: 1 south 2 west 4 north-grant 8 east-grant; 32: "
                        "compute wave, missing (>> 8): 1 west 2 south 4 east-LDS 8 east-grant "
                        "16 north-grant 32 state window; 128: loader, >> 8 which one -- tile = "
                        "its first compute wave's, step = that wave's filled diagonals], "
                        "K=%d W=%d%s)",
                        err[1], c->sp.ntiles, err[2], err[3], K, c->sp.W,
                        c->world > 1 ? "; multi-GPU: a neighbour rank may not be running" : "");
        return fail(BURG_EHIP,
                    "streaming engine: an edge wait timed out (tile %u of %d, diagonal %u, "
                    "edges %u [1 west 2 south 4 east 8 north], K=%d W=%d)",
                    err[1], c->sp.ntiles, err[2], err[3], K, c->sp.W);
    }
    if (pipe) {
        c->qbase = (int)((c->qbase + (long long)K) % (2 * kPipeR));
        unsigned long long tm[3] = {0, 0, 0};  // t_entry, t_halo_first, t_first_max
        HIPCHK(hipMemcpy(tm, &c->d_sstats->t_entry, sizeof tm, hipMemcpyDeviceToHost));
        const unsigned long long none = ~0ull;
        c->last_ramp_ms = (tm[0] != none && tm[2] >= tm[0]) ? (double)(tm[2] - tm[0]) / 1e5 : 0.0;
        c->last_halo_wait_ms = (tm[0] != none && tm[1] != none && tm[1] >= tm[0])
                                   ? (double)(tm[1] - tm[0]) / 1e5
                                   : -1.0;
    }
    guard.ok = true;
    return 0;
}

void stream_stats_begin(burg_ctx *c)
{
    c->paired_launches = 0;
    (void)hipMemsetAsync(c->d_sstats, 0, sizeof(StreamStats), c->stream);
}

int stream_stats_end(burg_ctx *c, burg_stats *st, int64_t steps, int64_t launches)
{
    StreamStats ss{};
    HIPCHK(hipMemcpyAsync(&ss, c->d_sstats, sizeof ss, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (st) {
        st->steps = steps;
        st->tile_marches = (int64_t)ss.tile_steps;
        st->passes = steps;
        st->max_passes = steps > 0 ? 1 : 0;
        st->unconverged_steps = 0;
        st->engine = c->eng_eff;
        st->stream_w = c->sp.W;
        st->stream_tiles = c->sp.ntiles;
        st->stall_spins = (int64_t)ss.stall_spins;
        st->slow_diagonals = (int64_t)ss.slow_diagonals;
        if (const char *e = std::getenv("BURG_STREAM_DEBUG"))  // diagnostics
            if (std::atoi(e) & 8)
                std::fprintf(stderr,
                             c->eng_eff == BURG_ENGINE_PIPE
                                 ? "[pipe] blocks that waited, by missing kind: east %llu north %llu "
                                   "west %llu south %llu window / store wave %llu; comm polls %llu\n"
                                 : "[stream] slow-path causes: east-busy %llu north-busy %llu "
                                   "west-unwritten %llu south-unwritten %llu range %llu repoll %llu\n",
                             ss.why[0], ss.why[1], ss.why[2], ss.why[3], ss.why[4], ss.why[5]);
        if (const char *e = std::getenv("BURG_STREAM_DEBUG"))
            if ((std::atoi(e) & 8) && ss.prof[0])
                std::fprintf(stderr, "[pipe] compute-wave clocks: loop %llu, store waits %llu (%.1f%%), "
                                     "readiness waits %llu (%.1f%%)\n",
                             ss.prof[0], ss.prof[1], 100.0 * ss.prof[1] / ss.prof[0], ss.prof[2],
                             100.0 * ss.prof[2] / ss.prof[0]);
        if (const char *e = std::getenv("BURG_STREAM_DEBUG"))
            if ((std::atoi(e) & 8) && ss.prof[0])
                std::fprintf(stderr, "[pipe] readiness waits by compute wave: %.1f%% %.1f%% %.1f%% %.1f%%\n",
                             400.0 * ss.prof[4] / ss.prof[0], 400.0 * ss.prof[5] / ss.prof[0],
                             400.0 * ss.prof[6] / ss.prof[0], 400.0 * ss.prof[7] / ss.prof[0]);
        st->slow_ticks = (int64_t)ss.slow_ticks;
        st->stream_launches = launches;
        st->ieee_diagonals = (int64_t)ss.ieee_diagonals;
        st->comm_polls = c->eng_eff == BURG_ENGINE_PIPE ? (int64_t)ss.why[5] : 0;
        st->nonfinite_diagonals = (int64_t)ss.nonfinite_diagonals;
        st->paired_launches = c->paired_launches;
        if (c->eng_eff == BURG_ENGINE_PIPE) {
            // (s_memrealtime: 100 MHz)
            st->ramp_ms = c->last_ramp_ms;
            st->halo_wait_ms = c->last_halo_wait_ms;
            st->south_waits_local = (int64_t)ss.south_blocks[0];
            st->south_waits_halo = (int64_t)ss.south_blocks[1];
            st->south_wait_ms_local = (double)ss.south_rt[0] / 1e5;
            st->south_wait_ms_halo = (double)ss.south_rt[1] / 1e5;
        } else {
            st->halo_wait_ms = -1.0;
        }
        st->bounds_checks = c->bounds_checks;
        st->bounds_hits = c->bounds_hits;
    }
    if (ss.nonfinite_diagonals && !std::getenv("BURG_ALLOW_NONFINITE"))  // (diagnostics knob)
        return fail(BURG_ENAN,
                    "the march produced non-finite states (NaN/Inf) on %llu diagonals: a NaN/Inf "
                    "input or a negative discriminant 0.25 + hx*Cu + hy*Cv",
                    (unsigned long long)ss.nonfinite_diagonals);
    return 0;
}

// advance the device state d_state[cur] by num_steps with the streaming engine
int stream_advance(burg_ctx *c, int num_steps, burg_stats *st)
{
    if (int e = stream_setup(c)) return e;
    const int W = c->sp.W;
    const long long L = 2LL * W + 32;
    if (int e = ensure_ring(c, L)) return e;
    stream_stats_begin(c);
    CHK(launch_ring_load(stream_args(c, L, 0, 0), W, c->d_state[c->cur], c->stream));
    float ms = 0.f;
    long long origin = 0;
    int done = 0, last = 0;
    int64_t launches = 0;
    while (done < num_steps) {
        const int K = std::min(num_steps - done, stream_max_steps(c));
        if (int e = stream_launch(c, L, origin, K, &ms)) return e;
        origin = (origin + (long long)K * W) % L;
        done += K;
        last = K;
        ++launches;
    }
    if (num_steps > 0) {
        // the final state is state `last` of the last launch (origin before it)
        const long long o_last = ((origin - (long long)last * W) % L + L) % L;
        CHK(launch_ring_extract(stream_args(c, L, o_last, 0), W, last, 1, 1,
                                c->d_state[c->cur ^ 1], 1, c->m(), c->stream));
        c->cur ^= 1;
    }
    if (int e = check_bounds(c, "stream_advance")) return e;
    if (int e = stream_stats_end(c, st, num_steps, launches)) return e;
    if (st) {
        st->loop_ms = ms;
        if (c->profile) {
            st->march_kernel_ms = ms;
            st->march_launches = launches;
        }
    }
    return 0;
}

// Entries per tile of a trajectory ring of L entries (the tile stride): the
// HBM channel a ring entry lands on follows its address, and all tiles
// write the same ring position at about the same time -- a stride that is a
// multiple of a large power of two (a retained-window ring: Lw + n (W + 64) =
// 2^8 x odd KB at 16384 x 2048) puts every tile's stream on the same
// channels.  Default: an odd number of entries (1 KB each).  BURG_RING_PAD=n
// (A/B knob): exactly n extra entries.
long long ring_stride(long long L)
{
    static long long pad = -2;
    if (pad == -2) {
        pad = -1;
        if (const char *e = std::getenv("BURG_RING_PAD")) pad = std::atoll(e);
    }
    if (pad >= 0) return L + pad;
    return L | 1;
}

// The trajectory ring for num_steps: C steps per launch, L entries.  A ring
// already sized to the memory limit is reused as it is: the next call would
// only get the same size back, after a free and a fresh allocation of up to
// ~240 GB (seconds per call at 8192^2).
int plain_ring(burg_ctx *c, int num_steps, long long *C_out, long long *L_out)
{
    const int W = c->sp.W;
    const size_t per_entry = (size_t)c->sp.ntiles * kWave * sizeof(d2);
    long long C = std::min(num_steps, stream_max_steps(c));
    if (const char *e = std::getenv("BURG_STREAM_CHUNK")) {  // test knob: force chunking
        const long long v = std::atoll(e);
        if (v > 0) C = std::min(C, v);
    }
    if (const char *e = std::getenv("BURG_RING_CAP")) {  // test knob: a ring of at most v steps
        const long long v = std::atoll(e);
        if (v > 0) C = std::min(C, v);
    }
    const long long have_L = (long long)(c->ring_entries / (c->sp.ntiles * (size_t)kWave));
    bool maxed = false;
    const long long pad = ring_stride(0);  // (at most this many entries of stride padding)
    if (ring_stride(C * W + W + 96) > have_L && !(c->ring_maxed && have_L >= 2 * W + 96 + pad)) {
        // need a (bigger) ring: size it against free memory
        dfree(c->d_ring);
        c->ring_entries = 0;
        size_t freeb = 0, totalb = 0;
        HIPCHK(hipMemGetInfo(&freeb, &totalb));
        const long long Lmax = (long long)(freeb / 100 * 85 / per_entry) - pad;
        const long long Cmem = (Lmax - W - 96) / W;
        maxed = Cmem < C;
        C = std::min<long long>(C, Cmem);
        if (C < 1) return fail(BURG_ENOMEM, "not enough device memory for a one-step ring");
    } else {
        C = std::min<long long>(C, (have_L - pad - W - 96) / W);
        maxed = c->ring_maxed;
    }
    const long long L = C * W + W + 96;
    if (int e = ensure_ring(c, ring_stride(L))) return e;
    c->ring_maxed = maxed;
    *C_out = C;
    *L_out = L;
    return 0;
}

// Does the whole num_steps trajectory fit a plain ring (85 % of free HBM plus
// the ring already held, one buffer descriptor)?
bool plain_ring_fits(burg_ctx *c, int num_steps)
{
    const int W = c->sp.W;
    if (num_steps > stream_max_steps(c)) return false;
    const size_t per_entry = (size_t)c->sp.ntiles * kWave * sizeof(d2);
    size_t freeb = 0, totalb = 0;
    if (hipMemGetInfo(&freeb, &totalb) != hipSuccess) return false;
    const size_t need = (size_t)((long long)num_steps * W + W + 96) * per_entry;
    const size_t have = c->ring_entries * sizeof(d2);
    return need <= have || need <= (freeb + have) / 100 * 85;
}

// snap_every <= 0 ("auto"): every state when the whole trajectory fits a
// plain ring, else every 10th
int resolve_snap_every(burg_ctx *c, int num_steps, int snap_every)
{
    if (snap_every > 0) return snap_every;
    return plain_ring_fits(c, num_steps) ? 1 : 10;
}

// The layout of a retained-window trajectory ring (pure arithmetic:
// trajectory_ring and burg_ring_audit): a working ring of Lw entries -- up to
// the whole trajectory's diagonals, at most Lw_cap (the memory budget), at
// least 2W + 128, a multiple of every block length -- then n = num_steps / k
// windows of W + 64 entries from entry Lw.  BURG_RET_LW=m: exactly m W + 128
// (A/B knob).  False when even the shortest working ring does not fit.
bool retained_layout(int W, int num_steps, int k, long long Lw_cap, TrajMap *mp)
{
    const int n = num_steps / k;
    const long long Lwin = (long long)n * (W + 64);
    long long Lw = (long long)num_steps * W + W + 96;
    Lw = std::min(Lw, Lw_cap);
    Lw = std::min(Lw, (1LL << 21) - 2 - Lwin);
    Lw = Lw / 16 * 16;
    if (const char *e = std::getenv("BURG_RET_LW")) Lw = std::max(2LL, std::atoll(e)) * W + 128;
    *mp = TrajMap{};
    mp->L = Lw;
    mp->origin = 0;
    mp->Lt = ring_stride(Lw + Lwin);
    mp->base = Lw;
    mp->k = k;
    mp->n = n;
    return Lw >= 2LL * W + 128;
}

// The ring of a trajectory keeping every snap_every-th state (DESIGN.md
// section 4.1d).  snap_every = 1: the plain ring (every state while it fits;
// capped by free HBM it keeps the last C).  snap_every = k >= 2 on the pipe
// engine: a working ring of 2W + 128 entries plus num_steps / k retained
// windows of W + 64 entries (ring_pos) -- every k-th state survives the whole
// launch at no extra traffic.  Narrow tiles whose windows would overlap (k W <
// W + 64) and the streaming engine keep every state (a plain ring, which must
// then hold the whole trajectory).
int trajectory_ring(burg_ctx *c, int num_steps, int snap_every, TrajMap *mp, long long *C_out,
                    int *k_out = nullptr)
{
    if (int e = stream_setup(c)) return e;
    if (num_steps < 1) return fail(BURG_EINVAL, "num_steps must be >= 1");
    const int W = c->sp.W;
    const int k = resolve_snap_every(c, num_steps, snap_every);
    if (k_out) *k_out = k;
    *mp = TrajMap{};
    if (k >= 2 && c->eng_eff == BURG_ENGINE_PIPE && (long long)k * W >= W + 64) {
        const int n = num_steps / k;
        const size_t per_entry = (size_t)c->sp.ntiles * kWave * sizeof(d2);
        const long long Lwin = (long long)n * (W + 64);
        const size_t have = c->ring_entries * sizeof(d2);
        size_t freeb = 0, totalb = 0;
        HIPCHK(hipMemGetInfo(&freeb, &totalb));
        const size_t avail = (freeb + have) / 100 * 85;
        const size_t ret0 = c->d_ret0 ? 0 : c->m() * sizeof(double);
        // The working ring: as long as the memory budget allows, up to the
        // whole trajectory's diagonals -- each tile then walks a long region
        // of its ring as the plain ring does.  (Round 4: with a short working
        // ring of 2W + 128 entries the windowed trajectory ran 93-95 ms on
        // some boxes and allocations and 110-112 ms on others, while the
        // plain capped ring held 93-95 ms everywhere, profiles/r04/
        // ret_variance.)
        const long long Lmem = avail > ret0 ? (long long)((avail - ret0) / per_entry) - Lwin - 2 : 0;
        if (!retained_layout(W, num_steps, k, Lmem, mp)) {
            if (Lwin + 2LL * W + 128 >= (1LL << 21))
                return fail(BURG_ESHAPE, "%d retained states of %d-wide tiles exceed one buffer "
                            "descriptor per tile (2 GiB); raise snap_every", n, W);
            return fail(BURG_ENOMEM, "%d retained states (%.1f GB) do not fit in HBM; raise "
                        "snap_every", n, (double)(Lwin + 2LL * W + 128) * per_entry / 1e9);
        }
        const long long Lt = mp->Lt;
        const size_t need = (size_t)Lt * per_entry;
        if (need > have || have > need + need / 4 + ((size_t)1 << 30)) {
            dfree(c->d_ring);
            c->ring_entries = 0;
        }
        if (int e = ensure_ring(c, Lt)) return e;
        if (!c->d_ret0)
            if (int e = dalloc(&c->d_ret0, c->m())) return e;
        *C_out = num_steps;
        return 0;
    }
    long long C = 0, L = 0;
    if (int e = plain_ring(c, num_steps, &C, &L)) return e;
    if (k >= 2 && C < num_steps)
        return fail(BURG_ENOMEM, "snap_every=%d on %d-wide tiles keeps every state, and the "
                    "%d-step trajectory does not fit in HBM", k, W, num_steps);
    mp->L = L;
    mp->Lt = std::min<long long>(ring_stride(L),
                                 (long long)(c->ring_entries / (c->sp.ntiles * (size_t)kWave)));
    mp->k = 0;
    mp->n = 0;
    *C_out = C;
    return 0;
}

// One device-resident trajectory: num_steps steps from d_state[cur] (or the
// uploaded initial state) in ONE launch; the final state becomes
// d_state[cur].  The states kept in HBM (burg_trajectory_retained, copied out
// by burg_trajectory_copy):
//   * snap_every = 1: every state, in the ring (the reference's snapshot
//     matrix in ring layout, C/hypernet2D.py:89-126 keeps them all); a ring
//     that does not fit in 85 % of free HBM holds C < num_steps steps and
//     wraps INSIDE the launch -- the last C + 1 states stay, the older ones
//     are overwritten;
//   * snap_every = k >= 2: states 0, k, 2k, ... in retained windows
//     (trajectory_ring), whatever the grid size;
//   * snap_every <= 0: 1 if the whole trajectory fits, else 10.
// Only a trajectory longer than one buffer descriptor can address
// (stream_max_steps) or BURG_STREAM_CHUNK (tests) splits a plain-ring
// trajectory into several launches, each continuing from the previous one's
// last states; the retained states are then those of the last launch.
int stream_trajectory(burg_ctx *c, int num_steps, int snap_every, bool from_initial,
                      burg_stats *st)
{
    TrajMap mp;
    long long C = 0;
    int k = 1;
    if (int e = trajectory_ring(c, num_steps, snap_every, &mp, &C, &k)) return e;
    const int W = c->sp.W;
    if (from_initial && !c->d_w0) return fail(BURG_ESTATE, "no uploaded initial state");
    const double *start = from_initial ? c->d_w0 : c->d_state[c->cur];
    stream_stats_begin(c);
    CHK(launch_ring_load(stream_args(c, mp.L, 0, 0, &mp), W, start, c->stream));
    if (mp.k > 0)
        HIPCHK(hipMemcpyAsync(c->d_ret0, start, c->m() * sizeof(double), hipMemcpyDeviceToDevice,
                              c->stream));
    // A plain ring of fewer steps than the trajectory (capped by free memory)
    // wraps INSIDE one launch, as stream_advance's two-step ring does: the
    // states older than C steps are overwritten either way, and the
    // wavefront's fill and drain (nx + rows diagonals, ~7 % of a 16384 x 2048
    // slab's trajectory) are paid once, not per chunk.
    long long Kmax = std::max<long long>(C, stream_max_steps(c));
    if (mp.k > 0) Kmax = num_steps;  // retained windows: one launch (the map is per launch)
    if (const char *e = std::getenv("BURG_STREAM_CHUNK"))
        if (std::atoll(e) > 0 && mp.k == 0) Kmax = C;
    float ms = 0.f;
    long long origin = 0;
    int done = 0, last = 0;
    int64_t launches = 0;
    while (done < num_steps) {
        const int K = (int)std::min<long long>(num_steps - done, Kmax);
        if (int e = stream_launch(c, mp.L, origin, K, &ms, &mp)) return e;
        origin = (origin + (long long)K * W) % mp.L;
        done += K;
        last = K;
        ++launches;
    }
    const long long o_last = ((origin - (long long)last * W) % mp.L + mp.L) % mp.L;
    mp.origin = o_last;
    CHK(launch_ring_extract(stream_args(c, mp.L, o_last, 0, &mp), W, last, 1, 1,
                            c->d_state[c->cur ^ 1], 1, c->m(), c->stream));
    if (int e = check_bounds(c, "trajectory")) return e;
    c->cur ^= 1;
    // what stays resident
    TrajRecord &tr = c->tr;
    tr = TrajRecord{};
    tr.map = mp;
    tr.T = num_steps;
    tr.state0 = num_steps - last;
    if (mp.k > 0) {
        tr.first = 0;
        tr.count = mp.n + 1;
        tr.stride = mp.k;
        tr.ret0 = true;
    } else {
        // state r of the last launch occupies its diagonals (r-1) W .. r W + 62;
        // it is intact unless a later diagonal (up to last W + 62) reused an
        // entry, i.e. while (r-1) W + L > last W + 62
        // (snap_every k >= 2 on a plain ring -- narrow tiles whose windows
        // would overlap -- keeps every state: report the multiples of k)
        long long r0 = 0;
        while (r0 <= last && (r0 - 1) * W + mp.L <= (long long)last * W + 62) ++r0;
        const int64_t f = (tr.state0 + r0 + k - 1) / k * k;
        tr.first = f;
        tr.count = f <= num_steps ? (num_steps - f) / k + 1 : 0;
        tr.stride = k;
    }
    tr.valid = true;
    if (int e = stream_stats_end(c, st, num_steps, launches)) return e;
    if (st) {
        st->loop_ms = ms;
        st->march_kernel_ms = ms;
        st->march_launches = launches;
    }
    return 0;
}

// burg_run for the march solver on the streaming engine: the ring holds a
// chunk of C steps; after each chunk the snapshot columns it covers are
// transposed into the host matrix.
int stream_run(burg_ctx *c, const double *w0, int num_steps, double *snaps, int64_t ld_snaps,
               int snap_every, burg_stats *st, int32_t *step_iters, double *step_rel)
{
    if (int e = stream_setup(c)) return e;
    c->tr.valid = false;  // the ring is overwritten
    const int W = c->sp.W;
    const size_t m = c->m(), bytes = m * sizeof(double);
    size_t freeb = 0, totalb = 0;
    HIPCHK(hipMemGetInfo(&freeb, &totalb));
    const size_t per_entry = (size_t)c->sp.ntiles * kWave * sizeof(d2);
    // ring: up to a third of free memory (a step of ring = one state)
    long long Lmax = (long long)(freeb / 3 / per_entry);
    long long C = (Lmax - W - 96) / W;
    C = std::min<long long>(C, std::max(num_steps, 1));
    C = std::min<long long>(C, stream_max_steps(c));
    if (const char *e = std::getenv("BURG_STREAM_CHUNK")) {  // test knob: force chunking
        const long long v = std::atoll(e);
        if (v > 0) C = std::min(C, v);
    }
    if (C < 1) return fail(BURG_ENOMEM, "not enough device memory for a one-step ring");
    const long long L = C * W + W + 96;
    if ((size_t)c->sp.ntiles * (size_t)L * kWave > c->ring_entries) {  // else reuse the ring
        dfree(c->d_ring);
        c->ring_entries = 0;
        c->ring_maxed = false;  // sized for this run, not to the memory limit
        if (int e = ensure_ring(c, L)) return e;
    }

    // snapshot staging: S columns at a time
    int S = 0;
    double *d_tr = nullptr;
    const int64_t ncols = num_steps / snap_every + 1;
    if (snaps) {
        HIPCHK(hipMemGetInfo(&freeb, &totalb));
        S = (int)std::min<int64_t>(ncols, 64);
        while (S > 1 && (size_t)S * bytes > freeb / 3) S /= 2;
        if (int e = dalloc(&d_tr, (size_t)S * m)) return e;
    }
    float flush_ms = 0.f;
    hipEvent_t f0 = nullptr, f1 = nullptr;
    (void)hipEventCreate(&f0);
    (void)hipEventCreate(&f1);
    // copy host columns [col, col+cnt) = states k0 + j*snap_every (relative to origin)
    auto flush = [&](long long origin, int k0, int cnt, int64_t col) -> int {
        for (int j0 = 0; j0 < cnt; j0 += S) {
            const int n = std::min(S, cnt - j0);
            HIPCHK(hipEventRecord(f0, c->stream));
            CHK(launch_ring_extract(stream_args(c, L, origin, 0), W, k0 + j0 * snap_every,
                                    snap_every, n, d_tr, n, (size_t)S * m, c->stream));
            HIPCHK(d2h_2d(snaps + col + j0, (size_t)ld_snaps * sizeof(double), d_tr,
                          n * sizeof(double), n * sizeof(double), m, c->stream));
            HIPCHK(hipEventRecord(f1, c->stream));
            HIPCHK(hipEventSynchronize(f1));
            float t = 0.f;
            (void)hipEventElapsedTime(&t, f0, f1);
            flush_ms += t;
        }
        return 0;
    };

    int rc = BURG_OK;
    stream_stats_begin(c);
    HIPCHK(h2d(c->d_state[c->cur], w0, bytes, c->stream));
    CHK(launch_ring_load(stream_args(c, L, 0, 0), W, c->d_state[c->cur], c->stream));
    if (snaps) rc = flush(0, 0, 1, 0);
    float ms = 0.f;
    long long origin = 0;
    int done = 0, last = 0;
    int64_t launches = 0;
    while (rc == BURG_OK && done < num_steps) {
        const int K = (int)std::min<long long>(num_steps - done, C);
        rc = stream_launch(c, L, origin, K, &ms);
        if (rc) break;
        ++launches;
        if (snaps) {
            // columns j with done < j*snap_every <= done + K
            const int64_t j0 = done / snap_every + 1, j1 = (done + K) / snap_every;
            if (j1 >= j0)
                rc = flush(origin, (int)(j0 * snap_every - done), (int)(j1 - j0 + 1), j0);
        }
        origin = (origin + (long long)K * W) % L;
        done += K;
        last = K;
    }
    if (rc == BURG_OK && num_steps > 0) {
        const long long o_last = ((origin - (long long)last * W) % L + L) % L;
        rc = launch_ring_extract(stream_args(c, L, o_last, 0), W, last, 1, 1,
                                 c->d_state[c->cur ^ 1], 1, m, c->stream);
        if (rc == -3) rc = fail(BURG_EHIP, "ring extract launch failed");
        else c->cur ^= 1;
    }
    if (rc == BURG_OK) rc = check_bounds(c, "burg_run (stream)");
    if (rc == BURG_OK) rc = stream_stats_end(c, st, num_steps, launches);
    if (st) {
        st->loop_ms = ms;
        st->flush_ms = flush_ms;
        if (c->profile) {
            st->march_kernel_ms = ms;
            st->march_launches = launches;
        }
    }
    for (int s = 0; s < num_steps; ++s) {
        if (step_iters) step_iters[s] = 1;
        if (step_rel) step_rel[s] = 0.0;
    }
    (void)hipStreamSynchronize(c->stream);
    dfree(d_tr);
    // the ring of a long run can be large: give it back
    dfree(c->d_ring);
    c->ring_entries = 0;
    (void)hipEventDestroy(f0);
    (void)hipEventDestroy(f1);
    return rc;
}

// ---- multi-GPU halo rings ------------------------------------------------
// One ring per rank boundary b (between ranks b-1 and b): kPipeR step slots x
// nx granules of 16 B, all sentinel colour 0 at creation, written by the
// producer rank b-1's top strip and polled by the consumer rank b's comm
// waves, both at system scope (sc0 sc1); no host thread touches it at run
// time.  Where it lives:
//   * mode 2 (default): the consumer's own device memory -- uncached
//     (hipDeviceMallocUncached: remote stores arriving over xGMI are seen by
//     the polls without an L2 invalidate), exported with hipIpcGetMemHandle
//     and opened by the producer (hipIpcOpenMemHandle): producer stores cross
//     xGMI once, consumer polls stay on its own HBM;
//   * mode 1: pinned POSIX shared host memory mapped into both GPUs (the
//     fallback, and BURG_HALO=host).
// Rendezvous: a POSIX shared-memory object per boundary, created by the
// consumer: the host ring followed by a control page (the IPC handle, whether
// the device ring exists, and the mode the producer chose when it connected).
// The consumer reads the producer's choice at its first launch.
struct HaloCtl {
    uint32_t magic;
    uint32_t dev_ok;  // consumer: device ring exported
    volatile uint32_t choice;  // producer: 1 host ring, 2 device ring (the consumer may
                               // demote 2 to 1 in burg_slab_verify)
    uint32_t pad;
    hipIpcMemHandle_t handle;
};
// Device-ring self-test: two granules just past the ring (never part of the
// step slots).  The consumer stores kProbeC at granule 1 when it exports the
// ring; the producer, having opened it, must read kProbeC back over xGMI and
// stores kProbeP at granule 0, which the consumer must read in
// burg_slab_verify.  Either check failing puts the boundary on the host ring.
constexpr size_t kHaloProbeBytes = 256;
constexpr unsigned kProbeC[4] = {0xB0A6C7A1u, 0x3FF0C0DEu, 0x12345678u, 0x40090000u};
constexpr unsigned kProbeP[4] = {0x5A5A0001u, 0x3FF1C0DEu, 0x9ABCDEF0u, 0x400A0000u};
constexpr uint32_t kHaloMagic = 0xB0A6C7A1u;
constexpr size_t kHaloCtlBytes = 4096;
static_assert(sizeof(HaloCtl) <= kHaloCtlBytes, "halo control page");

std::string halo_shm_name(const std::string &job, int boundary)
{
    return "/burg_" + job + "_b" + std::to_string(boundary);
}

HaloCtl *halo_ctl(const burg_ctx *c, void *host) { return (HaloCtl *)((char *)host + c->halo_bytes); }

bool halo_force_host()
{
    const char *e = std::getenv("BURG_HALO");
    return e && std::strcmp(e, "host") == 0;
}

int halo_map(burg_ctx *c, const std::string &name, bool create, void **host, d2 **dev)
{
    const size_t bytes = c->halo_bytes + kHaloCtlBytes;
    const int fd = shm_open(name.c_str(), create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
    if (fd < 0) return fail(BURG_EHALO, "shm_open(%s): %s", name.c_str(), strerror(errno));
    if (create && ftruncate(fd, (off_t)bytes) != 0) {
        close(fd);
        shm_unlink(name.c_str());
        return fail(BURG_EHALO, "ftruncate(%s): %s", name.c_str(), strerror(errno));
    }
    void *p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return fail(BURG_EHALO, "mmap(%s): %s", name.c_str(), strerror(errno));
    if (create) {
        // sentinel colour 0 (pipe.hip): {lo 0xBEEF5A5A, hi 0x7FF4DEAD} in both halves
        uint32_t *w = (uint32_t *)p;
        for (size_t i = 0; i < c->halo_bytes / 4; i += 2) {
            w[i] = 0xBEEF5A5Au;
            w[i + 1] = 0x7FF4DEADu;
        }
        std::memset((char *)p + c->halo_bytes, 0, kHaloCtlBytes);
    }
    hipError_t e = hipHostRegister(p, bytes, hipHostRegisterMapped);
    if (e != hipSuccess) {
        munmap(p, bytes);
        return fail(BURG_EHALO, "hipHostRegister(%s, %zu): %s", name.c_str(), bytes,
                    hipGetErrorString(e));
    }
    void *dp = nullptr;
    e = hipHostGetDevicePointer(&dp, p, 0);
    if (e != hipSuccess) {
        (void)hipHostUnregister(p);
        munmap(p, bytes);
        return fail(BURG_EHALO, "hipHostGetDevicePointer(%s): %s", name.c_str(), hipGetErrorString(e));
    }
    *host = p;
    *dev = (d2 *)dp;
    return 0;
}

void halo_unmap(burg_ctx *c, void *&host, d2 *&dev)
{
    if (host) {
        (void)hipHostUnregister(host);
        munmap(host, c->halo_bytes + kHaloCtlBytes);
    }
    host = nullptr;
    dev = nullptr;
}

// consumer: the device ring in its own memory, exported for the producer
// (any failure leaves the host ring as the only option)
void halo_export_device_ring(burg_ctx *c, HaloCtl *ctl)
{
    if (halo_force_host()) return;
    void *r = nullptr;
    const size_t bytes = c->halo_bytes + kHaloProbeBytes;
    if (hipExtMallocWithFlags(&r, bytes, hipDeviceMallocUncached) != hipSuccess || !r) {
        (void)hipGetLastError();
        c->halo_note = "hipExtMallocWithFlags(uncached) failed";
        return;
    }
    hipIpcMemHandle_t h{};
    const int probe0 = (int)(c->halo_bytes / 16);
    unsigned got[4];
    if (launch_pipe_fill(r, bytes / 16, 0, c->stream) != 0 ||
        halo_probe(r, bytes, probe0 + 1, kProbeC, -1, kProbeC, 0.0, got, c->stream) != 0 ||
        hipStreamSynchronize(c->stream) != hipSuccess || hipIpcGetMemHandle(&h, r) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFree(r);
        c->halo_note = "device ring export failed";
        return;
    }
    c->halo_in_ring = (d2 *)r;
    ctl->handle = h;
    ctl->dev_ok = 1;
}

// consumer, first launch after the barrier that follows every rank's
// burg_slab_connect: take the ring the producer chose
int halo_resolve_in(burg_ctx *c)
{
    if (c->rank == 0 || c->halo_in_mode) return 0;
    HaloCtl *ctl = halo_ctl(c, c->halo_in_host);
    const uint32_t ch = ctl->choice;
    if (ch == 2 && c->halo_in_ring) {
        c->halo_in_dev = c->halo_in_ring;
    } else if (ch == 1) {
        c->halo_in_dev = c->halo_in_hostdev;
    } else {
        return fail(BURG_ESTATE, "rank %d: the rank below has not connected to the halo ring yet "
                                 "(burg_slab_connect on every rank, then a barrier, before the "
                                 "first launch)", c->rank);
    }
    c->halo_in_mode = (int)ch;
    return 0;
}

// producer, first launch (after the barrier that follows burg_slab_verify):
// take the consumer's verdict on the device ring
void halo_resolve_out(burg_ctx *c)
{
    if (c->halo_out_resolved || c->rank + 1 >= c->world) return;
    c->halo_out_resolved = true;
    HaloCtl *ctl = halo_ctl(c, c->halo_out_host);
    if (c->halo_out_mode == 2 && __atomic_load_n(&ctl->choice, __ATOMIC_ACQUIRE) == 1) {
        c->halo_out_dev = c->halo_out_hostdev;
        c->halo_out_mode = 1;
        c->halo_note = "the rank above rejected the device ring (burg_slab_verify)";
    }
}

}  // namespace

extern "C" {

int burg_slab_verify(burg_ctx *c)
{
    if (!c) return fail(BURG_EINVAL, "null context");
    if (c->world == 1 || c->rank == 0) return BURG_OK;
    if (!c->halo_connected)
        return fail(BURG_ESTATE, "burg_slab_verify before burg_slab_connect");
    HIPCHK(hipSetDevice(c->device));
    HaloCtl *ctl = halo_ctl(c, c->halo_in_host);
    const uint32_t ch = __atomic_load_n(&ctl->choice, __ATOMIC_ACQUIRE);
    if (ch == 0)
        return fail(BURG_ESTATE, "rank %d: the rank below has not connected to the halo ring yet",
                    c->rank);
    if (ch != 2 || !c->halo_in_ring) return BURG_OK;
    const size_t bytes = c->halo_bytes + kHaloProbeBytes;
    unsigned got[4] = {0, 0, 0, 0};
    const int pr = halo_probe(c->halo_in_ring, bytes, -1, kProbeP, (int)(c->halo_bytes / 16),
                              kProbeP, 0.25, got, c->stream);
    // BURG_HALO_REJECT=1: test hook, reject a good ring (exercises the demotion)
    const char *rej = std::getenv("BURG_HALO_REJECT");
    const bool force = rej && std::strcmp(rej, "1") == 0;
    if (force || pr != 0 || std::memcmp(got, kProbeP, sizeof got) != 0) {
        (void)hipGetLastError();
        c->halo_note = force ? "device ring rejected by BURG_HALO_REJECT"
                       : pr  ? "consumer probe kernel failed"
                             : "the producer's probe store never arrived in the device ring";
        __atomic_store_n(&ctl->choice, 1u, __ATOMIC_RELEASE);  // both sides use the host ring
    }
    return BURG_OK;
}

const char *burg_slab_halo_note(burg_ctx *c) { return c ? c->halo_note.c_str() : ""; }

int burg_abi_version(void) { return BURG_ABI_VERSION; }

const char *burg_last_error(void) { return g_err.c_str(); }

int burg_ctx_create(int device, int nx, int ny, burg_ctx **out)
{
    return burg_ctx_create_slab(device, nx, ny, 0, ny, 0, 1, nullptr, out);
}

int burg_ctx_create_slab(int device, int nx, int ny_total, int row0, int nrows, int rank,
                         int world, const char *halo_name, burg_ctx **out)
{
    if (!out) return fail(BURG_EINVAL, "null out pointer");
    *out = nullptr;
    if (nx < 1 || ny_total < 1 || row0 < 0 || nrows < 1 || row0 + nrows > ny_total)
        return fail(BURG_EINVAL, "bad grid: nx=%d ny=%d row0=%d nrows=%d", nx, ny_total, row0,
                    nrows);
    if (world < 1 || rank < 0 || rank >= world)
        return fail(BURG_EINVAL, "bad rank %d of world %d", rank, world);
    if (world == 1 && (row0 != 0 || nrows != ny_total))
        return fail(BURG_EINVAL, "a single-rank context owns the whole grid");
    if (world > 1) {
        if (!halo_name || !*halo_name || std::strlen(halo_name) > 64 ||
            std::strchr(halo_name, '/'))
            return fail(BURG_EINVAL, "multi-GPU slabs need a halo name (1-64 chars, no '/')");
        if ((rank == 0) != (row0 == 0) || (rank == world - 1) != (row0 + nrows == ny_total))
            return fail(BURG_EINVAL, "rank %d of %d does not own its slab's end rows", rank, world);
    }
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev)
        return fail(BURG_EINVAL, "device %d out of range (%d visible)", device, ndev);
    HIPCHK(hipSetDevice(device));
    burg_ctx *c = new burg_ctx();
    c->device = device;
    c->nx = nx;
    c->ny_total = ny_total;
    c->row0 = row0;
    c->nrows = nrows;
    c->rank = rank;
    c->world = world;
    c->engine = BURG_ENGINE_PIPE;
    if (const char *e = std::getenv("BURG_SPIN_SECONDS")) {
        const double v = std::atof(e);
        if (v > 0) c->spin_ticks = (long long)(v * 1e8);
    }
    int e = 0;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
        burg_ctx_destroy(c);
        return fail(BURG_EHIP, "stream/event creation failed");
    }
    if ((e = dalloc(&c->d_state[0], c->m())) || (e = dalloc(&c->d_state[1], c->m())) ||
        (e = dalloc(&c->d_stats, 1)) || (e = dalloc(&c->d_stats_solve, 1))) {
        burg_ctx_destroy(c);
        return e;
    }
    (void)hipMemsetAsync(c->d_stats, 0, sizeof(DevStats), c->stream);
    (void)hipMemsetAsync(c->d_stats_solve, 0, sizeof(DevStats), c->stream);
    if ((e = engine_alloc(c))) {
        burg_ctx_destroy(c);
        return e;
    }
    if (world > 1) {
        c->halo_name = halo_name;
        c->halo_bytes = (size_t)kPipeR * nx * sizeof(d2);
        if (rank > 0) {
            const std::string nm = halo_shm_name(c->halo_name, rank);
            if ((e = halo_map(c, nm, true, &c->halo_in_host, &c->halo_in_hostdev))) {
                burg_ctx_destroy(c);
                return e;
            }
            HaloCtl *ctl = halo_ctl(c, c->halo_in_host);
            halo_export_device_ring(c, ctl);
            __atomic_store_n(&ctl->magic, kHaloMagic, __ATOMIC_RELEASE);
        }
    } else {
        c->halo_connected = true;
    }
    *out = c;
    return BURG_OK;
}

int burg_slab_halo_mode(burg_ctx *c, int *in_mode, int *out_mode)
{
    if (!c || !in_mode || !out_mode) return fail(BURG_EINVAL, "null argument");
    if (c->world > 1 && c->halo_connected) CHK(halo_resolve_in(c));
    *in_mode = c->rank > 0 ? c->halo_in_mode : 0;
    *out_mode = c->rank + 1 < c->world ? c->halo_out_mode : 0;
    return BURG_OK;
}

int burg_slab_connect(burg_ctx *c)
{
    if (!c) return fail(BURG_EINVAL, "null context");
    if (c->world == 1 || c->halo_connected) return BURG_OK;
    HIPCHK(hipSetDevice(c->device));
    if (c->rank + 1 < c->world) {
        const std::string nm = halo_shm_name(c->halo_name, c->rank + 1);
        if (int e = halo_map(c, nm, false, &c->halo_out_host, &c->halo_out_hostdev)) return e;
        HaloCtl *ctl = halo_ctl(c, c->halo_out_host);
        if (__atomic_load_n(&ctl->magic, __ATOMIC_ACQUIRE) != kHaloMagic)
            return fail(BURG_EHALO, "halo ring %s: the rank above has not finished creating it",
                        nm.c_str());
        uint32_t choice = 1;
        c->halo_out_dev = c->halo_out_hostdev;
        if (ctl->dev_ok && !halo_force_host()) {
            void *p = nullptr;
            if (hipIpcOpenMemHandle(&p, ctl->handle, hipIpcMemLazyEnablePeerAccess) == hipSuccess && p) {
                // read the consumer's probe back and leave ours, across the link
                const size_t bytes = c->halo_bytes + kHaloProbeBytes;
                const int probe0 = (int)(c->halo_bytes / 16);
                unsigned got[4] = {0, 0, 0, 0};
                const int pr = halo_probe(p, bytes, probe0, kProbeP, probe0 + 1, kProbeC, 0.25, got,
                                          c->stream);
                if (pr == 0 && std::memcmp(got, kProbeC, sizeof got) == 0) {
                    c->halo_out_ipc = p;
                    c->halo_out_dev = (d2 *)p;
                    choice = 2;
                } else {
                    (void)hipGetLastError();
                    (void)hipIpcCloseMemHandle(p);
                    c->halo_note = pr ? "producer probe kernel failed"
                                      : "producer read a wrong probe from the device ring";
                }
            } else {
                (void)hipGetLastError();  // fall back to the host ring
                c->halo_note = "hipIpcOpenMemHandle failed";
            }
        }
        c->halo_out_mode = (int)choice;
        __atomic_store_n(&ctl->choice, choice, __ATOMIC_RELEASE);
    }
    c->halo_connected = true;
    return BURG_OK;
}

void burg_ctx_destroy(burg_ctx *c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto ev : c->prof_ev) (void)hipEventDestroy(ev);
    dfree(c->d_inv_dx);
    dfree(c->d_inv_dy);
    dfree(c->d_src);
    dfree(c->d_lbc);
    dfree(c->d_edges);
    dfree(c->d_counters);
    dfree(c->d_stats);
    dfree(c->d_stats_solve);
    dfree(c->d_state[0]);
    dfree(c->d_state[1]);
    dfree(c->d_w0);
    dfree(c->d_r);
    dfree(c->d_d);
    dfree(c->d_x);
    dfree(c->d_partials);
    dfree(c->d_sumsq);
    dfree(c->d_halo_rows);
    dfree(c->d_ret0);
    if (c->bat_child) burg_ctx_destroy(c->bat_child);
    stream_free(c);
    if (c->halo_out_ipc) (void)hipIpcCloseMemHandle(c->halo_out_ipc);
    if (c->halo_in_ring) (void)hipFree(c->halo_in_ring);
    halo_unmap(c, c->halo_in_host, c->halo_in_hostdev);
    halo_unmap(c, c->halo_out_host, c->halo_out_hostdev);
    if (c->world > 1 && c->rank > 0) shm_unlink(halo_shm_name(c->halo_name, c->rank).c_str());
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int burg_set_problem(burg_ctx *c, const double *inv_dx, const double *inv_dy,
                     const double *src, const double *lbc, double dt)
{
    if (!c) return fail(BURG_EINVAL, "null context");
    if (!inv_dx || !inv_dy || !src || !lbc) return fail(BURG_EINVAL, "null coefficient array");
    if (!(dt > 0.0) || !std::isfinite(dt)) return fail(BURG_EINVAL, "dt must be > 0");
    // the march cell's fast window (cell_math.h) relies on h_x = dt/4 / dx and
    // h_y = dt/4 / dy in (0, 2^100): q then stays finite and >= 0.25
    for (int i = 0; i < c->nx; ++i)
        if (!(0.25 * dt * inv_dx[i] > 0.0 && 0.25 * dt * inv_dx[i] < 0x1p100))
            return fail(BURG_EINVAL, "dt/dx out of range (0, 2^102) at column %d", i);
    for (int i = 0; i < c->ny_total; ++i)
        if (!(0.25 * dt * inv_dy[i] > 0.0 && 0.25 * dt * inv_dy[i] < 0x1p100))
            return fail(BURG_EINVAL, "dt/dy out of range (0, 2^102) at row %d", i);
    HIPCHK(hipSetDevice(c->device));
    if (!c->d_inv_dx) {
        if (int e = dalloc(&c->d_inv_dx, (size_t)c->nx)) return e;
        if (int e = dalloc(&c->d_inv_dy, (size_t)c->ny_total)) return e;
        if (int e = dalloc(&c->d_src, (size_t)c->nx)) return e;
        if (int e = dalloc(&c->d_lbc, (size_t)c->ny_total)) return e;
    }
    HIPCHK(h2d(c->d_inv_dx, inv_dx, sizeof(double) * c->nx, c->stream));
    HIPCHK(h2d(c->d_inv_dy, inv_dy, sizeof(double) * c->ny_total, c->stream));
    HIPCHK(h2d(c->d_src, src, sizeof(double) * c->nx, c->stream));
    HIPCHK(h2d(c->d_lbc, lbc, sizeof(double) * c->ny_total, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->dt = dt;
    c->cf.inv_dx = c->d_inv_dx;
    c->cf.inv_dy = c->d_inv_dy + c->row0;
    c->cf.src = c->d_src;
    c->cf.lbc = c->d_lbc + c->row0;
    c->cf.alpha = 0.5 * dt;
    c->cf.nx = c->nx;
    c->cf.ny = c->nrows;
    c->have_problem = true;
    c->colc_ready = false;
    return BURG_OK;
}

int burg_set_options(burg_ctx *c, int tile_w, int par_passes, double tol, int profile)
{
    if (!c) return fail(BURG_EINVAL, "null context");
    if (tile_w != 64 && tile_w != 128) return fail(BURG_EINVAL, "tile_w must be 64 or 128");
    if (!(tol >= 0.0) || !(tol < 1e-6)) return fail(BURG_EINVAL, "tol must be in [0, 1e-6)");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->tw = tile_w;
    c->par_passes_opt = par_passes;
    c->tol = tol;
    c->profile = profile ? 1 : 0;
    return engine_alloc(c);
}

int burg_set_engine(burg_ctx *c, int engine, int stream_w, int tiles_target)
{
    if (!c) return fail(BURG_EINVAL, "null context");
    if (engine != BURG_ENGINE_STREAM && engine != BURG_ENGINE_TILES && engine != BURG_ENGINE_PIPE)
        return fail(BURG_EINVAL, "unknown engine %d", engine);
    if (c->world > 1 && engine != BURG_ENGINE_PIPE)
        return fail(BURG_EINVAL, "multi-GPU slabs run on the pipe engine only");
    if (stream_w != 0 && !stream_width_supported(stream_w))
        return fail(BURG_EINVAL, "stream_w must be 0 or a power of two in [8, 4096]");
    if (tiles_target < 0) return fail(BURG_EINVAL, "tiles_target < 0");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    const bool replan = engine != c->engine;
    c->engine = engine;
    if (replan || stream_w != c->stream_w_opt || tiles_target != c->tiles_target_opt) {
        stream_free(c);
        c->stream_w_opt = stream_w;
        c->tiles_target_opt = tiles_target;
    }
    return BURG_OK;
}

int burg_residual(burg_ctx *c, const double *w, const double *wp, double *r, double *norm)
{
    BURG_TRACE("burg_residual");
    if (int e = check_ready(c)) return e;
    if (!w || !wp || !r) return fail(BURG_EINVAL, "null array");
    if (int e = ensure_scratch(c)) return e;
    const size_t bytes = c->m() * sizeof(double);
    HIPCHK(h2d(c->d_x, w, bytes, c->stream));
    HIPCHK(h2d(c->d_d, wp, bytes, c->stream));
    double nrm = 0.0;
    if (int e = residual_norm(c, c->d_x, c->d_d, c->d_r, &nrm)) return e;
    HIPCHK(d2h(r, c->d_r, bytes, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (norm) *norm = nrm;
    return BURG_OK;
}

int burg_slab_residual(burg_ctx *c, const double *w, const double *wp, const double *halo_w,
                       const double *halo_wp, double *r, double *sumsq)
{
    BURG_TRACE("burg_slab_residual");
    if (int e = check_ready(c)) return e;
    if (!w || !wp || !r) return fail(BURG_EINVAL, "null array");
    if ((halo_w == nullptr) != (halo_wp == nullptr))
        return fail(BURG_EINVAL, "halo_w and halo_wp must both be given or both be NULL");
    if (halo_w && c->row0 == 0)
        return fail(BURG_EINVAL, "the bottom slab (row 0) has no south halo row");
    if (!halo_w && c->row0 > 0)
        return fail(BURG_EINVAL, "a slab above row 0 needs the south halo rows (rows %d of w, wp)",
                    c->row0 - 1);
    if (int e = ensure_scratch(c)) return e;
    const size_t bytes = c->m() * sizeof(double), hb = 2 * (size_t)c->nx * sizeof(double);
    HIPCHK(h2d(c->d_x, w, bytes, c->stream));
    HIPCHK(h2d(c->d_d, wp, bytes, c->stream));
    // the halo rows go to a scratch buffer kept by the context (allocated on
    // first use: no hipMalloc / hipFree -- a device-wide sync -- per call)
    const double *d_halo = nullptr;
    if (halo_w) {
        if (!c->d_halo_rows)
            if (int e = dalloc(&c->d_halo_rows, 4 * (size_t)c->nx)) return e;
        HIPCHK(h2d(c->d_halo_rows, halo_w, hb, c->stream));
        HIPCHK(h2d(c->d_halo_rows + 2 * c->nx, halo_wp, hb, c->stream));
        d_halo = c->d_halo_rows;
    }
    int rc = launch_residual(c->cf, c->d_x, c->d_d, c->d_r, c->d_partials, c->d_sumsq, d_halo,
                             d_halo ? d_halo + 2 * c->nx : nullptr, c->stream);
    double s = 0.0;
    if (rc == 0 &&
        (d2h(r, c->d_r, bytes, c->stream) != hipSuccess ||
         hipMemcpyAsync(&s, c->d_sumsq, sizeof s, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
         hipStreamSynchronize(c->stream) != hipSuccess))
        rc = -3;
    if (rc) return fail(BURG_EHIP, "slab residual failed: %s", hipGetErrorString(hipGetLastError()));
    if (sumsq) *sumsq = s;
    return BURG_OK;
}

int burg_jvp(burg_ctx *c, const double *w, const double *x, double *y)
{
    BURG_TRACE("burg_jvp");
    if (int e = check_ready(c)) return e;
    if (!w || !x || !y) return fail(BURG_EINVAL, "null array");
    if (int e = ensure_scratch(c)) return e;
    const size_t bytes = c->m() * sizeof(double);
    HIPCHK(h2d(c->d_x, w, bytes, c->stream));
    HIPCHK(h2d(c->d_d, x, bytes, c->stream));
    CHK(launch_jvp(c->cf, c->d_x, c->d_d, c->d_r, c->stream));
    HIPCHK(d2h(y, c->d_r, bytes, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return BURG_OK;
}

int burg_block_solve(burg_ctx *c, const double *w, const double *rhs, double *delta)
{
    BURG_TRACE("burg_block_solve");
    if (int e = check_ready(c)) return e;
    if (!w || !rhs || !delta) return fail(BURG_EINVAL, "null array");
    if (int e = ensure_scratch(c)) return e;
    const size_t bytes = c->m() * sizeof(double);
    HIPCHK(h2d(c->d_x, w, bytes, c->stream));
    HIPCHK(h2d(c->d_r, rhs, bytes, c->stream));
    if (int e = block_solve(c, c->d_x, c->d_r, c->d_d)) return e;
    HIPCHK(d2h(delta, c->d_d, bytes, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return BURG_OK;
}

int burg_upload_state(burg_ctx *c, const double *w)
{
    if (int e = check_ready(c)) return e;
    if (!w) return fail(BURG_EINVAL, "null state");
    HIPCHK(h2d(c->d_state[c->cur], w, c->m() * sizeof(double), c->stream));
    if (!c->d_w0)
        if (int e = dalloc(&c->d_w0, c->m())) return e;
    {
        // uniform (u plane | v plane each one value, bitwise)? -- the paired
        // sweep kernel's condition (pipe_args)
        const size_t n = c->m() / 2;
        uint64_t u0 = 0, v0 = 0;
        std::memcpy(&u0, &w[0], 8);
        std::memcpy(&v0, &w[n], 8);
        bool uni = true;
        for (size_t i = 0; i < n && uni; ++i) {
            uint64_t x, y;
            std::memcpy(&x, &w[i], 8);
            std::memcpy(&y, &w[n + i], 8);
            uni = x == u0 && y == v0;
        }
        c->w0_uni = uni;
        c->w0c[0] = (unsigned)u0;
        c->w0c[1] = (unsigned)(u0 >> 32);
        c->w0c[2] = (unsigned)v0;
        c->w0c[3] = (unsigned)(v0 >> 32);
    }
    HIPCHK(hipMemcpyAsync(c->d_w0, c->d_state[c->cur], c->m() * sizeof(double),
                          hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return BURG_OK;
}

int burg_download_state(burg_ctx *c, double *w)
{
    if (int e = check_ready(c)) return e;
    if (!w) return fail(BURG_EINVAL, "null state");
    HIPCHK(d2h(w, c->d_state[c->cur], c->m() * sizeof(double), c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return BURG_OK;
}

int burg_kernel_bench(burg_ctx *c, int which, int reps, double *avg_ms)
{
    if (int e = check_ready(c)) return e;
    if (!avg_ms) return fail(BURG_EINVAL, "null avg_ms");
    if (reps < 1) return fail(BURG_EINVAL, "reps < 1");
    if (which != BURG_KERNEL_RESIDUAL && which != BURG_KERNEL_JVP)
        return fail(BURG_EINVAL, "unknown kernel %d", which);
    if (c->world > 1) return fail(BURG_EINVAL, "burg_kernel_bench: single-GPU contexts only");
    if (!c->d_w0) return fail(BURG_ESTATE, "burg_kernel_bench: call burg_upload_state first");
    if (int e = ensure_scratch(c)) return e;
    const size_t bytes = c->m() * sizeof(double);
    HIPCHK(hipMemcpyAsync(c->d_x, c->d_w0, bytes, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_d, c->d_state[c->cur], bytes, hipMemcpyDeviceToDevice,
                          c->stream));
    auto once = [&]() -> int {
        if (which == BURG_KERNEL_RESIDUAL)
            return launch_residual(c->cf, c->d_x, c->d_d, c->d_r, c->d_partials, c->d_sumsq,
                                   nullptr, nullptr, c->stream);
        return launch_jvp(c->cf, c->d_x, c->d_d, c->d_r, c->stream);
    };
    CHK(once());  // warm (code object, TLB)
    HIPCHK(hipEventRecord(c->ev0, c->stream));
    for (int i = 0; i < reps; ++i) CHK(once());
    HIPCHK(hipEventRecord(c->ev1, c->stream));
    HIPCHK(hipEventSynchronize(c->ev1));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    *avg_ms = (double)ms / reps;
    return BURG_OK;
}

int burg_advance(burg_ctx *c, int num_steps, int solver, burg_stats *st)
{
    BURG_TRACE("burg_advance");
    if (int e = check_ready(c)) return e;
    if (num_steps < 0) return fail(BURG_EINVAL, "num_steps < 0");
    if (solver != BURG_SOLVER_MARCH && solver != BURG_SOLVER_NEWTON)
        return fail(BURG_EINVAL, "unknown solver %d", solver);
    if (st) std::memset(st, 0, sizeof *st);
    if (solver == BURG_SOLVER_MARCH && c->engine != BURG_ENGINE_TILES)
        return stream_advance(c, num_steps, st);
    HIPCHK(hipMemsetAsync(c->d_stats, 0, sizeof(DevStats), c->stream));
    if (solver == BURG_SOLVER_NEWTON)
        if (int e = ensure_scratch(c)) return e;
    HIPCHK(hipEventRecord(c->ev0, c->stream));
    int64_t nupd = 0;
    int maxupd = 0;
    double rel = 0.0;
    for (int s = 0; s < num_steps; ++s) {
        const double *wp = c->d_state[c->cur];
        double *w = c->d_state[c->cur ^ 1];
        if (solver == BURG_SOLVER_MARCH) {
            if (int e = march_step(c, wp, w)) return e;
        } else {
            int its = 0;
            if (int e = newton_step(c, wp, w, 100, 1e-12, &its, &rel)) return e;
            nupd += its;
            maxupd = std::max(maxupd, its);
        }
        c->cur ^= 1;
    }
    HIPCHK(hipEventRecord(c->ev1, c->stream));
    HIPCHK(hipEventSynchronize(c->ev1));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    if (int e = read_stats(c, st)) return e;
    if (st) {
        st->loop_ms = ms;
        st->newton_updates = nupd;
        st->newton_max_updates = maxupd;
        st->last_rel = rel;
        if (solver == BURG_SOLVER_NEWTON) st->steps = num_steps;
    }
    collect_profile(c, st);
    return BURG_OK;
}

int burg_trajectory_ex(burg_ctx *c, int num_steps, int snap_every, int from_initial,
                       burg_stats *st)
{
    BURG_TRACE("burg_trajectory");
    if (int e = check_ready(c)) return e;
    if (st) std::memset(st, 0, sizeof *st);
    if (c->engine == BURG_ENGINE_TILES)
        return fail(BURG_EINVAL, "burg_trajectory runs on the stream/pipe engines");
    return stream_trajectory(c, num_steps, snap_every, from_initial != 0, st);
}

int burg_trajectory(burg_ctx *c, int num_steps, int from_initial, burg_stats *st)
{
    return burg_trajectory_ex(c, num_steps, 1, from_initial, st);
}

int burg_reserve_trajectory_ex(burg_ctx *c, int num_steps, int snap_every)
{
    BURG_TRACE("burg_reserve_trajectory");
    if (int e = check_ready(c)) return e;
    if (c->engine == BURG_ENGINE_TILES)
        return fail(BURG_EINVAL, "burg_reserve_trajectory serves the stream/pipe engines");
    TrajMap mp;
    long long C = 0;
    if (int e = trajectory_ring(c, num_steps, snap_every, &mp, &C)) return e;
    HIPCHK(hipStreamSynchronize(c->stream));
    return BURG_OK;
}

int burg_reserve_trajectory(burg_ctx *c, int num_steps)
{
    return burg_reserve_trajectory_ex(c, num_steps, 1);
}

int burg_trajectory_plan(burg_ctx *c, int num_steps, int snap_every, int *snap_every_out,
                         int64_t *retained_states, int64_t *ring_bytes)
{
    if (int e = check_ready(c)) return e;
    if (c->engine == BURG_ENGINE_TILES)
        return fail(BURG_EINVAL, "burg_trajectory_plan serves the stream/pipe engines");
    if (num_steps < 1) return fail(BURG_EINVAL, "num_steps must be >= 1");
    if (int e = stream_setup(c)) return e;
    const int k = resolve_snap_every(c, num_steps, snap_every);
    const int W = c->sp.W;
    const size_t per_entry = (size_t)c->sp.ntiles * kWave * sizeof(d2);
    int64_t nret = 0, bytes = 0;
    if (k >= 2 && c->eng_eff == BURG_ENGINE_PIPE && (long long)k * W >= W + 64) {
        nret = num_steps / k + 1;
        bytes = (int64_t)((2LL * W + 128 + (long long)(num_steps / k) * (W + 64)) * per_entry);
    } else if (plain_ring_fits(c, num_steps)) {
        nret = k >= 2 ? num_steps / k + 1 : num_steps + 1;
        bytes = (int64_t)(((long long)num_steps * W + W + 96) * per_entry);
    } else {
        nret = -1;  // a capped plain ring: the last C + 1 states (known after the run)
    }
    if (snap_every_out) *snap_every_out = k;
    if (retained_states) *retained_states = nret;
    if (ring_bytes) *ring_bytes = bytes;
    return BURG_OK;
}

int burg_trajectory_retained(burg_ctx *c, int64_t *first_state, int64_t *count, int *stride)
{
    if (!c) return fail(BURG_EINVAL, "null context");
    if (!c->tr.valid) return fail(BURG_ESTATE, "no trajectory resident (burg_trajectory_ex)");
    if (first_state) *first_state = c->tr.first;
    if (count) *count = c->tr.count;
    if (stride) *stride = c->tr.stride;
    return BURG_OK;
}

static int check_device_ptr(const burg_ctx *c, const void *p, const char *what);

// Columns col0 .. col0 + ncols - 1 of the resident trajectory (state
// first + j * stride in column j) into the C-order (2n x ld_out) matrix `out`
// at column offsets 0 .. ncols - 1: host memory (staged through the pinned
// bounce buffers, hostxfer.hip) or, with out_on_device, device memory of this GPU.
int burg_trajectory_copy(burg_ctx *c, int64_t col0, int64_t ncols, double *out, int64_t ld_out,
                         int out_on_device)
{
    BURG_TRACE("burg_trajectory_copy");
    if (int e = check_ready(c)) return e;
    const TrajRecord &tr = c->tr;
    if (!tr.valid || !c->sp_ready || !c->d_ring)
        return fail(BURG_ESTATE, "no trajectory resident (burg_trajectory_ex)");
    if (!out) return fail(BURG_EINVAL, "null output");
    if (col0 < 0 || ncols < 0 || col0 + ncols > tr.count)
        return fail(BURG_EINVAL, "columns [%lld, %lld) outside the %lld retained", (long long)col0,
                    (long long)(col0 + ncols), (long long)tr.count);
    if (ld_out < ncols || ld_out > INT32_MAX) return fail(BURG_EINVAL, "ld_out=%lld", (long long)ld_out);
    if (ncols == 0) return BURG_OK;
    if (out_on_device)
        if (int e = check_device_ptr(c, out, "out")) return e;
    const int W = c->sp.W;
    const size_t m = c->m();
    const StreamArgs ra = stream_args(c, tr.map.L, tr.map.origin, 0, &tr.map);
    // state q of the trajectory -> (relative state of the map's launch)
    auto rel = [&](int64_t j) { return tr.first + j * tr.stride - tr.state0; };
    int64_t j = col0;
    const int64_t j1 = col0 + ncols;
    int rc = BURG_OK;
    double *d_tr = nullptr;
    int S = 0;
    if (!out_on_device) {
        size_t freeb = 0, totalb = 0;
        HIPCHK(hipMemGetInfo(&freeb, &totalb));
        S = (int)std::min<int64_t>(ncols, 64);
        while (S > 1 && (size_t)S * m * sizeof(double) > freeb / 3) S /= 2;
        if (int e = dalloc(&d_tr, (size_t)S * m)) return e;
    }
    while (j < j1 && rc == BURG_OK) {
        double *dst = out_on_device ? out + (j - col0) : d_tr;
        const int ldo = out_on_device ? (int)ld_out : S;
        const size_t cap = out_on_device ? m * (size_t)ld_out - (size_t)(j - col0) : (size_t)S * m;
        int n = 0;
        if (tr.ret0 && rel(j) == 0) {
            // the initial state: its copy (the working ring has moved on)
            const double *p0 = c->d_ret0;
            if (launch_transpose(&p0, 1, m, dst, ldo, cap, bflag(c), c->stream))
                rc = fail(BURG_EHIP, "column copy failed");
            n = 1;
        } else {
            n = (int)std::min<int64_t>(j1 - j, out_on_device ? INT32_MAX : S);
            if (launch_ring_extract(ra, W, (int)rel(j), tr.stride, n, dst, ldo, cap, c->stream))
                rc = fail(BURG_EHIP, "ring extract launch failed");
        }
        if (rc == BURG_OK && !out_on_device &&
            d2h_2d(out + (j - col0), (size_t)ld_out * sizeof(double), d_tr,
                   (size_t)S * sizeof(double), (size_t)n * sizeof(double), m, c->stream) != hipSuccess)
            rc = fail(BURG_EHIP, "snapshot copy failed: %s", hipGetErrorString(hipGetLastError()));
        if (rc == BURG_OK && !out_on_device && hipStreamSynchronize(c->stream) != hipSuccess)
            rc = fail(BURG_EHIP, "snapshot copy failed: %s", hipGetErrorString(hipGetLastError()));
        j += n;
    }
    if (rc == BURG_OK && hipStreamSynchronize(c->stream) != hipSuccess)
        rc = fail(BURG_EHIP, "snapshot copy failed: %s", hipGetErrorString(hipGetLastError()));
    if (rc == BURG_OK) rc = check_bounds(c, "burg_trajectory_copy");
    dfree(d_tr);
    return rc;
}

static int check_device_ptr(const burg_ctx *c, const void *p, const char *what);

// Where a sweep's snapshot matrices go: nmu host matrices (C-order, leading
// dimension ld_host) or one device matrix (C-order, ld_dev) holding mu j's
// columns at j * ncols ... (j + 1) * ncols - 1 (np.hstack of the per-mu
// matrices, as C/run_prom.py:59-71 builds it); neither: states stay in HBM.
struct SweepOut {
    double *const *host = nullptr;
    int64_t ld_host = 0;
    double *dev = nullptr;
    int64_t ld_dev = 0;
};

// Side-by-side sweep groups: how many trajectories of this grid run at once
// as separate domains of one launch (0: none -- the grid alone fills half the
// chip or more, a slab, or a forced tile width).  BURG_SWEEP_BATCH=G forces G
// (1: off).
constexpr int kBatchMax = 16;
int batch_group(burg_ctx *c, int nmu)
{
    if (c->world > 1 || nmu < 2 || c->eng_eff != BURG_ENGINE_PIPE) return 0;
    if (const char *e = std::getenv("BURG_SWEEP_BATCH")) {
        const int v = std::atoi(e);
        return v >= 2 ? std::min({v, nmu, kBatchMax}) : 0;
    }
    if (c->stream_w_opt != 0 || c->tiles_target_opt != 0) return 0;
    // only a grid that leaves at least half of the CUs idle (one workgroup
    // per CU is the pipe engine's own plan; a grid that fills the chip, e.g.
    // 1024^2, runs back to back in time, section 4.1c)
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess)
        return 0;
    const int wgs = c->sp.nti * c->nwj;
    const int cap = pipe_max_resident_blocks(c->sp.W, false);
    if (cap <= 0 || 2 * wgs > ncu) return 0;
    return std::min({nmu, cap / wgs, kBatchMax});
}

// burg_sweep for small grids: the reference's
// drivers run a snapshot set one trajectory at a time (C/run_prom.py:59-71);
// a 250^2 grid fills ~32 of 256 CUs, so G trajectories run side by side as G
// independent domains stacked in ONE launch of an internal context (each
// domain's rows padded to whole strips; its own column table (mu2) and inlet
// rows (mu1)).  Every trajectory is the same exact march, bit for bit.
// Returns 1 when the mode does not apply (the caller runs the serial sweep).
static int sweep_side_by_side(burg_ctx *c, int nmu, const double *src_b, const double *lbc_b,
                              int T, int snap_every, const SweepOut &out, burg_stats *st)
{
    const int G = batch_group(c, nmu);
    if (G < 2) return 1;
    const int nx = c->nx, ny = c->nrows;
    const int nti_d = (ny + kWave - 1) / kWave, ny_pad = nti_d * kWave;
    const size_t m = c->m(), n = c->n();
    const int64_t ncols = T / snap_every + 1;
    if (!c->bat_child || c->bat_child_G != G) {
        if (c->bat_child) burg_ctx_destroy(c->bat_child);
        c->bat_child = nullptr;
        burg_ctx *ch = nullptr;
        if (int e = burg_ctx_create(c->device, nx, G * ny_pad, &ch)) return e;
        ch->bat_nd = G;
        ch->bat_ny_d = ny;
        // The stacked grid's tile target: 4096 lets it take the narrowest
        // tiles that stay resident (W = 8 at 9 x 250^2: 1 152 tiles, two
        // workgroups on some CUs) -- 2.86 ms per 9-trajectory launch against
        // 4.03 ms with W = 16 (profiles/r04/sweep250; back to back in time:
        // 19.47 ms).  BURG_SWEEP_BATCH_TILES overrides (A/B knob).
        ch->tiles_target_opt = 4096;
        if (const char *e = std::getenv("BURG_SWEEP_BATCH_TILES")) ch->tiles_target_opt = std::atoi(e);
        c->bat_child = ch;
        c->bat_child_G = G;
    }
    burg_ctx *ch = c->bat_child;
    ch->spin_ticks = c->spin_ticks;
    ch->engine = BURG_ENGINE_PIPE;
    // host copies of the grid's coefficient rows and of w0
    std::vector<double> ix(nx), iy(ny), w0(m);
    HIPCHK(d2h(ix.data(), c->cf.inv_dx, sizeof(double) * nx, c->stream));
    HIPCHK(d2h(iy.data(), c->cf.inv_dy, sizeof(double) * ny, c->stream));
    HIPCHK(d2h(w0.data(), c->d_w0, sizeof(double) * m, c->stream));
    const size_t nc = ch->n(), dpl = (size_t)ny_pad * nx;  // child plane, one domain's rows
    std::vector<double> iyt((size_t)G * ny_pad), lbt((size_t)G * ny_pad), w0s(2 * nc, 1.0);
    for (int j = 0; j < G; ++j)
        for (int r = 0; r < ny_pad; ++r) iyt[(size_t)j * ny_pad + r] = iy[std::min(r, ny - 1)];
    for (int j = 0; j < G; ++j) {
        std::memcpy(&w0s[j * dpl], &w0[0], sizeof(double) * n);
        std::memcpy(&w0s[nc + j * dpl], &w0[n], sizeof(double) * n);
    }
    double *d_srcb = nullptr, *d_tr = nullptr;
    d2 *d_colcb = nullptr;
    int S = 0;
    auto cleanup = [&]() {
        ch->ov_colc = nullptr;
        (void)hipStreamSynchronize(ch->stream);
        (void)hipStreamSynchronize(c->stream);
        // the internal context's ring (G trajectories of states) is given back:
        // the parent context may need the memory next
        dfree(ch->d_ring);
        ch->ring_entries = 0;
        ch->ring_maxed = false;
        ch->tr.valid = false;
        dfree(d_srcb);
        dfree(d_colcb);
        dfree(d_tr);
    };
    int rc = BURG_OK;
    double ms = 0.0, flush_ms = 0.0;
    int64_t ieee = 0, launches = 0, polls = 0, slow = 0, spins = 0;
    std::vector<double> srcg((size_t)G * nx);
    for (int g0 = 0; g0 < nmu && rc == BURG_OK; g0 += G) {
        const int nb = std::min(G, nmu - g0);
        for (int j = 0; j < G; ++j) {
            const int mj = g0 + std::min(j, nb - 1);  // (a short last group repeats its last mu)
            for (int r = 0; r < ny_pad; ++r)
                lbt[(size_t)j * ny_pad + r] =
                    lbc_b[(size_t)mj * c->ny_total + c->row0 + std::min(r, ny - 1)];
            std::memcpy(&srcg[(size_t)j * nx], src_b + (size_t)mj * nx, sizeof(double) * nx);
        }
        if ((rc = burg_set_problem(ch, ix.data(), iyt.data(), srcg.data(), lbt.data(), c->dt))) break;
        if ((rc = stream_setup(ch))) break;
        if (ch->eng_eff != BURG_ENGINE_PIPE) {
            if (g0 == 0) {
                cleanup();
                return 1;  // the stacked grid does not fit resident: serial sweep
            }
            rc = fail(BURG_ESHAPE, "side-by-side sweep lost its pipe plan");
            break;
        }
        const size_t ncolp = (size_t)ch->sp.ntj * ch->sp.W;
        if (!d_srcb) {
            if ((rc = dalloc(&d_srcb, (size_t)G * nx)) || (rc = dalloc(&d_colcb, (size_t)G * ncolp)))
                break;
            if (out.host) {
                size_t freeb = 0, totalb = 0;
                if (hipMemGetInfo(&freeb, &totalb) != hipSuccess) {
                    rc = fail(BURG_EHIP, "hipMemGetInfo failed");
                    break;
                }
                S = (int)std::min<int64_t>(ncols, 64);
                while (S > 1 && (size_t)S * m * sizeof(double) > freeb / 3) S /= 2;
                if ((rc = dalloc(&d_tr, (size_t)S * m))) break;
            }
        }
        if (h2d(d_srcb, srcg.data(), sizeof(double) * G * nx, ch->stream) != hipSuccess ||
            launch_colc_batch(ch->cf, G, d_srcb, (int)ncolp, d_colcb, ch->stream) != 0) {
            rc = fail(BURG_EHIP, "side-by-side sweep: column tables: %s",
                      hipGetErrorString(hipGetLastError()));
            break;
        }
        ch->bat_colc_stride = ncolp;
        ch->ov_colc = d_colcb;
        if ((rc = burg_upload_state(ch, w0s.data()))) break;
        burg_stats cst{};
        rc = stream_trajectory(ch, T, snap_every, true, &cst);
        ch->ov_colc = nullptr;
        if (rc) break;
        const TrajRecord &tr = ch->tr;
        if (!(tr.valid && tr.first == 0 && tr.stride == snap_every && tr.count == ncols)) {
            rc = fail(BURG_ENOMEM, "side-by-side sweep: the %d-trajectory group's states do not "
                      "fit in HBM", G);
            break;
        }
        ms += cst.loop_ms;
        ieee += cst.ieee_diagonals;
        polls += cst.comm_polls;
        slow += cst.slow_diagonals;
        spins += cst.stall_spins;
        ++launches;
        // each domain's snapshot columns: 0 = w0, k = state k * snap_every
        hipEvent_t f0 = nullptr, f1 = nullptr;
        (void)hipEventCreate(&f0);
        (void)hipEventCreate(&f1);
        (void)hipEventRecord(f0, ch->stream);
        const int W = ch->sp.W;
        for (int j = 0; j < nb && rc == BURG_OK && (out.host || out.dev); ++j) {
            StreamArgs va = stream_args(ch, tr.map.L, tr.map.origin, 0, &tr.map);
            va.ring += (size_t)j * nti_d * ch->sp.ntj * (size_t)va.Lt * kWave;
            va.cf.ny = ny;
            va.nti = nti_d;
            va.ntiles = nti_d * ch->sp.ntj;
            if (out.dev) {
                double *dst = out.dev + (size_t)(g0 + j) * ncols;
                const int ldo = (int)out.ld_dev;
                const size_t cap = m * (size_t)out.ld_dev - (size_t)(g0 + j) * ncols;
                const double *p0 = c->d_w0;
                if (launch_transpose(&p0, 1, m, dst, ldo, cap, bflag(ch), ch->stream) ||
                    (ncols > 1 && launch_ring_extract(va, W, snap_every, snap_every, (int)(ncols - 1),
                                                      dst + 1, ldo, cap - 1, ch->stream)))
                    rc = fail(BURG_EHIP, "sweep snapshot extract failed");
                continue;
            }
            double *dst = out.host[g0 + j];
            const double *p0 = c->d_w0;
            for (int64_t k0 = 0; k0 < ncols && rc == BURG_OK; k0 += S) {
                const int cnt = (int)std::min<int64_t>(S, ncols - k0);
                int e = 0;
                if (k0 == 0) {
                    e = launch_transpose(&p0, 1, m, d_tr, S, (size_t)S * m, bflag(ch), ch->stream);
                    if (!e && cnt > 1)
                        e = launch_ring_extract(va, W, snap_every, snap_every, cnt - 1, d_tr + 1, S,
                                                (size_t)S * m - 1, ch->stream);
                } else {
                    e = launch_ring_extract(va, W, (int)(k0 * snap_every), snap_every, cnt, d_tr, S,
                                            (size_t)S * m, ch->stream);
                }
                if (e || d2h_2d(dst + k0, (size_t)out.ld_host * sizeof(double), d_tr,
                                (size_t)S * sizeof(double), (size_t)cnt * sizeof(double), m,
                                ch->stream) != hipSuccess ||
                    hipStreamSynchronize(ch->stream) != hipSuccess)
                    rc = fail(BURG_EHIP, "sweep snapshot copy failed");
            }
        }
        (void)hipEventRecord(f1, ch->stream);
        (void)hipEventSynchronize(f1);
        float t = 0.f;
        (void)hipEventElapsedTime(&t, f0, f1);
        flush_ms += t;
        (void)hipEventDestroy(f0);
        (void)hipEventDestroy(f1);
        if (rc == BURG_OK) rc = check_bounds(ch, "side-by-side sweep");
        if (rc == BURG_OK && g0 + nb == nmu) {
            // the last trajectory's final state becomes the parent's resident state
            const double *fs = ch->d_state[ch->cur] + (size_t)(nb - 1) * dpl;
            double *dstate = c->d_state[c->cur ^ 1];
            if (hipMemcpyAsync(dstate, fs, sizeof(double) * n, hipMemcpyDeviceToDevice, ch->stream) !=
                    hipSuccess ||
                hipMemcpyAsync(dstate + n, fs + nc, sizeof(double) * n, hipMemcpyDeviceToDevice,
                               ch->stream) != hipSuccess ||
                hipStreamSynchronize(ch->stream) != hipSuccess)
                rc = fail(BURG_EHIP, "resident state copy failed");
            else
                c->cur ^= 1;
        }
    }
    if (st) {
        st->steps = (int64_t)nmu * T;
        st->passes = st->steps;
        st->max_passes = 1;
        st->engine = BURG_ENGINE_PIPE;
        st->stream_w = ch->sp.W;
        st->stream_tiles = ch->sp.ntiles;
        st->loop_ms = ms;
        st->march_kernel_ms = ms;
        st->flush_ms = flush_ms;
        st->march_launches = launches;
        st->stream_launches = launches;
        st->ieee_diagonals = ieee;
        st->comm_polls = polls;
        st->slow_diagonals = slow;
        st->stall_spins = spins;
        st->tile_marches = (int64_t)nmu * T * (c->sp.ntiles > 0 ? c->sp.ntiles : 1);
    }
    cleanup();
    return rc;
}

static int sweep_impl(burg_ctx *c, int nmu, const double *src_b, const double *lbc_b,
                      int num_steps, const SweepOut &out, int snap_every, burg_stats *st)
{
    double *const *snaps = out.host;
    const int64_t ld_snaps = out.ld_host;
    if (int e = check_ready(c)) return e;
    if (st) std::memset(st, 0, sizeof *st);
    if (nmu < 1) return fail(BURG_EINVAL, "nmu must be >= 1");
    if (!src_b || !lbc_b) return fail(BURG_EINVAL, "null coefficient table");
    if (num_steps < 1) return fail(BURG_EINVAL, "num_steps must be >= 1");
    if (snap_every < 1) return fail(BURG_EINVAL, "snap_every must be >= 1");
    const int64_t ncols = num_steps / snap_every + 1;
    if (snaps) {
        if (ld_snaps < ncols)
            return fail(BURG_EINVAL, "ld_snaps=%lld < %lld columns", (long long)ld_snaps,
                        (long long)ncols);
        for (int j = 0; j < nmu; ++j)
            if (!snaps[j]) return fail(BURG_EINVAL, "null snapshot matrix %d", j);
    }
    if (out.dev) {
        if (out.ld_dev < (int64_t)nmu * ncols || out.ld_dev > INT32_MAX)
            return fail(BURG_EINVAL, "ld_out=%lld: need nmu * (num_steps / snap_every + 1) = %lld "
                        "columns", (long long)out.ld_dev, (long long)nmu * ncols);
        if (int e = check_device_ptr(c, out.dev, "out")) return e;
    }
    if (c->engine == BURG_ENGINE_TILES) return fail(BURG_EINVAL, "burg_sweep runs on the pipe engine");
    if (!c->d_w0) return fail(BURG_ESTATE, "burg_sweep: upload the initial state first");
    if (int e = stream_setup(c)) return e;
    if (c->eng_eff != BURG_ENGINE_PIPE)
        return fail(BURG_ESHAPE, "burg_sweep runs on the pipe engine; this %d x %d grid needs "
                    "the streaming engine's wider tiles", c->nx, c->nrows);
    {
        const int r = sweep_side_by_side(c, nmu, src_b, lbc_b, num_steps, snap_every, out, st);
        if (r <= 0) return r;  // done (or failed); 1: the serial sweep below
    }
    // narrow tiles run a group of trajectories per launch (the sweep kernel);
    // wide tiles one launch per trajectory with that mu's coefficient tables
    const bool narrow = pipe_sweep_width_supported(c->sp.W);
    if (narrow) {
        const int cap = pipe_max_resident_blocks(c->sp.W, true);
        if (cap < c->sp.nti * c->nwj)
            return fail(BURG_ESHAPE, "burg_sweep: %d workgroups of the sweep kernel cannot all be "
                        "resident (%d)", c->sp.nti * c->nwj, cap);
    }
    const int W = c->sp.W, T = num_steps;
    const size_t ncolp = (size_t)c->sp.ntj * W, m = c->m();
    // per-trajectory coefficient tables (this slab's rows of lbc)
    double *d_srcb = nullptr, *d_lbcb = nullptr, *d_tr = nullptr;
    d2 *d_colcb = nullptr;
    int rc = BURG_OK;
    auto cleanup = [&]() {
        c->sw_T = 0;
        c->sw_colc = nullptr;
        c->sw_lbc = nullptr;
        c->ov_colc = nullptr;
        c->ov_lbc = nullptr;
        (void)hipStreamSynchronize(c->stream);
        dfree(d_srcb);
        dfree(d_lbcb);
        dfree(d_colcb);
        dfree(d_tr);
    };
    if ((rc = dalloc(&d_srcb, (size_t)nmu * c->nx)) || (rc = dalloc(&d_lbcb, (size_t)nmu * c->nrows)) ||
        (rc = dalloc(&d_colcb, (size_t)nmu * ncolp))) {
        cleanup();
        return rc;
    }
    // (a failure from here on still goes through cleanup: no device buffer leaks)
    if (h2d(d_srcb, src_b, sizeof(double) * nmu * c->nx, c->stream) != hipSuccess ||
        h2d_2d(d_lbcb, sizeof(double) * c->nrows, lbc_b + c->row0, sizeof(double) * c->ny_total,
               sizeof(double) * c->nrows, nmu, c->stream) != hipSuccess ||
        launch_colc_batch(c->cf, nmu, d_srcb, (int)ncolp, d_colcb, c->stream) != 0) {
        rc = fail(BURG_EHIP, "burg_sweep: coefficient tables: %s", hipGetErrorString(hipGetLastError()));
        cleanup();
        return rc;
    }

    // trajectories per launch: as many as the ring budget (a third of free
    // HBM) holds -- the sweep's states all stay resident until extracted
    size_t freeb = 0, totalb = 0;
    HIPCHK(hipMemGetInfo(&freeb, &totalb));
    const size_t per_entry = (size_t)c->sp.ntiles * kWave * sizeof(d2);
    const long long Lmax = (long long)(freeb / 3 / per_entry);
    // (the paired sweep layout reaches 2 (8 K + 70) + 1 entries: L = K W + 2 W + 128)
    long long G = (Lmax - 2 * W - 128) / ((long long)T * W);
    G = std::min<long long>(G, nmu);
    G = std::min<long long>(G, stream_max_steps(c) / T);
    G = std::min<long long>(G, narrow ? kPipeSweepMax : 1);
    if (const char *e = std::getenv("BURG_SWEEP_GROUP")) {  // test knob: force grouping
        const long long v = std::atoll(e);
        if (v > 0) G = std::min(G, v);
    }
    if (G < 1) {
        cleanup();
        return fail(BURG_ENOMEM, "not enough device memory for one %d-step trajectory ring", T);
    }
    const long long L = G * T * W + 2 * W + 128;
    if ((rc = ensure_ring(c, L))) {
        cleanup();
        return rc;
    }
    int S = 0;
    if (snaps) {
        HIPCHK(hipMemGetInfo(&freeb, &totalb));
        S = (int)std::min<int64_t>(ncols, 64);
        while (S > 1 && (size_t)S * m * sizeof(double) > freeb / 3) S /= 2;
        if ((rc = dalloc(&d_tr, (size_t)S * m))) {
            cleanup();
            return rc;
        }
    }
    float ms = 0.f, flush_ms = 0.f;
    hipEvent_t f0 = nullptr, f1 = nullptr;
    (void)hipEventCreate(&f0);
    (void)hipEventCreate(&f1);
    stream_stats_begin(c);
    int64_t launches = 0;
    int last_nb = 0;
    for (int g0 = 0; g0 < nmu && rc == BURG_OK; g0 += (int)G) {
        const int nb = (int)std::min<long long>(G, nmu - g0);
        if ((rc = launch_ring_load(stream_args(c, L, 0, 0), W, c->d_w0, c->stream))) break;
        if (narrow) {
            c->sw_T = T;
            c->sw_colc = d_colcb + (size_t)g0 * ncolp;
            c->sw_lbc = d_lbcb + (size_t)g0 * c->nrows;
        } else {
            c->ov_colc = d_colcb + (size_t)g0 * ncolp;
            c->ov_lbc = d_lbcb + (size_t)g0 * c->nrows;
        }
        rc = stream_launch(c, L, 0, nb * T, &ms);
        // the launch's states as it laid them out (paired sweep layout or not)
        StreamArgs xa = stream_args(c, L, 0, 0);
        xa.play = c->last_play;
        c->sw_T = 0;
        c->ov_colc = nullptr;
        c->ov_lbc = nullptr;
        if (rc) break;
        ++launches;
        last_nb = nb;
        if (out.dev) {
            // straight into the device matrix: column 0 = w0, then the states
            for (int j = 0; j < nb && rc == BURG_OK; ++j) {
                double *dst = out.dev + (size_t)(g0 + j) * ncols;
                const size_t cap = m * (size_t)out.ld_dev - (size_t)(g0 + j) * ncols;
                const double *p0 = c->d_w0;
                if (launch_transpose(&p0, 1, m, dst, (int)out.ld_dev, cap, bflag(c), c->stream) ||
                    (ncols > 1 && launch_ring_extract(xa, W,
                                                      (int)(j * T + snap_every), snap_every,
                                                      (int)(ncols - 1), dst + 1, (int)out.ld_dev,
                                                      cap - 1, c->stream)))
                    rc = fail(BURG_EHIP, "snapshot extract failed");
            }
            continue;
        }
        if (!snaps) continue;
        (void)hipEventRecord(f0, c->stream);
        for (int j = 0; j < nb && rc == BURG_OK; ++j) {
            double *dst = snaps[g0 + j];
            // column 0 = the initial state
            if (d2h_2d(dst, (size_t)ld_snaps * sizeof(double), c->d_w0, sizeof(double),
                       sizeof(double), m, c->stream) != hipSuccess) {
                rc = fail(BURG_EHIP, "snapshot copy failed");
                break;
            }
            // columns 1.. = launch states j*T + k*snap_every
            for (int64_t k0 = 1; k0 < ncols; k0 += S) {
                const int n = (int)std::min<int64_t>(S, ncols - k0);
                if (launch_ring_extract(xa, W,
                                        (int)(j * T + k0 * snap_every), snap_every, n, d_tr, n,
                                        (size_t)S * m, c->stream) ||
                    d2h_2d(dst + k0, (size_t)ld_snaps * sizeof(double), d_tr,
                           n * sizeof(double), n * sizeof(double), m, c->stream) != hipSuccess) {
                    rc = fail(BURG_EHIP, "snapshot extract failed");
                    break;
                }
            }
        }
        (void)hipEventRecord(f1, c->stream);
        (void)hipEventSynchronize(f1);
        float t = 0.f;
        (void)hipEventElapsedTime(&t, f0, f1);
        flush_ms += t;
    }
    if (rc == BURG_OK) {
        // the last trajectory's final state becomes the resident state
        StreamArgs fa = stream_args(c, L, 0, 0);
        fa.play = c->last_play;
        rc = launch_ring_extract(fa, W, last_nb * T, 1, 1,
                                 c->d_state[c->cur ^ 1], 1, m, c->stream);
        if (rc) rc = fail(BURG_EHIP, "ring extract launch failed");
        else c->cur ^= 1;
    }
    if (rc == BURG_OK) rc = check_bounds(c, "burg_sweep");
    if (rc == BURG_OK) rc = stream_stats_end(c, st, (int64_t)nmu * T, launches);
    if (st) {
        st->loop_ms = ms;
        st->flush_ms = flush_ms;
        st->march_kernel_ms = ms;
        st->march_launches = launches;
    }
    (void)hipEventDestroy(f0);
    (void)hipEventDestroy(f1);
    cleanup();
    return rc;
}

int burg_sweep(burg_ctx *c, int nmu, const double *src_b, const double *lbc_b, int num_steps,
               double *const *snaps, int64_t ld_snaps, int snap_every, burg_stats *st)
{
    BURG_TRACE("burg_sweep");
    SweepOut so;
    so.host = snaps;
    so.ld_host = ld_snaps;
    return sweep_impl(c, nmu, src_b, lbc_b, num_steps, so, snap_every, st);
}

int burg_sweep_device(burg_ctx *c, int nmu, const double *src_b, const double *lbc_b,
                      int num_steps, int snap_every, double *d_out, int64_t ld_out,
                      burg_stats *st)
{
    BURG_TRACE("burg_sweep_device");
    if (!d_out) return fail(BURG_EINVAL, "null output");
    SweepOut so;
    so.dev = d_out;
    so.ld_dev = ld_out;
    return sweep_impl(c, nmu, src_b, lbc_b, num_steps, so, snap_every, st);
}

int burg_ecsw_matrix(burg_ctx *c, int n_snaps, const double *states, const double *prev_states,
                     int n_pod, const double *basis, double *C, burg_stats *st)
{
    BURG_TRACE("burg_ecsw_matrix");
    if (int e = check_ready(c)) return e;
    if (st) std::memset(st, 0, sizeof *st);
    if (n_snaps < 1 || n_pod < 1) return fail(BURG_EINVAL, "n_snaps and n_pod must be >= 1");
    if (!states || !prev_states || !basis || !C) return fail(BURG_EINVAL, "null array");
    if (c->world > 1) return fail(BURG_EINVAL, "burg_ecsw_matrix: single-GPU contexts only");
    const size_t m = c->m(), n = c->n();
    const size_t blk = (size_t)n_pod * n;  // one snapshot's C rows
    double *d_b = nullptr, *d_bt = nullptr, *d_w = nullptr, *d_cb = nullptr;
    int rc = BURG_OK;
    auto cleanup = [&]() {
        (void)hipStreamSynchronize(c->stream);
        dfree(d_b);
        dfree(d_bt);
        dfree(d_w);
        dfree(d_cb);
    };
    if ((rc = dalloc(&d_b, m * n_pod)) || (rc = dalloc(&d_bt, m * n_pod)) ||
        (rc = dalloc(&d_w, 2 * m)) || (rc = dalloc(&d_cb, blk))) {
        cleanup();
        return rc;
    }
    if (h2d(d_b, basis, sizeof(double) * m * n_pod, c->stream) != hipSuccess ||
        launch_basis_transpose(d_b, d_bt, m, n_pod, c->stream) != 0) {
        rc = fail(BURG_EHIP, "burg_ecsw_matrix: basis upload: %s", hipGetErrorString(hipGetLastError()));
        cleanup();
        return rc;
    }
    float kern = 0.f, copy = 0.f;
    hipEvent_t e2 = nullptr;
    (void)hipEventCreate(&e2);
    for (int i = 0; i < n_snaps && rc == BURG_OK; ++i) {
        if (h2d(d_w, states + (size_t)i * m, sizeof(double) * m, c->stream) != hipSuccess ||
            h2d(d_w + m, prev_states + (size_t)i * m, sizeof(double) * m, c->stream) != hipSuccess) {
            rc = fail(BURG_EHIP, "state upload failed");
            break;
        }
        (void)hipEventRecord(c->ev0, c->stream);
        if (launch_ecsw(c->cf, d_w, d_w + m, d_bt, n_pod, d_cb, c->stream)) {
            rc = fail(BURG_EHIP, "ecsw kernel launch failed");
            break;
        }
        (void)hipEventRecord(c->ev1, c->stream);
        if (d2h(C + (size_t)i * blk, d_cb, sizeof(double) * blk, c->stream) != hipSuccess) {
            rc = fail(BURG_EHIP, "C block copy failed");
            break;
        }
        (void)hipEventRecord(e2, c->stream);
        if (hipEventSynchronize(e2) != hipSuccess) {
            rc = fail(BURG_EHIP, "ecsw: %s", hipGetErrorString(hipGetLastError()));
            break;
        }
        float t = 0.f;
        (void)hipEventElapsedTime(&t, c->ev0, c->ev1);
        kern += t;
        (void)hipEventElapsedTime(&t, c->ev1, e2);
        copy += t;
    }
    (void)hipEventDestroy(e2);
    if (st) {
        st->loop_ms = kern;
        st->flush_ms = copy;
        st->steps = n_snaps;
    }
    cleanup();
    return rc;
}

// `p` must be device memory of the context's GPU (not host, not another GPU):
// the ECSW block entry reads and writes through it from a kernel
static int check_device_ptr(const burg_ctx *c, const void *p, const char *what)
{
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return fail(BURG_EINVAL, "%s: not a HIP allocation", what);
    }
    if (at.type != hipMemoryTypeDevice || at.device != c->device)
        return fail(BURG_EINVAL, "%s: not device memory of GPU %d", what, c->device);
    return BURG_OK;
}

int burg_ecsw_block_device(burg_ctx *c, const double *d_state, const double *d_prev, int n_pod,
                           const double *d_basis_t, double *d_C, float *kernel_ms)
{
    BURG_TRACE("burg_ecsw_block_device");
    if (int e = check_ready(c)) return e;
    if (kernel_ms) *kernel_ms = 0.f;
    if (n_pod < 1) return fail(BURG_EINVAL, "n_pod must be >= 1");
    if (!d_state || !d_prev || !d_basis_t || !d_C) return fail(BURG_EINVAL, "null array");
    if (c->world > 1) return fail(BURG_EINVAL, "burg_ecsw_block_device: single-GPU contexts only");
    if (int e = check_device_ptr(c, d_state, "state")) return e;
    if (int e = check_device_ptr(c, d_prev, "prev_state")) return e;
    if (int e = check_device_ptr(c, d_basis_t, "basis_t")) return e;
    if (int e = check_device_ptr(c, d_C, "C")) return e;
    HIPCHK(hipEventRecord(c->ev0, c->stream));
    if (launch_ecsw(c->cf, d_state, d_prev, d_basis_t, n_pod, d_C, c->stream))
        return fail(BURG_EHIP, "ecsw kernel launch failed");
    HIPCHK(hipEventRecord(c->ev1, c->stream));
    if (hipEventSynchronize(c->ev1) != hipSuccess)
        return fail(BURG_EHIP, "ecsw: %s", hipGetErrorString(hipGetLastError()));
    if (kernel_ms) (void)hipEventElapsedTime(kernel_ms, c->ev0, c->ev1);
    return BURG_OK;
}

int burg_run(burg_ctx *c, const double *w0, int num_steps, int solver, int newton_max_its,
             double newton_rtol, double *snaps, int64_t ld_snaps, int snap_every,
             burg_stats *st, int32_t *step_iters, double *step_rel)
{
    BURG_TRACE("burg_run");
    if (int e = check_ready(c)) return e;
    if (!w0) return fail(BURG_EINVAL, "null w0");
    if (num_steps < 0) return fail(BURG_EINVAL, "num_steps < 0");
    if (snap_every < 1) return fail(BURG_EINVAL, "snap_every must be >= 1");
    if (solver != BURG_SOLVER_MARCH && solver != BURG_SOLVER_NEWTON)
        return fail(BURG_EINVAL, "unknown solver %d", solver);
    const int64_t ncols = num_steps / snap_every + 1;
    if (snaps && ld_snaps < ncols)
        return fail(BURG_EINVAL, "ld_snaps=%lld < %lld columns", (long long)ld_snaps,
                    (long long)ncols);
    if (newton_max_its < 0) return fail(BURG_EINVAL, "newton_max_its < 0");
    if (st) std::memset(st, 0, sizeof *st);
    if (solver == BURG_SOLVER_MARCH && c->engine != BURG_ENGINE_TILES)
        return stream_run(c, w0, num_steps, snaps, ld_snaps, snap_every, st, step_iters,
                          step_rel);
    if (int e = ensure_scratch(c)) return e;
    const size_t m = c->m(), bytes = m * sizeof(double);

    // snapshot chunk: up to S device states, transposed into (m x S) and
    // copied as a 2D block into columns [col0, col0+S) of the host matrix.
    int S = 0;
    double *d_chunk = nullptr, *d_tr = nullptr;
    if (snaps) {
        size_t freeb = 0, totalb = 0;
        HIPCHK(hipMemGetInfo(&freeb, &totalb));
        const size_t budget = freeb / 4;
        S = (int)std::min<int64_t>(ncols, 64);
        while (S > 1 && (size_t)S * 2 * bytes > budget) S /= 2;
        if (int e = dalloc(&d_chunk, (size_t)S * m)) return e;
        if (int e = dalloc(&d_tr, (size_t)S * m)) {
            dfree(d_chunk);
            return e;
        }
    }
    std::vector<const double *> slots;
    int64_t col0 = 0;
    float flush_ms = 0.f;
    hipEvent_t f0 = nullptr, f1 = nullptr;
    (void)hipEventCreate(&f0);
    (void)hipEventCreate(&f1);
    auto flush = [&]() -> int {
        if (slots.empty()) return 0;
        HIPCHK(hipEventRecord(f0, c->stream));
        CHK(launch_transpose(slots.data(), (int)slots.size(), m, d_tr, (int)slots.size(),
                             (size_t)S * m, bflag(c), c->stream));
        HIPCHK(d2h_2d(snaps + col0, (size_t)ld_snaps * sizeof(double), d_tr,
                      slots.size() * sizeof(double), slots.size() * sizeof(double), m, c->stream));
        HIPCHK(hipEventRecord(f1, c->stream));
        HIPCHK(hipEventSynchronize(f1));
        float t = 0.f;
        (void)hipEventElapsedTime(&t, f0, f1);
        flush_ms += t;
        col0 += (int64_t)slots.size();
        slots.clear();
        return 0;
    };
    auto keep = [&](const double *state) -> int {
        double *slot = d_chunk + slots.size() * m;
        HIPCHK(hipMemcpyAsync(slot, state, bytes, hipMemcpyDeviceToDevice, c->stream));
        slots.push_back(slot);
        if ((int)slots.size() == S) return flush();
        return 0;
    };

    int rc = BURG_OK;
    HIPCHK(hipMemsetAsync(c->d_stats, 0, sizeof(DevStats), c->stream));
    HIPCHK(h2d(c->d_state[c->cur], w0, bytes, c->stream));
    if (snaps) rc = keep(c->d_state[c->cur]);
    int64_t nupd = 0;
    int maxupd = 0;
    double rel = 0.0;
    float loop_ms = 0.f;
    long long prev_passes = 0;
    for (int s = 0; s < num_steps && rc == BURG_OK; ++s) {
        HIPCHK(hipEventRecord(c->ev0, c->stream));
        const double *wp = c->d_state[c->cur];
        double *w = c->d_state[c->cur ^ 1];
        if (solver == BURG_SOLVER_MARCH) {
            rc = march_step(c, wp, w);
            if (step_iters && rc == BURG_OK) {
                // passes of this step = max_passes delta of a one-step stats window
                DevStats ds{};
                HIPCHK(hipMemcpyAsync(&ds, c->d_stats, sizeof ds, hipMemcpyDeviceToHost,
                                      c->stream));
                HIPCHK(hipStreamSynchronize(c->stream));
                step_iters[s] = (int32_t)(ds.passes - prev_passes);
                prev_passes = ds.passes;
            }
            if (step_rel) step_rel[s] = 0.0;
        } else {
            int its = 0;
            rc = newton_step(c, wp, w, newton_max_its, newton_rtol, &its, &rel);
            nupd += its;
            maxupd = std::max(maxupd, its);
            if (step_iters) step_iters[s] = its;
            if (step_rel) step_rel[s] = rel;
        }
        HIPCHK(hipEventRecord(c->ev1, c->stream));
        c->cur ^= 1;
        if (rc == BURG_OK && snaps && (s + 1) % snap_every == 0) {
            HIPCHK(hipEventSynchronize(c->ev1));
            float t = 0.f;
            (void)hipEventElapsedTime(&t, c->ev0, c->ev1);
            loop_ms += t;
            rc = keep(c->d_state[c->cur]);
        } else if (rc == BURG_OK) {
            HIPCHK(hipEventSynchronize(c->ev1));
            float t = 0.f;
            (void)hipEventElapsedTime(&t, c->ev0, c->ev1);
            loop_ms += t;
        }
    }
    if (rc == BURG_OK && snaps) rc = flush();
    if (rc == BURG_OK) rc = check_bounds(c, "burg_run");
    if (rc == BURG_OK) rc = read_stats(c, st);
    if (st) {
        st->loop_ms = loop_ms;
        st->flush_ms = flush_ms;
        st->newton_updates = nupd;
        st->newton_max_updates = maxupd;
        st->last_rel = rel;
        if (solver == BURG_SOLVER_NEWTON) st->steps = num_steps;
    }
    collect_profile(c, st);
    (void)hipStreamSynchronize(c->stream);
    dfree(d_chunk);
    dfree(d_tr);
    (void)hipEventDestroy(f0);
    (void)hipEventDestroy(f1);
    if (rc == BURG_OK && st && st->unconverged_steps > 0)
        return fail(BURG_ENOCONV, "%d steps hit the pass cap", st->unconverged_steps);
    return rc;
}

// The .npy header np.save writes for a C-order float64 (m, ncols) array
// (format 1.0: magic, version, little-endian header length, the dict padded
// with spaces to a 64-byte boundary, newline).
static std::string npy_header(size_t m, size_t ncols)
{
    std::string d = "{'descr': '<f8', 'fortran_order': False, 'shape': (" + std::to_string(m) +
                    ", " + std::to_string(ncols) + "), }";
    size_t total = 10 + d.size() + 1;
    const size_t pad = (64 - total % 64) % 64;
    d.append(pad, ' ');
    d.push_back('\n');
    std::string h("\x93NUMPY\x01\x00", 8);
    const unsigned short hl = (unsigned short)d.size();
    h.push_back((char)(hl & 0xff));
    h.push_back((char)(hl >> 8));
    return h + d;
}

// burg_run_npy: one trajectory, its snapshot matrix written straight into a
// .npy file (load_or_compute_snaps' cache, C/hypernet2D.py:3141-3143; np.save
// in run_fom.main's timed region, C/run_fom.py:41-43).  The trajectory stays
// in the HBM ring; row blocks of the C-order matrix are gathered on the
// device, copied into a pool of pinned host buffers and written at their file
// offsets (pwrite) by writer threads while the next blocks are gathered and
// copied.  One writer by default: buffered writes into one file serialise on
// the file (the GPU box's host: 11 GB/s with 1 thread, 10-11 with 2-8;
// memcpy into a shared mapping 3-7 GB/s; profiles/r05/ab/npy), so the call
// runs at that rate.  Like np.save, the file is left in the page cache (no
// fsync; BURG_NPY_FSYNC=1 adds one -- 0.75 -> 1.35 s at 1024^2 x 500).
int burg_run_npy(burg_ctx *c, const double *w0, int num_steps, int snap_every, const char *path,
                 burg_stats *st)
{
    return burg_run_npy_ex(c, w0, num_steps, snap_every, path, 0, st);
}

// burg_run_npy_ex: the same, with BURG_NPY_GLOBAL -- a slab context writes
// its rows at their places in the WHOLE grid's (2 nx ny_total, ncols) matrix:
// its u rows at global rows row0 nx ..., its v rows at nx ny_total + row0 nx
// ... (the reference layout, C/hypernet2D.py:89-90,126; SURVEY.md 8(e): "each
// GPU copies its slab rows directly into the right rows") -- and
// BURG_NPY_EXISTING -- the file exists already, made by one rank with the
// whole matrix's header and size (checked here), and is neither truncated nor
// given a header, so every rank of a job writes into the same file at once.
int burg_run_npy_ex(burg_ctx *c, const double *w0, int num_steps, int snap_every, const char *path,
                    int flags, burg_stats *st)
{
    BURG_TRACE("burg_run_npy");
    if (int e = check_ready(c)) return e;
    if (st) std::memset(st, 0, sizeof *st);
    if (!w0 || !path || !*path) return fail(BURG_EINVAL, "null w0 or path");
    if (num_steps < 1 || snap_every < 1) return fail(BURG_EINVAL, "num_steps, snap_every >= 1");
    if (flags & ~(BURG_NPY_GLOBAL | BURG_NPY_EXISTING)) return fail(BURG_EINVAL, "unknown flags %#x", flags);
    if (c->engine == BURG_ENGINE_TILES) return fail(BURG_EINVAL, "burg_run_npy runs on the stream/pipe engines");
    if (int e = stream_setup(c)) return e;
    if (num_steps > stream_max_steps(c))
        return fail(BURG_EINVAL, "num_steps %d exceeds one launch (%d)", num_steps, stream_max_steps(c));
    const int W = c->sp.W;
    const size_t m = c->m();
    const int64_t ncols = num_steps / snap_every + 1;
    // the file's matrix and where this context's rows go: local row e < n is
    // u row e, at file row urow0 + e; e >= n at vrow0 + e - n
    const bool global = (flags & BURG_NPY_GLOBAL) != 0;
    const size_t nloc = c->n();
    const size_t n_file = global ? (size_t)c->nx * c->ny_total : nloc;
    const size_t m_file = 2 * n_file;
    const size_t urow0 = global ? (size_t)c->row0 * c->nx : 0;
    const size_t vrow0 = n_file + urow0;
    const long long L = (long long)num_steps * W + W + 96;
    const size_t per_entry = (size_t)c->sp.ntiles * kWave * sizeof(d2);
    size_t freeb = 0, totalb = 0;
    HIPCHK(hipMemGetInfo(&freeb, &totalb));
    const size_t need = (size_t)L * per_entry, have = c->ring_entries * sizeof(d2);
    if (need > have && need > (freeb + have) / 100 * 85)
        return fail(BURG_ENOMEM, "the %d-step trajectory (%.1f GB of ring) does not fit in HBM; "
                    "use burg_run", num_steps, (double)need / 1e9);
    if (int e = ensure_ring(c, L)) return e;
    // row blocks: about 32 MB each (at least one row); NW writer threads
    // (BURG_NPY_WRITERS, default 1), max(4, 2 NW) pinned buffers
    const size_t row_bytes = (size_t)ncols * sizeof(double);
    size_t R = std::max<size_t>(1, ((size_t)32 << 20) / row_bytes);
    if (const char *e = std::getenv("BURG_NPY_BLOCK_ROWS")) {  // test knob: force many blocks
        const long long v = std::atoll(e);
        if (v > 0) R = std::min(R, (size_t)v);
    }
    R = std::min(R, m);
    int NW = 1;
    if (const char *e = std::getenv("BURG_NPY_WRITERS")) NW = std::max(1, std::min(16, std::atoi(e)));
    const int NBUF = std::max(4, 2 * NW);
    const bool want_fsync = [] {
        const char *e = std::getenv("BURG_NPY_FSYNC");
        return e && std::atoi(e) != 0;
    }();
    double *d_blk = nullptr;
    std::vector<double *> h_blk(NBUF, nullptr);
    int fd = -1;
    int rc = BURG_OK;
    std::vector<std::thread> writers;
    std::mutex mu;
    std::condition_variable cv;
    struct Job {
        int buf;
        off_t off;
        size_t bytes;
    };
    std::vector<Job> jobs;     // filled buffers waiting for a writer
    std::vector<int> free_buf;  // buffers the device may copy into
    bool stop = false, werr = false;
    int werrno = 0;
    auto cleanup = [&]() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto &t : writers)
            if (t.joinable()) t.join();
        (void)hipStreamSynchronize(c->stream);
        dfree(d_blk);
        for (auto &h : h_blk)
            if (h) (void)hipHostFree(h), h = nullptr;
        if (fd >= 0) close(fd);
    };
    if ((rc = dalloc(&d_blk, 2 * R * (size_t)ncols))) return rc;
    for (int i = 0; i < NBUF; ++i) {
        if (hipHostMalloc((void **)&h_blk[i], R * row_bytes, hipHostMallocDefault) != hipSuccess) {
            cleanup();
            return fail(BURG_ENOMEM, "pinned staging buffers (%d x %zu bytes)", NBUF, R * row_bytes);
        }
        free_buf.push_back(i);
    }
    const std::string hdr = npy_header(m_file, (size_t)ncols);
    const off_t file_bytes = (off_t)(hdr.size() + m_file * row_bytes);
    if (flags & BURG_NPY_EXISTING) {
        // another rank made the file: it must already be this matrix's
        fd = open(path, O_RDWR);
        if (fd < 0) {
            cleanup();
            return fail(BURG_EINVAL, "open(%s): %s", path, strerror(errno));
        }
        std::string got(hdr.size(), '\0');
        struct stat sb {};
        if (pread(fd, &got[0], got.size(), 0) != (ssize_t)got.size() || got != hdr ||
            fstat(fd, &sb) != 0 || sb.st_size < file_bytes) {
            cleanup();
            return fail(BURG_EINVAL, "%s is not a (%zu, %lld) float64 .npy of %lld bytes made for this "
                        "trajectory (BURG_NPY_EXISTING)", path, m_file, (long long)ncols,
                        (long long)file_bytes);
        }
    } else {
        fd = open(path, O_CREAT | O_TRUNC | O_WRONLY, 0644);
        if (fd < 0) {
            cleanup();
            return fail(BURG_EINVAL, "open(%s): %s", path, strerror(errno));
        }
        if (write(fd, hdr.data(), hdr.size()) != (ssize_t)hdr.size() ||
            (global && ftruncate(fd, file_bytes) != 0)) {
            cleanup();
            return fail(BURG_EINVAL, "write(%s): %s", path, strerror(errno));
        }
    }
    for (int w = 0; w < NW; ++w)
        writers.emplace_back([&]() {
            for (;;) {
                Job j;
                {
                    std::unique_lock<std::mutex> g(mu);
                    cv.wait(g, [&] { return !jobs.empty() || stop; });
                    if (jobs.empty()) return;
                    j = jobs.back();
                    jobs.pop_back();
                }
                const char *p = (const char *)h_blk[j.buf];
                size_t left = j.bytes;
                off_t off = j.off;
                bool ok = true;
                int en = 0;
                while (left > 0) {
                    const ssize_t wr = pwrite(fd, p, left, off);
                    if (wr <= 0) {
                        ok = false;
                        en = errno;
                        break;
                    }
                    p += wr;
                    off += wr;
                    left -= (size_t)wr;
                }
                {
                    std::lock_guard<std::mutex> g(mu);
                    if (!ok && !werr) werr = true, werrno = en;
                    free_buf.push_back(j.buf);
                }
                cv.notify_all();
            }
        });

    // the trajectory: one launch, every state in the ring
    const auto t_start = std::chrono::steady_clock::now();
    stream_stats_begin(c);
    HIPCHK(h2d(c->d_state[c->cur], w0, m * sizeof(double), c->stream));
    CHK(launch_ring_load(stream_args(c, L, 0, 0), W, c->d_state[c->cur], c->stream));
    float ms = 0.f;
    if ((rc = stream_launch(c, L, 0, num_steps, &ms))) {
        cleanup();
        return rc;
    }
    // row blocks -> pinned buffers -> writer pool -> file
    float flush_ms = 0.f;
    hipEvent_t f0 = nullptr, f1 = nullptr;
    (void)hipEventCreate(&f0);
    (void)hipEventCreate(&f1);
    // a buffer taken off free_buf goes back on every failure path, so the
    // drain below (every buffer free again) always ends
    auto give_back = [&](int b) {
        {
            std::lock_guard<std::mutex> g(mu);
            free_buf.push_back(b);
        }
        cv.notify_all();
    };
    // test knob: the copy of row block BURG_TEST_FAIL_NPY_BLOCK (0-based)
    // fails as a faulted gather or D2H would (tests/test_gpu_parity.py)
    long long fail_blk = -1;
    if (const char *e = std::getenv("BURG_TEST_FAIL_NPY_BLOCK")) fail_blk = std::atoll(e);
    int di = 0;  // device gather buffer (two, alternating)
    long long blk = 0;
    // (a block stays inside the u rows or inside the v rows: the two land in
    // different places of a global file)
    for (size_t e0 = 0, ne = 0; e0 < m && rc == BURG_OK; e0 += ne, di ^= 1, ++blk) {
        ne = std::min(R, (e0 < nloc ? nloc : m) - e0);
        const size_t frow = e0 < nloc ? urow0 + e0 : vrow0 + (e0 - nloc);
        int b = -1;
        {
            std::unique_lock<std::mutex> g(mu);
            cv.wait(g, [&] { return !free_buf.empty() || werr; });
            if (werr) break;
            b = free_buf.back();
            free_buf.pop_back();
        }
        double *dst = d_blk + (size_t)di * R * ncols;
        (void)hipEventRecord(f0, c->stream);
        if (blk == fail_blk ||
            launch_ring_extract_rows(stream_args(c, L, 0, 0), W, e0, ne, 0, snap_every, (int)ncols,
                                     dst, R * (size_t)ncols, c->stream) ||
            hipMemcpyAsync(h_blk[b], dst, ne * row_bytes, hipMemcpyDeviceToHost, c->stream) !=
                hipSuccess) {
            give_back(b);
            rc = fail(BURG_EHIP, "snapshot row block copy failed (rows %zu..%zu)", e0, e0 + ne);
            break;
        }
        (void)hipEventRecord(f1, c->stream);
        if (hipEventSynchronize(f1) != hipSuccess) {
            give_back(b);
            rc = fail(BURG_EHIP, "snapshot row block copy failed: %s", hipGetErrorString(hipGetLastError()));
            break;
        }
        float t = 0.f;
        (void)hipEventElapsedTime(&t, f0, f1);
        flush_ms += t;
        {
            std::lock_guard<std::mutex> g(mu);
            jobs.push_back({b, (off_t)(hdr.size() + frow * row_bytes), ne * row_bytes});
        }
        cv.notify_all();
    }
    // drain the writers
    {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return (int)free_buf.size() == NBUF || (werr && jobs.empty()); });
    }
    if (werr && rc == BURG_OK) rc = fail(BURG_EINVAL, "write(%s) failed: %s", path, strerror(werrno));
    if (rc == BURG_OK && want_fsync) (void)fsync(fd);  // (not fatal: page cache is enough for np.load)
    const double wall_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    if (rc == BURG_OK) {
        const long long o_last = 0;
        rc = launch_ring_extract(stream_args(c, L, o_last, 0), W, num_steps, 1, 1,
                                 c->d_state[c->cur ^ 1], 1, m, c->stream);
        if (rc) rc = fail(BURG_EHIP, "ring extract launch failed");
        else c->cur ^= 1;
    }
    if (rc == BURG_OK) rc = check_bounds(c, "burg_run_npy");
    if (rc == BURG_OK) rc = stream_stats_end(c, st, num_steps, 1);
    if (st) {
        st->loop_ms = ms;
        st->flush_ms = flush_ms;
        st->march_kernel_ms = wall_ms;  // whole call (trajectory + write), wall clock
        st->march_launches = 1;
    }
    (void)hipEventDestroy(f0);
    (void)hipEventDestroy(f1);
    cleanup();
    return rc;
}

// LSPG PROM (C/hypernet2D.py:133-200 + gauss_newton_LSPG :1859-1929), lspg.hip.
// Device-resident: basis in (npod, 2n) planes and their transposes, state w
// and its transpose, y; the host sees only the residual norm per iteration
// (the reference's stopping tests) and the kept snapshots.
int burg_lspg(burg_ctx *c, const double *w0, int num_steps, int n_pod, const double *basis,
              int max_its, double relnorm_cutoff, double min_delta, double *snaps,
              int64_t ld_snaps, double *red_coords, int64_t ld_red, int32_t *step_its,
              double *step_rel, double *times_ms, burg_stats *st)
{
    BURG_TRACE("burg_lspg");
    if (int e = check_ready(c)) return e;
    if (st) std::memset(st, 0, sizeof *st);
    if (times_ms) times_ms[0] = times_ms[1] = times_ms[2] = 0.0;
    if (!w0 || !basis) return fail(BURG_EINVAL, "null w0 or basis");
    if (c->world > 1) return fail(BURG_EINVAL, "burg_lspg: single-GPU contexts only");
    if (c->nx != c->ny_total)
        return fail(BURG_ESHAPE, "burg_lspg: the LSPG Jacobian (row-only JDyec permutation, "
                                 "C/hypernet2D.py:165-167) needs nx == ny");
    if (n_pod < 1 || n_pod > kLspgMaxPod)
        return fail(BURG_EINVAL, "n_pod=%d outside [1, %d]", n_pod, kLspgMaxPod);
    if (num_steps < 0 || max_its < 1) return fail(BURG_EINVAL, "num_steps < 0 or max_its < 1");
    if (snaps && ld_snaps < num_steps + 1) return fail(BURG_EINVAL, "ld_snaps < num_steps + 1");
    if (red_coords && ld_red < num_steps + 1) return fail(BURG_EINVAL, "ld_red < num_steps + 1");
    if (int e = ensure_scratch(c)) return e;
    const size_t m = c->m(), n = c->n();
    const int N = c->nx;
    const int P = lspg_cols(n_pod);
    double *d_b = nullptr, *d_bt = nullptr, *d_btT = nullptr, *d_bk = nullptr, *d_w = nullptr,
           *d_wT = nullptr,
           *d_wp = nullptr, *d_y = nullptr, *d_part = nullptr, *d_G = nullptr, *d_chunk = nullptr,
           *d_tr = nullptr;
    unsigned *d_err = nullptr;
    int *d_info = nullptr;
    double *d_d0 = nullptr;
    rocblas_handle rh = nullptr;
    // solver of the npod x npod normal equations: our one-workgroup kernel or
    // rocSOLVER potrf/potrs (BURG_LSPG_SOLVE=kernel|lib)
    const char *solve_env = getenv("BURG_LSPG_SOLVE");
    const bool lib_solve = !(solve_env && std::strcmp(solve_env, "kernel") == 0);
    std::vector<hipEvent_t> evs;
    auto cleanup = [&]() {
        (void)hipStreamSynchronize(c->stream);
        if (rh) rocblas_destroy_handle(rh);
        dfree(d_info), dfree(d_d0);
        for (auto e : evs) (void)hipEventDestroy(e);
        dfree(d_b), dfree(d_bt), dfree(d_btT), dfree(d_bk), dfree(d_w), dfree(d_wT), dfree(d_wp), dfree(d_y);
        dfree(d_part), dfree(d_G), dfree(d_err), dfree(d_chunk), dfree(d_tr);
    };
    int rc = BURG_OK;
#define LCHK(expr)                  \
    do {                            \
        if ((rc = (expr)) != 0) {   \
            cleanup();              \
            return rc;              \
        }                           \
    } while (0)
#define LHIP(expr)                                                                     \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            rc = fail(BURG_EHIP, "burg_lspg: %s: %s", #expr, hipGetErrorString(e_));   \
            cleanup();                                                                 \
            return rc;                                                                 \
        }                                                                              \
    } while (0)
#define LLAUNCH(expr)                                                                  \
    do {                                                                               \
        if ((expr) != 0) {                                                             \
            rc = fail(BURG_EHIP, "burg_lspg: launch %s: %s", #expr,                    \
                      hipGetErrorString(hipGetLastError()));                           \
            cleanup();                                                                 \
            return rc;                                                                 \
        }                                                                              \
    } while (0)
    LCHK(dalloc(&d_b, m * n_pod));
    LCHK(dalloc(&d_bt, m * n_pod));
    LHIP(h2d(d_b, basis, sizeof(double) * m * n_pod, c->stream));
    LLAUNCH(launch_basis_transpose(d_b, d_bt, m, n_pod, c->stream));
    LHIP(hipStreamSynchronize(c->stream));
    dfree(d_b);
    LCHK(dalloc(&d_btT, m * n_pod));
    for (int p = 0; p < 2 * n_pod; ++p)
        LLAUNCH(launch_basis_transpose(d_bt + (size_t)p * n, d_btT + (size_t)p * n, N, N,
                                       c->stream));
    if (lspg_gram_blocked(n_pod)) {
        LCHK(dalloc(&d_bk, lspg_blocked_count(n, n_pod)));
        LLAUNCH(launch_lspg_block_basis(d_bt, d_btT, n, n_pod, d_bk, c->stream));
    }
    LCHK(dalloc(&d_w, m));
    LCHK(dalloc(&d_wT, m));
    LCHK(dalloc(&d_wp, m));
    LCHK(dalloc(&d_y, (size_t)kLspgMaxPod + 1));
    LCHK(dalloc(&d_part, lspg_partial_count(N, n_pod)));
    LCHK(dalloc(&d_G, (size_t)P * P));
    LCHK(dalloc(&d_err, 1));
    LHIP(hipMemsetAsync(d_err, 0, sizeof(unsigned), c->stream));
    if (lib_solve) {
        LCHK(dalloc(&d_info, 1));
        LCHK(dalloc(&d_d0, (size_t)P));
        if (rocblas_create_handle(&rh) != rocblas_status_success) {
            rc = fail(BURG_EHIP, "burg_lspg: rocblas_create_handle failed");
            cleanup();
            return rc;
        }
        rocblas_set_stream(rh, c->stream);
    }

    // kept snapshots: S states at a time, transposed into the C-order columns
    int S = 0;
    std::vector<const double *> slots;
    int64_t col0 = 0;
    float flush_ms = 0.f;
    if (snaps) {
        size_t freeb = 0, totalb = 0;
        LHIP(hipMemGetInfo(&freeb, &totalb));
        S = (int)std::min<int64_t>(num_steps + 1, 64);
        while (S > 1 && (size_t)S * 2 * m * sizeof(double) > freeb / 4) S /= 2;
        LCHK(dalloc(&d_chunk, (size_t)S * m));
        LCHK(dalloc(&d_tr, (size_t)S * m));
    }
    std::vector<double> yh((size_t)n_pod);
    for (int k = 0; k < 8; ++k) {
        hipEvent_t e = nullptr;
        LHIP(hipEventCreate(&e));
        evs.push_back(e);
    }
    float t_jac = 0.f, t_res = 0.f, t_ls = 0.f;
    auto elapsed = [&](int a, int b) {
        float t = 0.f;
        (void)hipEventElapsedTime(&t, evs[a], evs[b]);
        return t;
    };
    auto flush = [&]() -> int {
        if (slots.empty()) return 0;
        HIPCHK(hipEventRecord(evs[6], c->stream));
        CHK(launch_transpose(slots.data(), (int)slots.size(), m, d_tr, (int)slots.size(),
                             (size_t)S * m, bflag(c), c->stream));
        HIPCHK(d2h_2d(snaps + col0, (size_t)ld_snaps * sizeof(double), d_tr,
                      slots.size() * sizeof(double), slots.size() * sizeof(double), m, c->stream));
        HIPCHK(hipEventRecord(evs[7], c->stream));
        HIPCHK(hipEventSynchronize(evs[7]));
        flush_ms += elapsed(6, 7);
        col0 += (int64_t)slots.size();
        slots.clear();
        return 0;
    };
    // keep column j: w -> snapshot slot, y -> red_coords[:, j]
    auto keep = [&](int64_t j) -> int {
        if (snaps) {
            double *slot = d_chunk + slots.size() * m;
            HIPCHK(hipMemcpyAsync(slot, d_w, m * sizeof(double), hipMemcpyDeviceToDevice,
                                  c->stream));
            slots.push_back(slot);
            if ((int)slots.size() == S)
                if (int e = flush()) return e;
        }
        if (red_coords) {
            HIPCHK(d2h(yh.data(), d_y, sizeof(double) * n_pod, c->stream));
            for (int k = 0; k < n_pod; ++k) red_coords[(size_t)k * ld_red + j] = yh[k];
        }
        return 0;
    };
    auto expand = [&]() -> int {  // w = basis y and its transposed planes
        CHK(launch_lspg_expand(d_bt, d_y, n_pod, m, d_w, c->stream));
        CHK(launch_basis_transpose(d_w, d_wT, N, N, c->stream));
        CHK(launch_basis_transpose(d_w + n, d_wT + n, N, N, c->stream));
        return 0;
    };
    auto resnorm = [&](double *out) -> int {
        HIPCHK(hipEventRecord(evs[2], c->stream));
        if (int e = residual_norm(c, d_w, d_wp, c->d_r, out)) return e;
        HIPCHK(hipEventRecord(evs[3], c->stream));
        HIPCHK(hipEventSynchronize(evs[3]));
        t_res += elapsed(2, 3);
        return 0;
    };

    const auto t0 = std::chrono::steady_clock::now();
    LHIP(h2d(d_wp, w0, m * sizeof(double), c->stream));
    LLAUNCH(launch_lspg_project(d_bt, d_wp, n_pod, m, d_part, d_y, c->stream));  // y0 = V^T w0
    LCHK(expand());                                                              // w0 = V y0
    LCHK(keep(0));
    LspgArgs la{c->cf, d_w, d_wT, d_bt, d_btT, c->d_r, n_pod, d_bk};
    int64_t total_its = 0;
    for (int s = 0; s < num_steps; ++s) {
        LHIP(hipMemcpyAsync(d_wp, d_w, m * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
        double init = 0.0, rn = 0.0, prev = 0.0;
        LCHK(resnorm(&init));
        if (!std::isfinite(init)) {
            rc = fail(BURG_ENAN, "non-finite residual norm at LSPG step %d", s);
            break;
        }
        int nres = 0;
        for (int i = 0; i < max_its; ++i) {
            if (i > 0) LCHK(resnorm(&rn));
            else rn = init;  // func(w) at the same w as init_norm (:1898-1902)
            ++nres;
            if (rn / init < relnorm_cutoff) break;
            if (nres > 1 && std::fabs((prev - rn) / prev) < min_delta) break;
            prev = rn;
            LHIP(hipEventRecord(evs[0], c->stream));
            LLAUNCH(launch_lspg_gram(la, d_part, d_G, c->stream));
            LHIP(hipEventRecord(evs[1], c->stream));
            if (lib_solve)
                LLAUNCH(launch_lspg_solve_lib(rh, d_G, n_pod, d_d0, d_info, d_y, d_err, c->stream));
            else
                LLAUNCH(launch_lspg_solve(d_G, n_pod, d_y, nullptr, d_err, c->stream));
            LCHK(expand());
            LHIP(hipEventRecord(evs[4], c->stream));
            LHIP(hipEventSynchronize(evs[4]));
            t_jac += elapsed(0, 1);
            t_ls += elapsed(1, 4);
            ++total_its;
        }
        unsigned err = 0;
        LHIP(hipMemcpy(&err, d_err, sizeof err, hipMemcpyDeviceToHost));
        if (err) {
            rc = fail(BURG_ENOCONV, "LSPG step %d: J basis is rank-deficient (Cholesky pivot <= 0)", s);
            break;
        }
        if (step_its) step_its[s] = nres;
        if (step_rel) step_rel[s] = rn / init;
        if (st) st->last_rel = rn / init;
        LCHK(keep(s + 1));
    }
    if (rc == BURG_OK) LCHK(flush());
    LHIP(hipStreamSynchronize(c->stream));
    if (rc == BURG_OK) LCHK(check_bounds(c, "burg_lspg"));
    const double loop_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (st) {
        st->steps = num_steps;
        st->newton_updates = total_its;
        st->loop_ms = loop_ms;
        st->flush_ms = flush_ms;
    }
    if (times_ms) times_ms[0] = t_jac, times_ms[1] = t_res, times_ms[2] = t_ls;
#undef LCHK
#undef LHIP
#undef LLAUNCH
    cleanup();
    return rc;
}

int burg_pod(int device, int64_t m, int ns, const double *snaps, int k, double *U, double *sigma,
             double *ms)
{
    BURG_TRACE("burg_pod");
    return burg_pod_rsvd(device, m, ns, snaps, k, 0, 0, nullptr, U, sigma, ms);
}

static int pod_impl(int device, int64_t m, int ns, const double *snaps, bool snaps_on_device, int k,
                    int nrand, int n_iter, const double *omega, double *U, double *sigma, double *ms);

int burg_pod_rsvd(int device, int64_t m, int ns, const double *snaps, int k, int nrand, int n_iter,
                  const double *omega, double *U, double *sigma, double *ms)
{
    BURG_TRACE("burg_pod_rsvd");
    return pod_impl(device, m, ns, snaps, false, k, nrand, n_iter, omega, U, sigma, ms);
}

int burg_pod_rsvd_device(int device, int64_t m, int ns, const double *d_snaps, int k, int nrand,
                         int n_iter, const double *omega, double *U, double *sigma, double *ms)
{
    BURG_TRACE("burg_pod_rsvd_device");
    if (d_snaps) {
        hipPointerAttribute_t at{};
        if (hipPointerGetAttributes(&at, d_snaps) != hipSuccess || at.type != hipMemoryTypeDevice ||
            at.device != device) {
            (void)hipGetLastError();
            return fail(BURG_EINVAL, "burg_pod_rsvd_device: snaps is not device memory of GPU %d",
                        device);
        }
    }
    return pod_impl(device, m, ns, d_snaps, true, k, nrand, n_iter, omega, U, sigma, ms);
}

static int pod_impl(int device, int64_t m, int ns, const double *snaps, bool snaps_on_device, int k,
                    int nrand, int n_iter, const double *omega, double *U, double *sigma, double *ms)
{
    if (!snaps || !U || !sigma) return fail(BURG_EINVAL, "null array");
    if (omega && (nrand < k || nrand > ns || n_iter < 0))
        return fail(BURG_EINVAL, "burg_pod_rsvd: need k <= nrand <= ns and n_iter >= 0");
    if (m < 1 || ns < 1 || k < 1 || k > ns)
        return fail(BURG_EINVAL, "burg_pod: need m, ns >= 1 and 1 <= k <= ns (m=%lld ns=%d k=%d)",
                    (long long)m, ns, k);
    HIPCHK(hipSetDevice(device));
    hipStream_t st = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    double *d_s = nullptr, *d_u = nullptr, *d_sig = nullptr, *d_om = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    auto cleanup = [&]() {
        (void)hipStreamSynchronize(st);
        dfree(d_s), dfree(d_u), dfree(d_sig), dfree(d_om);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        (void)hipStreamDestroy(st);
    };
    const size_t mm = (size_t)m;
    int rc = BURG_OK;
    if ((!snaps_on_device && (rc = dalloc(&d_s, mm * ns))) || (rc = dalloc(&d_u, mm * k)) ||
        (rc = dalloc(&d_sig, (size_t)k))) {
        cleanup();
        return rc;
    }
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    if (!snaps_on_device &&
        h2d(d_s, snaps, sizeof(double) * mm * ns, st) != hipSuccess) {
        cleanup();
        return fail(BURG_EHIP, "burg_pod: snapshot upload failed");
    }
    const double *d_in = snaps_on_device ? snaps : d_s;
    if (omega) {
        if ((rc = dalloc(&d_om, (size_t)ns * nrand))) {
            cleanup();
            return rc;
        }
        if (h2d(d_om, omega, sizeof(double) * ns * nrand, st) != hipSuccess) {
            cleanup();
            return fail(BURG_EHIP, "burg_pod_rsvd: omega upload failed");
        }
    }
    (void)hipEventRecord(e0, st);
    char msg[256] = {0};
    const int r = omega ? pod_rsvd_device(st, mm, ns, d_in, k, nrand, n_iter, d_om, d_u, d_sig, msg,
                                          sizeof msg)
                        : pod_device(st, mm, ns, d_in, k, d_u, d_sig, msg, sizeof msg);
    (void)hipEventRecord(e1, st);
    if (r != 0) {
        cleanup();
        return fail(r == -1 ? BURG_EINVAL : r == -5 ? BURG_ENOMEM : r == -6 ? BURG_ENOCONV : BURG_EHIP,
                    "burg_pod: %s", msg);
    }
    if (d2h(U, d_u, sizeof(double) * mm * k, st) != hipSuccess ||
        d2h(sigma, d_sig, sizeof(double) * k, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
        cleanup();
        return fail(BURG_EHIP, "burg_pod: result download failed");
    }
    if (ms) {
        float t = 0.f;
        (void)hipEventElapsedTime(&t, e0, e1);
        *ms = t;
    }
    cleanup();
    return BURG_OK;
}

const char *burg_build_id(void) { return BURG_BUILD_ID; }
const char *burg_build_flags(void) { return BURG_BUILD_FLAGS; }

// Host-only replay of every ring entry the pipe engine's trajectory kernels
// form (include/burgers.h).  The walks below are the
// kernels' own: ring_load_kernel and ring_extract_kernel call ring_pos, the
// compute waves advance pw per diagonal from RetCursor::next at each block
// (retained windows) or from origin with a wrap at L, the loader wave reads
// diagonal d - W for d in blocks of U.  Cells are tracked per (entry, lane):
// lane l of diagonal s holds local time s - l.
int burg_ring_audit(int W, int num_steps, int snap_every, int ring_cap, int64_t *report)
{
    return burg_ring_audit_ex(W, num_steps, snap_every, ring_cap, 0, report);
}

int burg_ring_audit_ex(int W, int num_steps, int snap_every, int ring_cap, int flags, int64_t *report)
{
    if (!report) return fail(BURG_EINVAL, "null report");
    if (!pipe_width_supported(W)) return fail(BURG_EINVAL, "W=%d: not a pipe-engine width", W);
    if (num_steps < 1 || snap_every < 1 || ring_cap < 0)
        return fail(BURG_EINVAL, "num_steps, snap_every >= 1, ring_cap >= 0");
    if (flags & ~(BURG_AUDIT_PAIRED | BURG_AUDIT_PAIRED_LAYOUT)) return fail(BURG_EINVAL, "unknown flags %#x", flags);
    const bool paired = (flags & BURG_AUDIT_PAIRED) != 0;
    const bool play = (flags & BURG_AUDIT_PAIRED_LAYOUT) != 0;
    if (play && (!paired || snap_every != 1 || ring_cap != 0))
        return fail(BURG_EINVAL, "the paired sweep layout: BURG_AUDIT_PAIRED, snap_every 1, no ring cap");
    // (the paired-halves kernel: W = 16, plain rings -- pipe_args)
    if (paired && (W != 16 || (snap_every >= 2 && snap_every * W >= W + 64)))
        return fail(BURG_EINVAL, "the paired walk runs W = 16 on plain rings only");
    const int U = pipe_block_of(W);
    const int k = snap_every;
    TrajMap mp;
    long long K = num_steps;
    if (k >= 2 && (long long)k * W >= W + 64) {
        const long long cap = ring_cap > 0 ? (long long)ring_cap * W + 128 : LLONG_MAX;
        if (!retained_layout(W, num_steps, k, cap, &mp))
            return fail(BURG_ESHAPE, "no retained layout for W=%d, %d steps, snap_every %d", W,
                        num_steps, k);
    } else {
        long long C = std::min<long long>(num_steps, ((1 << 21) - 4096) / W - 1);
        if (ring_cap > 0) C = std::min<long long>(C, ring_cap);
        K = std::min<long long>(num_steps, std::max<long long>(C, ((1 << 21) - 4096) / W - 1));
        mp = TrajMap{};
        mp.L = play ? K * W + 2 * W + 128 : C * W + W + 96;  // (play: sweep_impl's ring)
        mp.Lt = ring_stride(mp.L);
    }
    struct RA {
        long long origin, L;
        int ret_k, ret_n;
        long long ret_base;
    } ra{mp.origin, mp.L, mp.k, mp.n, mp.base};
    const bool ret = mp.k > 0;
    const long long Lt = mp.Lt, KW = K * W;
    const long long total = KW + kWave - 1;  // diagonals of the launch
    int64_t acc = 0, maxe = -1, oob = 0, mism = 0, over = 0, early = 0;
    auto pos = [&](long long s) { return ring_pos(s, mp.origin, mp.L, W, mp.k, mp.n, mp.base); };
    auto chk = [&](long long e, long long s, bool compare) {
        ++acc;
        maxe = std::max<int64_t>(maxe, e);
        if (e < 0 || e >= Lt) ++oob;
        if (compare && e != pos(s)) ++mism;
    };
    // last writer (diagonal) of each (entry, lane); writer diagonal of each entry
    const long long NONE = LLONG_MIN;
    std::vector<long long> cell((size_t)Lt * kWave, NONE), ewr((size_t)Lt, NONE);
    auto write = [&](long long e, long long s, int lane) {
        if (e < 0 || e >= Lt) return;
        cell[(size_t)e * kWave + lane] = s;
    };
    auto write_entry = [&](long long e, long long s) {
        if (e < 0 || e >= Lt) return;
        // the content of diagonal p is read back (previous state) at p + W:
        // a later store to its entry before that would corrupt the read
        if (ewr[e] != NONE && ewr[e] != s && ewr[e] + W > s) ++early;
        ewr[e] = std::max(ewr[e], s);
    };
    // initial state (ring_load_kernel): state 0 of (lane, column cl) at diagonal cl + lane - W
    for (long long s = -W; s < kWave - 1; ++s) {
        chk(pos(s), s, false);
        write_entry(pos(s), s);
    }
    for (int lane = 0; lane < kWave; ++lane)
        for (int cl = 0; cl < W; ++cl) write(pos((long long)cl + lane - W), (long long)cl + lane - W, lane);
    // paired-halves kernel (pipe.hip PAIR): per lane, the A cell's entry eA
    // (+1 per paired diagonal, +9 past column 7) and B's at eA - 8 (own wrap);
    // steady blocks (full 8-diagonal blocks with no wrap of eA .. eA + 15 and
    // eB >= 0) take their entries from the block base instead -- both forms
    // are replayed and compared with each other and with ring_pos of the
    // standard W = 16 layout (cell (q, c) of lane r at diagonal 16 q + c + r)
    if (paired) {
        const long long K8 = 8 * K;
        const long long total2 = K8 + 8 + kWave - 1;  // lane 63's B cell ends at local time 8K + 7
        const unsigned Lu = (unsigned)mp.L;
        unsigned eA[kWave];
        for (int lane = 0; lane < kWave; ++lane) {
            long long e0l = mp.origin + 16LL * (((long long)-lane) >> 3) + ((-lane) & 7) + lane;
            e0l %= mp.L;
            eA[lane] = (unsigned)(e0l < 0 ? e0l + mp.L : e0l);
        }
        for (long long sb = 0; sb < total2 && play; sb += 8) {
            // the store wave's paired sweep layout: the block's halves of
            // diagonal sb + u at entries origin + 2 (sb + u) and + 1
            unsigned ep = (unsigned)((mp.origin + 2 * sb) % mp.L);
            for (int u = 0; u < 8; ++u) {
                const unsigned ep1 = ep + 1u == Lu ? 0u : ep + 1u;
                for (int lane = 0; lane < kWave; ++lane) {
                    const long long tau = sb + u - lane;
                    const long long cA = tau & 7, qA = tau >> 3;
                    const bool vA = tau >= 0 && tau < K8, vB = tau >= 8 && tau - 8 < K8;
                    const long long dA = 16 * qA + cA + lane, dB = dA - 8;  // (cell ids: standard diagonals)
                    if (vA) {
                        chk(ep, dA, false);
                        if ((long long)ep != ring_pos_paired(qA, (int)cA, lane, mp.origin, mp.L)) ++mism;
                        write(ep, dA, lane);
                    }
                    if (vB) {
                        chk(ep1, dB, false);
                        if ((long long)ep1 != ring_pos_paired(qA - 1, (int)(8 + cA), lane, mp.origin, mp.L)) ++mism;
                        write(ep1, dB, lane);
                    }
                }
                ep = ep1 + 1u == Lu ? 0u : ep1 + 1u;
            }
        }
        for (long long sb = 0; sb < total2 && !play; sb += 8) {
            // the kernel's steady test (a full strip assumed), wave-uniform
            bool steady = sb >= 72 && sb + 8 <= K8;
            for (int lane = 0; lane < kWave && steady; ++lane)
                steady = !(eA[lane] < 8u || eA[lane] + 15u >= Lu);
            for (int lane = 0; lane < kWave; ++lane) {
                const unsigned base = eA[lane];  // the block's first A entry
                const int c0 = (int)((sb - lane) & 7);
                const int uw8 = c0 == 0 ? 8 : ((8 - c0) & 7);  // A reaches column 0 (next step)
                for (int u = 0; u < 8; ++u) {
                    const long long tau = sb + u - lane;
                    const long long cA = tau & 7, qA = tau >> 3;  // (floor division)
                    const bool vA = tau >= 0 && tau < K8, vB = tau >= 8 && tau - 8 < K8;
                    const unsigned wa = eA[lane];
                    const unsigned wb = wa >= 8u ? wa - 8u : wa + Lu - 8u;
                    // steady2: A at base + u (+ 8 from uw8 on), B 8 below
                    if (steady) {
                        const unsigned ra = base + (unsigned)u + (u < uw8 ? 0u : 8u);
                        if (ra != wa || ra - 8u != wb) ++mism;
                    }
                    const long long dA = 16 * qA + cA + lane, dB = dA - 8;
                    if (vA) {
                        chk(wa, dA, true);
                        write_entry(wa, dA);
                        write(wa, dA, lane);
                    }
                    if (vB) {
                        chk(wb, dB, true);
                        write_entry(wb, dB);
                        write(wb, dB, lane);
                    }
                    eA[lane] += cA == 7 ? 9u : 1u;
                    if (eA[lane] >= Lu) eA[lane] -= Lu;
                }
                if (steady && eA[lane] != (base + 16u >= Lu ? base + 16u - Lu : base + 16u))
                    ++mism;  // steady2: eA += 16 (wrapped once at Lu)
            }
        }
    }
    // compute waves: one store per diagonal (lanes with local time in [0, KW))
    if (!paired) {
        RetCursor rc;
        rc.init(ra, W, 0);
        unsigned pw = (unsigned)mp.origin;
        const unsigned Lu = (unsigned)mp.L;
        for (long long sb = 0; sb < total; sb += U) {
            if (ret) pw = rc.next(ra, W, U);
            for (int u = 0; u < U; ++u) {
                const long long s = sb + u;
                const long long l0 = std::max<long long>(0, s - KW + 1), l1 = std::min<long long>(kWave - 1, s);
                if (l0 <= l1) {  // some lane stores
                    chk(pw, s, true);
                    write_entry(pw, s);
                    for (long long l = l0; l <= l1; ++l) write(pw, s, (int)l);
                }
                pw = pw + 1 == Lu ? 0u : pw + 1;
            }
        }
    }
    // loader wave (wide tiles): window slot of diagonal d <- entry of d - W
    if (W > 16) {
        RetCursor rc;
        rc.init(ra, W, -W);
        const long long tl = (total + U - 1) / U * U;
        for (long long nf = 0; nf < tl; nf += U) {
            long long e;
            if (ret) {
                e = rc.next(ra, W, U);
            } else {
                e = (mp.origin + nf - W) % mp.L;
                e = e < 0 ? e + mp.L : e;
            }
            for (int u = 0; u < U; ++u) {
                chk(e, nf - W + u, nf - W + u < total);
                e = e + 1 == mp.L ? 0 : e + 1;
            }
        }
    }
    // the retained states (burg_trajectory_copy -> ring_extract_kernel): every
    // cell must still hold the diagonal that produced it
    std::vector<long long> states;
    if (play) {
        for (long long q = 1; q <= K; ++q) states.push_back(q);  // (state 0: the uploaded w0)
    } else if (ret) {
        for (int j = 1; j <= mp.n; ++j) states.push_back((long long)j * k);  // (state 0: d_ret0)
    } else {
        long long r0 = 0;
        while (r0 <= K && (r0 - 1) * W + mp.L <= K * W + 62) ++r0;
        const long long f = (r0 + k - 1) / k * k;
        for (long long q = f; q <= K; q += k) states.push_back(q);
    }
    for (long long q : states)
        for (int lane = 0; lane < kWave; ++lane)
            for (int cl = 0; cl < W; ++cl) {
                const long long s = (q - 1) * W + cl + lane;
                const long long e = play ? ring_pos_paired(q - 1, cl, lane, mp.origin, mp.L) : pos(s);
                chk(e, s, false);
                if (e >= 0 && e < Lt && cell[(size_t)e * kWave + lane] != s) ++over;
            }
    report[0] = acc;
    report[1] = maxe;
    report[2] = Lt;
    report[3] = oob;
    report[4] = mism;
    report[5] = over;
    report[6] = early;
    report[7] = (int64_t)states.size() + (ret ? 1 : 0);
    report[8] = ret ? k : (k >= 2 ? k : 1);
    return BURG_OK;
}

}  // extern "C"
