// pipe.hip -- the pipe engine: K implicit time steps of the 2D inviscid Burgers
// FOM in ONE launch, exactly the sequential march (orc_march_step, bit for bit),
// pipelined over tiles and time steps.
//
// The dependence structure is the streaming engine's (stream.hip): the
// reference residual (C/hypernet2D.py:2512-2570) couples a cell only to itself
// and its west/south neighbours, so (step, row, column) is a 3-D wavefront.
// A tile is 64 rows (one per lane) x W columns; at diagonal s lane r works on
// local time t = s - r (step t / W, column t % W); the south inflow of lane r
// is lane r-1's north outflow of the previous diagonal (one DPP move) and the
// west inflow is the lane's own east outflow, except at tile edges.
//
// What is new here is WHO moves the edge data and through what:
//   * a workgroup = 4 compute waves = 4 horizontally adjacent tiles of one
//     strip, plus one comm wave (320 threads, one workgroup per CU);
//   * west->east edges between the workgroup's own tiles go through LDS rings;
//   * every edge that crosses workgroups is polled by the comm wave, which
//     deposits the granules into LDS inboxes, writes the global slot back to
//     "empty", and grants the compute waves permission to overwrite their
//     outbound global slots;
//   * so the compute waves never load from global memory: they read LDS, run
//     the cell chain and fire-and-forget their stores (trajectory ring and
//     outbound granules).  A global load's wait would also wait for every
//     older store of the wave (vmcnt counts both, in order) -- that coupling
//     cost the streaming engine half its time (profiles/r01/README.md).
//
// Global mailbox slots carry two sentinel colours: a slot is free for step q
// when it holds the sentinel of q's colour ((q / kPipeR) & 1); the consumer,
// after reading step q, writes the other colour -- the colour of step
// q + kPipeR.  A grant can then never be based on the emptiness that preceded
// the producer's own (possibly still in flight) store of step q - kPipeR.
//
// Multi-GPU: the bottom strip's south inflow and the top
// strip's north outflow may live in pinned host memory shared with the
// neighbour rank's process (halo_in / halo_out), accessed at system scope
// (sc0 sc1); the protocol is unchanged.
//
// Every wait is bounded in wall time (s_memrealtime): a wave that gives up
// sets the error word and the LDS abort flag, and the launch drains.
#include <climits>

#include "burg_internal.h"
#include "cell_math.h"

namespace burg {
namespace {

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// sentinel high words (signalling-NaN payloads: arithmetic never produces them)
constexpr unsigned kSentHi0 = 0x7FF4DEADu;  // global slot empty, colour 0
constexpr unsigned kSentHi1 = 0x7FF5DEADu;  // global slot empty, colour 1
constexpr unsigned kSentLo = 0xBEEF5A5Au;
constexpr unsigned kLdsEmptyHi = 0x7FF6DEADu;  // LDS slot empty
constexpr unsigned kOOB = 0xC0000000u;  // past every buffer's range: loads 0, stores dropped
constexpr int kR = kPipeR;
constexpr int kRL = kPipeRL;
constexpr unsigned G = kGranuleStride;
constexpr int kThreads = 5 * kWave;

__device__ __forceinline__ d2 as_d2(v4u v)
{
    d2 r;
    r.x = __hiloint2double((int)v.y, (int)v.x);
    r.y = __hiloint2double((int)v.w, (int)v.z);
    return r;
}

__device__ __forceinline__ v4u as_v4u(double a, double b)
{
    v4u v;
    v.x = (unsigned)__double2loint(a);
    v.y = (unsigned)__double2hiint(a);
    v.z = (unsigned)__double2loint(b);
    v.w = (unsigned)__double2hiint(b);
    return v;
}

__device__ __forceinline__ v4u sent_g(int color)
{
    const unsigned hi = color ? kSentHi1 : kSentHi0;
    v4u v;
    v.x = kSentLo;
    v.y = hi;
    v.z = kSentLo;
    v.w = hi;
    return v;
}

__device__ __forceinline__ v4u lds_empty_g()
{
    v4u v;
    v.x = kSentLo;
    v.y = kLdsEmptyHi;
    v.z = kSentLo;
    v.w = kLdsEmptyHi;
    return v;
}

// a global granule holds data (neither sentinel colour in either half)
__device__ __forceinline__ bool g_is_data(v4u g)
{
    return ((g.y & ~0x00010000u) != kSentHi0) && ((g.w & ~0x00010000u) != kSentHi0);
}
__device__ __forceinline__ bool g_is_empty(v4u g, int color)
{
    const unsigned hi = color ? kSentHi1 : kSentHi0;
    return g.y == hi && g.w == hi;
}
__device__ __forceinline__ bool l_is_data(v4u g) { return g.y != kLdsEmptyHi && g.w != kLdsEmptyHi; }

// lane i <- lane i-1; lane 0 keeps `old0`
__device__ __forceinline__ double shr1_or(double old0, double x)
{
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old0), __double2loint(x), 0x138,
                                               0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old0), __double2hiint(x), 0x138,
                                               0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

// device mailboxes: sc1 (agent scope, write-through, L1 bypass);
// host halo rings: sc0 sc1 (system scope)
__device__ __forceinline__ v4u ld_dev(__amdgpu_buffer_rsrc_t rs, unsigned off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
}
__device__ __forceinline__ v4u ld_sys(__amdgpu_buffer_rsrc_t rs, unsigned off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 17);
}
__device__ __forceinline__ void st_dev(__amdgpu_buffer_rsrc_t rs, unsigned off, v4u v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);
}
__device__ __forceinline__ void st_sys(__amdgpu_buffer_rsrc_t rs, unsigned off, v4u v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 17);
}
__device__ __forceinline__ void st_plain(__amdgpu_buffer_rsrc_t rs, unsigned off, v4u v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
}
__device__ __forceinline__ v4u ld_plain(__amdgpu_buffer_rsrc_t rs, unsigned off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, size_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ long long now_rt() { return (long long)__builtin_amdgcn_s_memrealtime(); }


// LDS accesses that must not be cached in registers or merged (polled / handed
// off between waves).  Explicit address space 3: a volatile access through a
// generic pointer becomes a flat_load, which waits on vmcnt (and so on every
// older global store of the wave) -- the coupling this engine exists to avoid.
typedef __attribute__((address_space(3))) v4u lds_v4u;
typedef __attribute__((address_space(3))) unsigned lds_u32;
typedef __attribute__((address_space(3))) int lds_i32;
__device__ __forceinline__ v4u lds_ld(const void *p) { return *(volatile lds_v4u *)p; }
__device__ __forceinline__ void lds_st(void *p, v4u v) { *(volatile lds_v4u *)p = v; }
__device__ __forceinline__ unsigned lds_ld32(const void *p) { return *(volatile lds_u32 *)p; }
__device__ __forceinline__ int lds_ldi(const void *p) { return *(volatile lds_i32 *)p; }
__device__ __forceinline__ void lds_sti(void *p, int v) { *(volatile lds_i32 *)p = v; }

template <int W>
constexpr int ilog2() { return W <= 1 ? 0 : 1 + ilog2<W / 2>(); }

// LDS image of one workgroup (SWEEP: a parameter sweep, burg_sweep -- the
// initial state and every trajectory's source / inlet terms stay on chip)
template <int W, bool SWEEP>
struct PipeLds {
    static constexpr int kSW = SWEEP ? kPipeSweepMax : 1;
    v4u st[4][W][kWave];    // per wave: the lane's outputs of the last W diagonals
    v4u st0[4][SWEEP ? W : 1][SWEEP ? kWave : 1];  // sweep: initial state, st's layout
    double srcb[kSW][4][W];                        // sweep: src of trajectory j, by column
    double lbt[kSW][kWave];                        // sweep: inlet term of trajectory j, by row
    v4u cc[4][W];           // per wave: {hx, src} of the tile's columns
    v4u ewe[3][kRL][kWave]; // wave k -> k+1 east outflow, by step slot and row
    v4u inw[kRL][kWave];    // west inflow of wave 0 (comm wave deposits)
    v4u ins[4][kRL][W];     // south inflow of each wave (comm wave deposits)
    v4u zero;               // inflow at the domain boundary
    int perm[8];            // [0..3] north grants per wave, [4] east grant of wave 3, [5] abort
};

template <int W, bool SWEEP>
__global__ __launch_bounds__(kThreads) void pipe_kernel(PipeArgs a)
{
    static_assert(W == 8 || W == 16, "pipe engine: W in {8, 16}");
    constexpr int LW = ilog2<W>();
    __shared__ PipeLds<W, SWEEP> sm;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & (kWave - 1);
    const int wg = blockIdx.x;
    const int ti = wg / a.nwj, g = wg - ti * a.nwj;
    const int tj0 = 4 * g;
    const int ntj = a.ntj;
    const int ny = a.cf.ny;
    const int nrow = min(kWave, ny - ti * kWave);
    const int top = nrow - 1;
    const int nval = min(4, ntj - tj0);  // valid tiles (waves) of this workgroup
    const int K = a.K;
    const int KW = K * W;
    const bool south_dev = ti > 0, south_host = ti == 0 && a.halo_in != nullptr;
    const bool north_dev = ti + 1 < a.nti, north_host = ti + 1 == a.nti && a.halo_out != nullptr;
    const int hcols = a.cf.nx;  // halo ring row length (granules): real columns only

    // ---- init (all waves), then one barrier; afterwards waves run freely
    for (int i = threadIdx.x; i < 3 * kRL * kWave; i += kThreads) (&sm.ewe[0][0][0])[i] = lds_empty_g();
    for (int i = threadIdx.x; i < kRL * kWave; i += kThreads) (&sm.inw[0][0])[i] = lds_empty_g();
    for (int i = threadIdx.x; i < 4 * kRL * W; i += kThreads) (&sm.ins[0][0][0])[i] = lds_empty_g();
    if (threadIdx.x < 8) sm.perm[threadIdx.x] = 0;
    if (threadIdx.x == 0) sm.zero = v4u{0u, 0u, 0u, 0u};
    // sweep: K / T trajectories of T steps (host guarantees <= kPipeSweepMax)
    const int nsw = SWEEP ? a.K / a.T : 1;
    if constexpr (SWEEP) {
        const size_t ncolp = (size_t)ntj * W;
        for (int i = threadIdx.x; i < nsw * 4 * W; i += kThreads) {
            const int j = i / (4 * W), kc = i - j * 4 * W;
            const int kk = kc / W, c = kc - kk * W;
            (&sm.srcb[0][0][0])[i] = tj0 + kk < ntj ? a.colc_b[j * ncolp + (size_t)(tj0 + kk) * W + c].y
                                                    : 0.0;
        }
        for (int i = threadIdx.x; i < nsw * kWave; i += kThreads) {
            const int j = i / kWave, l = i - j * kWave;
            (&sm.lbt[0][0])[i] = a.lbc_b[(size_t)j * ny + ti * kWave + min(l, nrow - 1)];
        }
    }
    if (wave < nval) {
        const int tile = ti * ntj + tj0 + wave;
        for (int c = lane; c < W; c += kWave) {
            const d2 v = a.colc[(size_t)(tj0 + wave) * W + c];
            sm.cc[wave][c] = as_v4u(v.x, v.y);
        }
        // state 0 of the lane's column c sits at diagonal c + lane - W (slot (c + lane) mod W)
        const __amdgpu_buffer_rsrc_t ring = rsrc(a.ring + (size_t)tile * a.L * kWave,
                                                 (size_t)a.L * kWave * 16);
        for (int c = 0; c < W; ++c) {
            long long e = (a.origin + c + lane - W) % a.L;
            e = e < 0 ? e + a.L : e;
            const v4u x0 = ld_plain(ring, (unsigned)e * 1024u + lane * 16u);
            sm.st[wave][(c + lane) & (W - 1)][lane] = x0;
            if constexpr (SWEEP) sm.st0[wave][(c + lane) & (W - 1)][lane] = x0;
        }
    }
    __syncthreads();

    if (wave == 4) {
        // ================= comm wave =================
        __builtin_amdgcn_s_setprio(0);
        constexpr int nS = 4 * W;      // south/north streams: (wave, column)
        constexpr int P = kWave / nS;  // lanes (step phases) per stream
        const int sidx = lane % nS, ph = lane / nS;
        const int kS = sidx / W, cS = sidx - kS * W;
        const bool kval = kS < nval;
        const int tS = ti * ntj + tj0 + kS;  // this lane's tile (S/N groups)
        const bool actS = kval && (south_dev || south_host);
        const bool actN = kval && (north_dev || north_host);
        const bool rowok = lane < nrow;
        const bool actW = tj0 > 0 && rowok;                     // west inflow of wave 0
        const bool actE = nval == 4 && tj0 + 4 < ntj && rowok;  // east outflow of wave 3
        const __amdgpu_buffer_rsrc_t wbox = rsrc(a.wbox, a.wbox_bytes);
        const __amdgpu_buffer_rsrc_t sbox = rsrc(a.sbox, a.sbox_bytes);
        const __amdgpu_buffer_rsrc_t hin = rsrc(a.halo_in, a.halo_in ? a.halo_bytes : 0);
        const __amdgpu_buffer_rsrc_t hout = rsrc(a.halo_out, a.halo_out ? a.halo_bytes : 0);
        // slot byte offsets (slot index added per step)
        // halo rings hold real columns only: a padding column (C >= nx) of a
        // boundary strip is served a zero inflow / granted at once
        const int C = (tj0 + kS) * W + cS;
        const bool virtS = south_host && C >= hcols, virtN = north_host && C >= hcols;
        const unsigned sS = south_dev ? ((unsigned)tS * kR * W + cS) * G : (unsigned)C * 16u;
        const unsigned sSstep = south_dev ? (unsigned)W * G : (unsigned)hcols * 16u;
        const unsigned sN = north_dev ? ((unsigned)(tS + ntj) * kR * W + cS) * G : (unsigned)C * 16u;
        const unsigned sNstep = north_dev ? (unsigned)W * G : (unsigned)hcols * 16u;
        const unsigned sW = ((unsigned)(ti * ntj + tj0) * kR * kWave + lane) * G;
        const unsigned sE = ((unsigned)(ti * ntj + tj0 + 4) * kR * kWave + lane) * G;
        const unsigned sWEstep = (unsigned)kWave * G;
        int qs = ph, qn = ph, qw = 0, qe = 0;
        long long t_prog = now_rt();
        unsigned long long iters = 0;
        for (;;) {
            const bool wS = actS && qs < K, wN = actN && qn < K;
            const bool wW = actW && qw < K, wE = actE && qe < K;
            if (!__any(wS || wN || wW || wE)) break;
            ++iters;
            const int aS = a.qbase + qs, aN = a.qbase + qn, aW = a.qbase + qw, aE = a.qbase + qe;
            const unsigned oS = wS && !virtS ? sS + (unsigned)(aS & (kR - 1)) * sSstep : kOOB;
            const unsigned oN = wN && !virtN ? sN + (unsigned)(aN & (kR - 1)) * sNstep : kOOB;
            const unsigned oW = wW ? sW + (unsigned)(aW & (kR - 1)) * sWEstep : kOOB;
            const unsigned oE = wE ? sE + (unsigned)(aE & (kR - 1)) * sWEstep : kOOB;
            const v4u gS = south_host ? ld_sys(hin, oS) : ld_dev(sbox, oS);  // OOB: zeros
            const v4u gN = north_host ? ld_sys(hout, oN) : ld_dev(sbox, oN);
            const v4u gW = ld_dev(wbox, oW);
            const v4u gE = ld_dev(wbox, oE);
            bool prog = false;
            if (wS && g_is_data(gS)) {
                v4u *slot = &sm.ins[kS][qs & (kRL - 1)][cS];
                if (!l_is_data(lds_ld(slot))) {
                    lds_st(slot, gS);
                    const v4u e = sent_g(((aS / kR) & 1) ^ 1);
                    if (south_host) st_sys(hin, oS, e);  // (virtual: oS is OOB, dropped)
                    else st_dev(sbox, oS, e);
                    qs += P;
                    prog = true;
                }
            }
            if (wW && g_is_data(gW)) {
                v4u *slot = &sm.inw[qw & (kRL - 1)][lane];
                if (!l_is_data(lds_ld(slot))) {
                    lds_st(slot, gW);
                    st_dev(wbox, oW, sent_g(((aW / kR) & 1) ^ 1));
                    ++qw;
                    prog = true;
                }
            }
            if (wN && (virtN || g_is_empty(gN, (aN / kR) & 1))) {
                qn += P;
                prog = true;
            }
            if (wE && g_is_empty(gE, (aE / kR) & 1)) {
                ++qe;
                prog = true;
            }
            // grants: north of wave k = min over its streams (all phases)
            int vN = actN ? qn : INT_MAX;
            for (int m = 1; m < W; m <<= 1) vN = min(vN, __shfl_xor(vN, m));
            if (P == 2) vN = min(vN, __shfl_xor(vN, 32));
            int vE = actE ? qe : INT_MAX;
            for (int m = 1; m < kWave; m <<= 1) vE = min(vE, __shfl_xor(vE, m));
            if (ph == 0 && cS == 0 && kval) lds_sti(&sm.perm[kS], vN);
            if (lane == 0) lds_sti(&sm.perm[4], vE);
            const long long tn = now_rt();
            if (__any(prog)) {
                t_prog = tn;
            } else {
                if (tn - t_prog > a.spin_ticks) {
                    if (lane == 0) {
                        lds_sti(&sm.perm[5], 1);
                        if (atomicOr(a.err, 1u) == 0) {
                            a.err[1] = (unsigned)(ti * ntj + tj0);
                            a.err[2] = (unsigned)min(min(wS ? qs : INT_MAX, wN ? qn : INT_MAX),
                                                     min(wW ? qw : INT_MAX, wE ? qe : INT_MAX));
                            a.err[3] = 16u | (__any(wS) ? 1u : 0u) | (__any(wW) ? 2u : 0u) |
                                       (__any(wN) ? 4u : 0u) | (__any(wE) ? 8u : 0u);
                        }
                    }
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (lds_ldi(&sm.perm[5])) break;
        }
        if (lane == 0) atomicAdd(&a.stats->why[5], iters);
        return;
    }
    if (wave >= nval) return;

    // ================= compute wave =================
    __builtin_amdgcn_s_setprio(1);
    const int k = wave;
    const int tj = tj0 + k;
    const int tile = ti * ntj + tj;
    const bool rowok = lane < nrow;
    const bool has_west = tj > 0;
    const bool has_south = south_dev || south_host;
    const bool east_lds = k < 3 && k + 1 < nval;
    const bool east_glob = k == 3 && tj + 1 < ntj;
    const bool has_north = north_dev || north_host;
    const bool col0_tile = tj == 0;
    const int r = ti * kWave + min(lane, top);
    const double ay = a.cf.alpha * a.cf.inv_dy[r];
    const double hy = 0.5 * ay;
    // inlet term of the lane's trajectory (sweep: lb of trajectory jl, lb_next
    // of jl + 1; qn = first step of trajectory jl + 1, whose W columns read
    // the initial state -- every trajectory starts from w0)
    double lb = SWEEP ? sm.lbt[0][lane] : a.cf.lbc[r];
    double lb_next = SWEEP ? sm.lbt[min(1, nsw - 1)][lane] : lb;
    int qn = SWEEP ? a.T : INT_MAX, jl = 0;
    // LDS rows of the src table for trajectories jl and jl + 1 (clamped)
    typedef __attribute__((address_space(3))) const double lds_f64;
    lds_f64 *src_cur = (lds_f64 *)&sm.srcb[0][k][0];
    lds_f64 *src_nxt = (lds_f64 *)&sm.srcb[min(1, nsw - 1)][k][0];
    const __amdgpu_buffer_rsrc_t ring = rsrc(a.ring + (size_t)tile * a.L * kWave,
                                             (size_t)a.L * kWave * 16);
    const __amdgpu_buffer_rsrc_t wbox = rsrc(a.wbox, a.wbox_bytes);
    const __amdgpu_buffer_rsrc_t sbox = rsrc(a.sbox, a.sbox_bytes);
    const __amdgpu_buffer_rsrc_t hout = rsrc(a.halo_out, a.halo_out ? a.halo_bytes : 0);
    const unsigned lane16 = lane * 16u;
    // outbound bases (slot offsets added per step)
    const unsigned eb = ((unsigned)(tile + 1) * kR * kWave + lane) * G;  // east tile's west box
    const unsigned nb = north_dev ? (unsigned)(tile + ntj) * kR * W * G
                                  : (unsigned)tj * W * 16u;                // + c
    const unsigned nstep = north_dev ? (unsigned)W * G : (unsigned)hcols * 16u;
    const int ncol_real = north_host ? hcols - tj * W : W;  // columns with a halo slot
    const unsigned ncol = north_dev ? G : 16u;
    v4u(*src_w)[kWave] = k == 0 ? sm.inw : sm.ewe[k - 1];
    v4u *const my_st = &sm.st[k][0][0];
    v4u *const my_st0 = &sm.st0[k][0][0];
    const long long L = a.L;
    long long pw = a.origin;
    const v4u lempty = lds_empty_g();

    double e0 = 0.0, e1 = 0.0, no0 = 0.0, no1 = 0.0;
    unsigned long long spins = 0, slow_n = 0, ieee_n = 0;
    bool aborted = false;

    // LDS inputs of diagonal s, read at the end of diagonal s - 1
    struct In {
        v4u xs, cs, gw, gs;
        int pn, pe;
        unsigned ee;
        bool nt;     // sweep: first step of the lane's next trajectory (state reset)
        double src;  // sweep: the column's source term of the step's trajectory
    };
    auto fetch = [&](int s) -> In {
        const int t = s - lane;
        const int c = t & (W - 1);
        const int q = t >> LW;
        const bool valid = (unsigned)t < (unsigned)KW;
        const bool need_w = has_west && c == 0 && valid && rowok;
        In in;
        if constexpr (SWEEP) {
            in.nt = q >= qn;
            in.xs = (in.nt ? my_st0 : my_st)[(s & (W - 1)) * kWave + lane];
            in.src = (in.nt ? src_nxt : src_cur)[c];
        } else {
            in.nt = false;
            in.xs = my_st[(s & (W - 1)) * kWave + lane];
            in.src = 0.0;
        }
        in.cs = sm.cc[k][c];
        in.gw = lds_ld(need_w ? &src_w[q & (kRL - 1)][lane] : &sm.zero);
        in.gs = lds_ld(has_south && s < KW ? &sm.ins[k][(s >> LW) & (kRL - 1)][s & (W - 1)] : &sm.zero);
        in.pn = lds_ldi(&sm.perm[k]);
        in.pe = lds_ldi(&sm.perm[4]);
        in.ee = east_lds ? lds_ld32((const char *)&sm.ewe[k][q & (kRL - 1)][lane] + 4) : kLdsEmptyHi;
        return in;
    };
    const int total = KW + kWave - 1;
    In in = fetch(0);
    // Land the prologue's global loads (row coefficients) here: a first use
    // inside the loop would put an s_waitcnt vmcnt(0) -- a wait on every store
    // in flight -- into every diagonal.
    __builtin_amdgcn_s_waitcnt(0);
    for (int s = 0; s < total; ++s) {
        const int t = s - lane;
        const int c = t & (W - 1);
        const int q = t >> LW;
        const bool valid = (unsigned)t < (unsigned)KW;
        const bool at0 = c == 0, atE = c == W - 1;
        const bool need_w = has_west && at0 && valid && rowok;
        const bool need_s = has_south && s < KW;  // wave-uniform (lane 0 consumes)
        const bool out_e = atE && valid && rowok;
        const bool out_n = lane == top && valid && has_north;
        // ---- inflow-independent part of the cell (MarchCell::pre, same op order)
        const d2 x = as_d2(in.xs);
        const d2 co = as_d2(in.cs);
        const double pu = x.x, pv = x.y;
        const double hx = co.x, ax = hx + hx;  // exact: hx = 0.5 * (alpha * inv_dx)
        const double lbu = SWEEP && in.nt ? lb_next : lb;
        const double srcc = SWEEP ? in.src : co.y;
        const double sl = (col0_tile && at0) ? srcc + lbu : srcc;
        MarchCell::Pre p;
        p.hx = hx;
        const double hu = 0.5 * pu;
        p.xfp = ax * (hu * pu);
        p.xhp = ax * (hu * pv);
        p.yhp = ay * (hu * pv);
        p.ygp = ay * ((0.5 * pv) * pv);
        p.bu = ((pu - p.xfp) - p.yhp) + sl;
        p.bv = (pv - p.ygp) - p.xhp;
        const MarchCell::Row rw{ay, hy, lbu};
        // ---- wait until inputs are deposited and outbound slots are granted
        auto blocked = [&](const In &v) -> bool {
            bool b = (need_w && !l_is_data(v.gw)) || (lane == 0 && need_s && !l_is_data(v.gs));
            b |= east_lds && out_e && v.ee != kLdsEmptyHi;
            b |= east_glob && out_e && q >= v.pe;
            b |= out_n && q >= v.pn;
            return b;
        };
        if (__builtin_expect(__any(blocked(in)), 0)) {
            const long long t0 = now_rt();
            ++slow_n;
            for (;;) {
                ++spins;
                __builtin_amdgcn_s_sleep(1);
                in = fetch(s);
                if (!__any(blocked(in))) break;
                if (lds_ldi(&sm.perm[5]) || now_rt() - t0 > a.spin_ticks) {
                    if (lane == 0 && !lds_ldi(&sm.perm[5])) {
                        lds_sti(&sm.perm[5], 1);
                        if (atomicOr(a.err, 1u) == 0) {
                            a.err[1] = (unsigned)tile;
                            a.err[2] = (unsigned)s;
                            a.err[3] = 32u;
                        }
                    }
                    aborted = true;
                    break;
                }
            }
            if (aborted) break;
        }
        // ---- the cell's chain
        if (at0) {
            const d2 gv = as_d2(in.gw);
            e0 = gv.x;
            e1 = gv.y;
        }
        const d2 sv = as_d2(in.gs);
        const double n0 = shr1_or(sv.x, no0);
        const double n1 = shr1_or(sv.y, no1);
        double oe0, oe1, on0, on1, o0, o1;
        bool ok;
        MarchCell::chain<true>(p, rw, e0, e1, n0, n1, oe0, oe1, on0, on1, o0, o1, ok);
        if (__builtin_expect(__any(!ok && valid && rowok), 0)) {
            MarchCell::chain<false>(p, rw, e0, e1, n0, n1, oe0, oe1, on0, on1, o0, o1, ok);
            ++ieee_n;
        }
        e0 = oe0;
        e1 = oe1;
        no0 = on0;
        no1 = on1;
        // ---- outputs (lanes that have not started keep their step-0 state)
        const v4u out = as_v4u(o0, o1);
        if (t >= 0) my_st[(s & (W - 1)) * kWave + lane] = out;
        st_plain(ring, valid ? (unsigned)pw * 1024u + lane16 : kOOB, out);
        pw = pw + 1 == L ? 0 : pw + 1;
        const v4u eo = as_v4u(oe0, oe1);
        const int aq = a.qbase + q;
        if (east_lds && out_e) lds_st(&sm.ewe[k][q & (kRL - 1)][lane], eo);
        if (east_glob) st_dev(wbox, out_e ? eb + (unsigned)(aq & (kR - 1)) * (kWave * G) : kOOB, eo);
        if (has_north) {
            const v4u no = as_v4u(on0, on1);
            const unsigned off = out_n && c < ncol_real
                                     ? nb + (unsigned)(aq & (kR - 1)) * nstep + (unsigned)c * ncol
                                       : kOOB;
            if (north_host) st_sys(hout, off, no);
            else st_dev(sbox, off, no);
        }
        // consumed inbound slots back to empty
        if (need_w) lds_st(&src_w[q & (kRL - 1)][lane], lempty);
        if (need_s && lane == 0) lds_st(&sm.ins[k][(s >> LW) & (kRL - 1)][s & (W - 1)], lempty);
        if constexpr (SWEEP) {
            // the lane finished the first step of its next trajectory: switch
            if (in.nt && atE) {
                ++jl;
                qn += a.T;
                lb = lb_next;
                src_cur = src_nxt;
                const int jn = min(jl + 1, nsw - 1);
                lb_next = sm.lbt[jn][lane];
                src_nxt = (lds_f64 *)&sm.srcb[jn][k][0];
            }
        }
        in = fetch(s + 1);
    }
    if (lane == 0) {
        if (spins) atomicAdd(&a.stats->stall_spins, spins);
        if (slow_n) atomicAdd(&a.stats->slow_diagonals, slow_n);
        if (ieee_n) atomicAdd(&a.stats->ieee_diagonals, ieee_n);
        atomicAdd(&a.stats->tile_steps, (unsigned long long)K);
    }
}

__global__ void pipe_fill_kernel(v4u *p, size_t n, int color)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = sent_g(color);
}

}  // namespace

bool pipe_width_supported(int W) { return W == 8 || W == 16; }

// resident workgroups of the pipe kernel (sweep = the burg_sweep variant,
// whose larger LDS image must also fit one workgroup per CU)
int pipe_max_resident_blocks(int W, bool sweep)
{
    int dev = 0, n = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -3;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return -3;
    const void *fn = W == 8 ? (sweep ? (const void *)pipe_kernel<8, true> : (const void *)pipe_kernel<8, false>)
                            : (sweep ? (const void *)pipe_kernel<16, true> : (const void *)pipe_kernel<16, false>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kThreads, 0) != hipSuccess) return -3;
    return n * ncu;
}

int launch_pipe(const PipeArgs &a, int W, hipStream_t st)
{
    const int blocks = a.nti * a.nwj;
    const bool sweep = a.colc_b != nullptr;
    if (sweep && (a.T < 1 || a.K % a.T != 0 || a.K / a.T > kPipeSweepMax)) return -1;
    if (W == 8 && !sweep)
        hipLaunchKernelGGL((pipe_kernel<8, false>), dim3(blocks), dim3(kThreads), 0, st, a);
    else if (W == 8)
        hipLaunchKernelGGL((pipe_kernel<8, true>), dim3(blocks), dim3(kThreads), 0, st, a);
    else if (W == 16 && !sweep)
        hipLaunchKernelGGL((pipe_kernel<16, false>), dim3(blocks), dim3(kThreads), 0, st, a);
    else if (W == 16)
        hipLaunchKernelGGL((pipe_kernel<16, true>), dim3(blocks), dim3(kThreads), 0, st, a);
    else
        return -1;
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_pipe_fill(void *p, size_t n16, int color, hipStream_t st)
{
    if (n16 == 0) return 0;
    hipLaunchKernelGGL(pipe_fill_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, st,
                       (v4u *)p, n16, color);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace burg
