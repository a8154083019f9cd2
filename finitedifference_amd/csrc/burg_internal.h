// burg_internal.h -- shared device/host declarations of libburgers_hip.so.
//
// Layout in HBM: every field is a row-major (ny, nx) fp64
// plane; a state is [u plane | v plane] exactly as the reference's
// w = [u.ravel(), v.ravel()] (C/run_fom.py:33-35), so device state <-> host
// snapshot column copies are plain memcpy/transposes.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace burg {

constexpr int kWave = 64;  // CDNA wavefront; also the tile height (one lane per row)

// Per-problem coefficient vectors (device pointers, slab-local rows).
struct Coeffs {
    const double *inv_dx;  // [nx]      1/dx_c
    const double *inv_dy;  // [ny]      1/dy_r   (rows of this slab)
    const double *src;     // [nx]      dt*0.02*exp(mu2*xc)
    const double *lbc;     // [ny]      0.5*dt*mu1^2/dx[r] (inlet, column 0 only)
    double alpha;          // 0.5*dt
    int nx, ny;            // local grid (ny = rows owned by this slab)
};

// Tile engine bookkeeping.  A tile is 64 rows x tw columns,
// marched by one wavefront.  Edge planes hold, per tile, the two outflow
// quantities of its east column (E: 2 x 64) and north row (N: 2 x tw); two
// generations (ping-pong by pass parity).  Wused/Sused keep the inflow each
// tile was last marched with.
struct Engine {
    double *eb[2];     // [ntiles][2][64]
    double *nb[2];     // [ntiles][2][tw]
    double *wused;     // [ntiles][2][64]
    double *sused;     // [ntiles][2][tw]
    int *counters;     // [kbound + 2]  tiles marched per pass (index = pass)
    int *ticket;       // arrival counter of the final pass (reset by its last workgroup)
    int kbound;        // #tile anti-diagonals + 1: passes that always reach the fixed point
    // Slab halo (multi-GPU): outflow (YH, YG) of the row below this slab,
    // [2][nx], and that row's previous-step state (u, v) [2][nx] for the
    // pass-1 guess.  nullptr => bottom rows see the domain boundary (zero).
    const double *halo_flux;
    const double *halo_wp;
    double tol;        // relative inflow motion that triggers a re-march
    int nti, ntj;      // tile grid
    int tw;            // tile width
};

// Accumulated per-run statistics kept on the device.
struct DevStats {
    long long tile_marches;
    long long passes;
    int max_passes;
    int unconverged_steps;
    long long steps;
    long long tail_passes;  // passes run by the final kernel's last workgroup
};

// ---- streaming engine (stream.hip) --------------------
struct d2 {
    double x, y;
};

struct StreamStats {
    unsigned long long tile_steps;      // tile x step units marched
    unsigned long long stall_spins;     // slow-path polls of not-yet-ready mailboxes
    unsigned long long ieee_diagonals;  // waves that took the slow path at least once
    unsigned long long slow_diagonals;  // diagonals that took the slow path (all waves)
    unsigned long long slow_ticks;      // s_memtime ticks spent in the slow path
    unsigned long long why[6];          // slow-path causes: 0 east slot busy, 1 north slot
                                        // busy, 2 west not written, 3 south not written,
                                        // 4 range (IEEE redo; pipe: the loader window or the
                                        // store wave), 5 entries that needed a re-poll
    unsigned long long nonfinite_diagonals;  // diagonals whose new state has a NaN / Inf
    unsigned long long prof[8];  // pipe, built with -DBURG_PIPE_PROF: compute-wave clocks in
                                 // [0] the loop, [1] block-start store waits, [2] readiness
                                 // waits, [4 + k] readiness waits of compute wave k
    // pipe launch diagnostics (s_memrealtime, 100 MHz; reset before every
    // launch, stream_launch): first workgroup entry (min), the latest compute
    // wave's first block (max), the halo strip's earliest first block (min;
    // ~0: no inbound halo); blocks that waited for south inflow and their
    // waiting time, [0] from a strip of this GPU, [1] from the halo ring
    unsigned long long t_entry, t_halo_first, t_first_max;
    unsigned long long south_blocks[2], south_rt[2];
};

// Tiling of a slab for the streaming engine: nti strips of 64 rows, ntj tiles
// of W columns; R mailbox slots (steps) per edge.
// Bytes per edge granule slot: one 128-B L2 line each, so that reading one
// granule never caches a neighbour granule before its producer wrote it.
constexpr int kGranuleStride = 128;
// pipe engine mailboxes: granules packed 16 B apart (a poll of 16 consecutive
// diagonals fetches 2 lines instead of 16; -DBURG_PIPE_G=128 for the round-2
// layout, one granule per line)
#ifndef BURG_PIPE_G
#define BURG_PIPE_G 16
#endif
constexpr int kPipeGranuleStride = BURG_PIPE_G;

struct StreamPlan {
    int W, nti, ntj, ntiles, R;
};

// Where a tile's ring keeps diagonal s of a launch (s >= -W: the launch's
// initial state sits at diagonals -W .. 62, state q >= 1 at diagonals
// (q-1) W .. q W + 62 -- lane l, column c of state q at (q-1) W + c + l).
//   * plain ring (k == 0): entry (origin + s) mod L;
//   * retained windows (k >= 2, one launch from origin 0; the snap_every of
//     burg_trajectory_ex): window j < n holds the
//     W + 64 diagonals starting at ((j+1) k - 1) W -- every cell of state
//     (j+1) k, which no later diagonal overwrites -- at entries base +
//     j (W + 64) + offset; every other diagonal goes to a working ring of L
//     entries whose position pauses inside the windows.  Each diagonal is
//     still stored exactly once: keeping every k-th state costs no traffic.
// Windows must not overlap (k W >= W + 64) and begin on block boundaries
// (W + 64, k W and L multiples of the block).
__host__ __device__ inline long long ring_pos(long long s, long long origin, long long L, int W,
                                              int k, int n, long long base)
{
    if (k > 0) {
        const long long r = s - (long long)(k - 1) * W;
        if (r >= 0) {
            const long long kw = (long long)k * W, j = r / kw, o = r - j * kw;
            if (j < n && o < W + 64) return base + j * (W + 64) + o;
            s -= (j < n ? j + 1 : n) * (long long)(W + 64);  // retained diagonals before s
        }
    }
    const long long d = (origin + s) % L;
    return d < 0 ? d + L : d;
}

// The paired sweep layout (pipe.hip's paired kernel with its store wave, in
// burg_sweep launches): the launch's step t >= 0,
// column c (0..15) of lane r -- computed at paired diagonal s = 8 t + c + r
// by half c / 8 -- sits at entry origin + 2 s + c / 8 (mod L), so that the
// store wave writes each half of a paired diagonal as one contiguous 1 KB
// entry.  The launch's initial state keeps ring_pos's layout (diagonals -W ..
// 62), which the kernel reads before it writes any entry.
__host__ __device__ inline long long ring_pos_paired(long long t, int c, int r, long long origin, long long L)
{
    const long long d = (origin + 2 * (8 * t + c + r) + (c >> 3)) % L;
    return d < 0 ? d + L : d;
}

// Walk of a tile's diagonals one block of U at a time through the retained
// windows of ring_pos (a.ret_k > 0): entry of the block's first diagonal,
// advanced per block without divisions.  The windows, the working ring's
// wrap (L a multiple of U, origin 0) and the blocks all start on multiples of
// U, so a block's U diagonals are U consecutive entries.  s0: first diagonal
// of the walk, <= 0.  A: any struct with origin, L, ret_k, ret_n, ret_base
// (PipeArgs on the device; burg_ring_audit replays the same walk on the host).
struct RetCursor {
    int j, o;    // window index, diagonal - (window j's first diagonal)
    unsigned w;  // working-ring position of the next diagonal outside a window
    template <class A>
    __host__ __device__ void init(const A &a, int W, int s0)
    {
        j = 0;
        o = s0 - (a.ret_k - 1) * W;
        long long e = (a.origin + s0) % a.L;
        w = (unsigned)(e < 0 ? e + a.L : e);
    }
    template <class A>
    __host__ __device__ unsigned next(const A &a, int W, int U)
    {
        const bool inw = (o >= 0) & (o < W + 64) & (j < a.ret_n);
        const unsigned e = inw ? (unsigned)a.ret_base + (unsigned)(j * (W + 64) + o) : w;
        if (!inw) w = w + U >= (unsigned)a.L ? w + U - (unsigned)a.L : w + U;
        o += U;
        if (o == a.ret_k * W) {
            o = 0;
            ++j;
        }
        return e;
    }
};

// The diagnosis words err[1..3] of a failed wait (tile, diagonal, kind), as
// three separate 32-bit stores: merged into one dwordx3 store the compiler
// would reuse its data VGPRs a few instructions later (the store-VGPR rule
// of DESIGN.md section 6.2 -- tools/store_reuse_check.py)
__device__ inline void set_err3(unsigned *err, unsigned tile, unsigned where, unsigned kind)
{
    *(volatile unsigned *)&err[1] = tile;
    *(volatile unsigned *)&err[2] = where;
    *(volatile unsigned *)&err[3] = kind;
}

struct StreamArgs {
    Coeffs cf;
    const d2 *colc;      // [ntj*W] {hx, src} per column
    d2 *ring;            // [ntiles][Lt][64] state by diagonal
    d2 *wbox;            // [ntiles][R][64] west-edge mailboxes
    d2 *sbox;            // [ntiles][R][W]  south-edge mailboxes
    size_t wbox_bytes, sbox_bytes;
    long long origin;    // ring entry of diagonal 0
    long long L;         // ring length (diagonals); the working ring with retained windows
    long long Lt;        // entries per tile (>= L: + the retained windows)
    int ret_k, ret_n;    // retained windows (ring_pos): snap_every, windows; 0: plain ring
    long long ret_base;  // entry of window 0
    int K;               // time steps of this launch
    int play;            // 1: the launch's states (k >= 1) in the paired sweep layout (ring_pos_paired)
    int flags;           // diagnostics only: bit 0 = ignore neighbours (wrong results)
    int nti, ntj, ntiles, R;
    unsigned *err;       // bit 0: a mailbox wait gave up
    StreamStats *stats;
};

// ---- pipe engine (pipe.hip) ---------------------------
// Same tiles and ring as the streaming engine; a workgroup holds 4 adjacent
// tiles of one strip (4 compute waves) plus one comm wave.  Global mailboxes
// use two sentinel colours so that a slot's emptiness is tied to a step.
#ifndef BURG_PIPE_R
#define BURG_PIPE_R 8
#endif
constexpr int kPipeR = BURG_PIPE_R;  // global mailbox slots (steps) per edge, power of two
// (8 is the only depth run and tested; a 16-step build failed its first wait
// in round 5, profiles/r05/ab/narrow/r16_error.txt -- refuse other depths)
static_assert(kPipeR == 8, "BURG_PIPE_R: only 8-step mailboxes are supported");
constexpr int kPipeRL = 4;  // LDS ring slots (steps) per intra-workgroup edge
constexpr int kPipeSweepMax = 9;   // trajectories per sweep launch (LDS-resident tables)

struct PipeArgs {
    Coeffs cf;
    const d2 *colc;       // [ntj*W] {hx, src}
    d2 *ring;             // [ntiles][L][64]
    d2 *wbox;             // [ntiles][kPipeR][64] granules (kGranuleStride apart)
    d2 *sbox;             // [ntiles][kPipeR][W]
    size_t wbox_bytes, sbox_bytes;
    // Multi-GPU halo rings in pinned host memory shared with the neighbour
    // ranks (system scope): [kPipeR][ntj*W] granules, 16 B apart.  nullptr:
    // no neighbour on that side (domain boundary).
    d2 *halo_in;          // south inflow of the bottom strip (written by rank-1)
    d2 *halo_out;         // north outflow of the top strip (read by rank+1)
    size_t halo_bytes;
    long long origin, L;  // ring entry of diagonal 0, ring length (working ring: ring_pos)
    long long Lt;         // ring entries per tile (>= L: + the retained windows)
    int ret_k, ret_n;     // retained windows (ring_pos): snap_every, windows; 0: plain ring
    long long ret_base;   // entry of window 0
    int K;                // steps of this launch
    // Parameter sweep (burg_sweep): the launch runs K / T trajectories of T
    // steps back to back, each from the initial state, trajectory j with
    // its own source / inlet coefficients.  T == K, colc_b == nullptr: one
    // trajectory (colc, cf.lbc).
    int T;
    const d2 *colc_b;     // [K/T][ntj*W] {hx, src_j}
    const double *lbc_b;  // [K/T][ny] inlet term of trajectory j, this slab's rows
    int qbase;            // absolute step of local step 0, mod 2*kPipeR (sentinel colour)
    int nti, ntj, ntiles, nwj;  // tile grid; nwj = workgroups per strip
    // side-by-side domains (burg_sweep at small grids): nd domains of nti_d
    // strips (ny_d real rows) each, stacked; domain j reads column table
    // colc + j * colc_dstride.  nd = 1: one domain, nti_d = nti, ny_d = cf.ny.
    int nd, nti_d, ny_d;
    size_t colc_dstride;
    int wg_cm;            // workgroup order: 1 column-major (tile row fastest), 0 row-major
    int pair;             // W = 16 run kernel with paired 8-column halves (pipe.hip PAIR)
    unsigned w0c[4];      // paired sweeps with a store wave: the uniform initial state {u0, v0} (bits)
    int play;             // paired sweeps with a store wave: states in the paired layout (ring_pos_paired)
    long long spin_ticks; // s_memrealtime ticks (100 MHz) a wait may last without progress
    long long census_ticks;  // how long the residency census may wait for the whole grid
    unsigned *err;        // [4]: flag, tile, diagonal/step, which wait (64: residency census)
    unsigned *census;     // workgroups checked in (zeroed before every launch)
    StreamStats *stats;
};

}  // namespace burg

// ---- host-side launch wrappers (defined in the .hip files) ----------------
namespace burg {

// pass = 1..P (final = false) over all tiles, then pass P+1 with final = true
int launch_march_pass(const Coeffs &cf, const Engine &eg, const double *wp, double *w,
                      int pass, bool final, DevStats *stats, hipStream_t st);
int launch_solve_pass(const Coeffs &cf, const Engine &eg, const double *w,
                      const double *rhs, double *delta, int pass, bool final,
                      DevStats *stats, hipStream_t st);

int launch_residual(const Coeffs &cf, const double *w, const double *wp, double *r,
                    double *partials, double *sumsq, const double *halo_w,
                    const double *halo_wp, hipStream_t st);
int residual_partials_count(const Coeffs &cf);
int launch_jvp(const Coeffs &cf, const double *w, const double *x, double *y,
               hipStream_t st);
int launch_axpy_neg(double *w, const double *d, size_t m, hipStream_t st);
StreamPlan plan_stream(int nx, int ny, int tiles_target, int w_force);
bool stream_width_supported(int W);
int stream_max_resident_blocks(int W, int *per_cu, int *cus);
int launch_stream(const StreamArgs &a, int W, hipStream_t st);
int launch_colc(const Coeffs &cf, int ncols_pad, void *colc, hipStream_t st);
int launch_colc_batch(const Coeffs &cf, int nb, const double *src_b, int ncols_pad, void *colc_b,
                      hipStream_t st);
int launch_fill_sentinel(void *p, size_t n16, hipStream_t st);
int launch_ring_load(const StreamArgs &a, int W, const double *w, hipStream_t st);
// (out_elems: doubles the caller's `out` holds -- the kernels check every
// ring entry and output index, StreamArgs::err[5] flags a violation)
int launch_ring_extract_rows(const StreamArgs &a, int W, size_t e0, size_t ne, int k0, int kstep,
                             int ncols, double *out, size_t out_elems, hipStream_t st);
int launch_ring_extract(const StreamArgs &a, int W, int k0, int kstep, int count, double *out,
                        int ldo, size_t out_elems, hipStream_t st);
bool pipe_width_supported(int W);
int pipe_block_of(int W);  // diagonals per block of the trajectory kernel
bool pipe_sweep_width_supported(int W);
bool pipe_pair_sweep_uniform_only();  // paired sweeps need a uniform initial state (PipeArgs::w0c)
int pipe_max_resident_blocks(int W, bool sweep = false);
int launch_pipe(const PipeArgs &a, int W, hipStream_t st);
int launch_pipe_fill(void *p, size_t n16, int color, hipStream_t st);
// halo ring self-test: system-scope store of `put` at granule put_at (>= 0),
// then poll granule get_at (>= 0) for `want` up to `seconds`; got = last read
int halo_probe(void *ring, size_t bytes, int put_at, const unsigned put[4], int get_at,
               const unsigned want[4], double seconds, unsigned got[4], hipStream_t st);
int launch_basis_transpose(const double *b, double *bt, size_t m, int npod, hipStream_t st);
int launch_ecsw(const Coeffs &cf, const double *w, const double *wp, const double *bt, int npod,
                double *cblk, hipStream_t st);
// LSPG PROM (lspg.hip): at most kLspgMaxPod POD vectors (the augmented
// Gram matrix [JV | -R]^T [JV | -R] is at most 128 x 128)
constexpr int kLspgMaxPod = 127;
struct LspgArgs {
    Coeffs cf;           // square grid (nx == ny), single domain
    const double *w;     // state (2n)
    const double *wT;    // state, each plane transposed (2n)
    const double *bt;    // basis, (npod, 2n)
    const double *btT;   // basis, (npod, 2n), each plane transposed
    const double *r;     // residual R(w; wp) (2n)
    int npod;
    const double *bk;    // basis blocked by 32-cell tiles (lspg_gram_blocked): [tile][k][2][32][2]
};
int lspg_cols(int npod);
size_t lspg_partial_count(int nx, int npod);
int launch_lspg_expand(const double *bt, const double *y, int npod, size_t m, double *w,
                       hipStream_t st);
int launch_lspg_project(const double *bt, const double *x, int npod, size_t m, double *scratch,
                        double *y, hipStream_t st);
int launch_lspg_gram(const LspgArgs &a, double *partial, double *G, hipStream_t st);
// the Gram kernel for npod reads the blocked basis (LspgArgs::bk): its size in
// doubles, and the kernel that builds it from bt / btT
bool lspg_gram_blocked(int npod);
size_t lspg_blocked_count(size_t n, int npod);
int launch_lspg_block_basis(const double *bt, const double *btT, size_t n, int npod, double *bk,
                            hipStream_t st);
int launch_lspg_solve(const double *G, int npod, double *y, double *dy, unsigned *err,
                      hipStream_t st);
// the same with rocSOLVER potrf/potrs (handle: a rocblas_handle on st)
int launch_lspg_solve_lib(void *handle, double *G, int npod, double *d0, int *info, double *y,
                          unsigned *err, hipStream_t st);
// POD (pod.hip): exact thin SVD of a C-order (m x ns) device matrix via
// rocSOLVER QR + SVD of R; U (m x k, C-order) and the k leading singular values
int pod_device(hipStream_t st, size_t m, int ns, const double *d_s, int k, double *d_u,
               double *d_sigma, char *msg, size_t msglen);
int pod_rsvd_device(hipStream_t st, size_t m, int ns, const double *d_s, int k, int nrand,
                    int n_iter, const double *d_omega, double *d_u, double *d_sigma, char *msg,
                    size_t msglen);
// (out_elems: doubles `out` holds; a write past it is dropped and sets *flag |= 2)
int launch_transpose(const double *const *states, int nstates, size_t m, double *out,
                     int ldo, size_t out_elems, unsigned *flag, hipStream_t st);

// Copies between caller host memory and the device, through the library's
// pinned bounce buffers (hostxfer.hip; synchronous: the caller's buffer is
// free / filled on return).  No caller memory is ever handed to the HIP
// runtime's copy engine or to hipHostRegister.
hipError_t h2d(void *dst, const void *src, size_t bytes, hipStream_t st);
hipError_t d2h(void *dst, const void *src, size_t bytes, hipStream_t st);
hipError_t d2h_2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width,
                  size_t height, hipStream_t st);
hipError_t h2d_2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width,
                  size_t height, hipStream_t st);

}  // namespace burg
