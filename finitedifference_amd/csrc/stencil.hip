// stencil.hip -- fully parallel (HBM-bound) kernels of the FOM path:
//   residual  (K1)  inviscid_burgers_res2D_alt, C/hypernet2D.py:2512-2570,
//                   fused with the per-block sum of squares for ||R||
//   jvp       (K2)  inviscid_burgers_exact_jac2D(w) @ x, :2627-2656
//   axpy            x -= delta (newton_raphson update, :1854)
//   transpose       step-major device snapshots -> (2n, T+1) C-order columns
//                   of the reference's snaps matrix (:89-90, :126)
// Op order of residual/jvp mirrors oracle/burgers_oracle.c (compiled with
// -ffp-contract=off on both sides), so GPU == oracle bit for bit.
#include <algorithm>
#include <cstdlib>

#include "burg_internal.h"

namespace burg {
namespace {

constexpr int kBlock = 256;

// Row-marching layout of the two stencils (K1, K2): a workgroup owns a strip
// of 256 columns x `rows` rows and walks it bottom to top.  Every cell's
// u, v (and up, vp or xu, xv) are loaded from HBM exactly once: the south
// neighbour's terms are the previous row's, carried in registers, and the
// west neighbour's terms are the left lane's, moved by one DPP wave shift
// (lane 0 of each wave computes its west terms from its own loads).  The
// neighbour terms are the SAME expressions the neighbour evaluates for
// itself, so the result is bitwise the one-cell-per-thread formulation
// (op order of oracle/burgers_oracle.c, -ffp-contract=off).

// lane i <- lane i-1 (wave shift); lane 0 keeps `old0`
__device__ __forceinline__ double wave_shr1(double old0, double x)
{
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old0), __double2loint(x), 0x138,
                                               0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old0), __double2hiint(x), 0x138,
                                               0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

// Sum of squares of the cells this block owns, tree-reduced in a fixed
// order (deterministic).
__device__ __forceinline__ void block_sumsq(double x, double *dst)
{
    __shared__ double red[kBlock];
    red[threadIdx.x] = x;
    __syncthreads();
    for (int s = kBlock / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) *dst = red[0];
}

// Which (column block, row block) workgroup `id` of the 1-D grid owns.  XCD:
// the dispatcher deals workgroups round-robin to the 8 XCDs (id mod 8 share
// one, MI355X_MICROARCH.md section "Workgroup dispatch"); the bijective
// remap gives each XCD a contiguous band of blocks in row-major order, so a
// block's west neighbour runs beside it and its south neighbour just before
// it on the SAME XCD -- their halo lines (the west column, the south row) are
// then still in that XCD's L2 instead of re-fetched from beyond it.
template <bool XCD>
__device__ __forceinline__ void block_of(int nbx, int nb, int &bx, int &by)
{
    int id = blockIdx.x;
    if constexpr (XCD) {
        const int q = nb / 8, r = nb % 8, x = id % 8;
        id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
    }
    by = id / nbx;
    bx = id - by * nbx;
}

// halo_w / halo_wp: [u row | v row] of the row below this slab (nullptr =
// domain boundary).  PF: the next row's loads are issued before the current
// row's arithmetic (two rows of loads in flight per lane).
template <bool XCD, bool PF>
__global__ __launch_bounds__(kBlock) void residual_kernel(Coeffs cf, const double *__restrict__ w,
                                                          const double *__restrict__ wp,
                                                          double *__restrict__ res,
                                                          double *__restrict__ partials,
                                                          const double *__restrict__ halo_w,
                                                          const double *__restrict__ halo_wp,
                                                          int rows, int nbx, int nb)
{
    int bx, by;
    block_of<XCD>(nbx, nb, bx, by);
    const int nx = cf.nx, ny = cf.ny;
    const size_t n = (size_t)nx * ny;
    const int c = bx * kBlock + threadIdx.x;
    const int r0 = by * rows;
    const int r1 = min(ny, r0 + rows);
    const bool colok = c < nx;
    const int cc = colok ? c : nx - 1;  // padding lanes mirror a real column, store nothing
    const bool lane0 = (threadIdx.x & (kWave - 1)) == 0;
    const bool west = c > 0;
    const double a = cf.alpha;
    const double idx = cf.inv_dx[cc];
    const double ax = a * idx;
    const double idxw = west ? cf.inv_dx[cc - 1] : 0.0;
    const double axw = a * idxw;
    const double srcc = cf.src[cc];
    const double *u = w, *v = w + n, *up = wp, *vp = wp + n;
    const bool lw = lane0 && west;

    // south carry: Sv, Suv of the row below r0 and a*inv_dy of that row
    bool has_s = false;
    double SvS = 0.0, SuvS = 0.0, ays = 0.0;
    if (r0 > 0 || halo_w != nullptr) {
        double uS, vS, upS, vpS;
        if (r0 > 0) {
            const size_t j = (size_t)(r0 - 1) * nx + cc;
            uS = u[j], vS = v[j], upS = up[j], vpS = vp[j];
        } else {
            uS = halo_w[cc], vS = halo_w[nx + cc], upS = halo_wp[cc], vpS = halo_wp[nx + cc];
        }
        ays = a * cf.inv_dy[r0 - 1];
        SvS = 0.5 * (vS * vS) + 0.5 * (vpS * vpS);
        SuvS = (0.5 * uS) * vS + (0.5 * upS) * vpS;
        has_s = true;
    }
    // the row's loads (own cell; lane 0 also its west cell)
    double nu = 0.0, nv = 0.0, nup = 0.0, nvp = 0.0, wu = 0.0, wv = 0.0, wup = 0.0, wvp = 0.0;
    auto load_row = [&](int r) {
        const size_t i = (size_t)r * nx + cc;
        nu = u[i], nv = v[i], nup = up[i], nvp = vp[i];
        if (lw) wu = u[i - 1], wv = v[i - 1], wup = up[i - 1], wvp = vp[i - 1];
    };
    if (PF && r0 < r1) load_row(r0);
    double sq = 0.0;
    for (int r = r0; r < r1; ++r) {
        const size_t i = (size_t)r * nx + cc;
        if (!PF) load_row(r);
        const double ui = nu, vi = nv, upi = nup, vpi = nvp;
        const double uj = wu, vj = wv, upj = wup, vpj = wvp;
        if (PF && r + 1 < r1) load_row(r + 1);
        double SuW0 = 0.0, SuvW0 = 0.0;
        if (lw) {
            SuW0 = 0.5 * (uj * uj) + 0.5 * (upj * upj);
            SuvW0 = (0.5 * uj) * vj + (0.5 * upj) * vpj;
        }
        const double ay = a * cf.inv_dy[r];
        const double Su = 0.5 * (ui * ui) + 0.5 * (upi * upi);
        const double Sv = 0.5 * (vi * vi) + 0.5 * (vpi * vpi);
        const double Suv = (0.5 * ui) * vi + (0.5 * upi) * vpi;
        const double SuW = wave_shr1(SuW0, Su);
        const double SuvW = wave_shr1(SuvW0, Suv);
        double dxu = ax * Su, dyuv = ay * Suv, dyv = ay * Sv, dxuv = idx * Suv;
        if (west) {
            dxu = dxu + (-axw) * SuW;
            dxuv = dxuv + (-idxw) * SuvW;
        }
        if (has_s) {
            dyuv = dyuv + (-ays) * SuvS;
            dyv = dyv + (-ays) * SvS;
        }
        double ru = ui - upi;
        ru = ru + dxu;
        ru = ru + dyuv;
        ru = ru - srcc;
        ru = ru - (c == 0 ? cf.lbc[r] : 0.0);
        double rv = vi - vpi;
        rv = rv + dyv;
        rv = rv + a * dxuv;
        if (colok) {
            __builtin_nontemporal_store(ru, &res[i]);
            __builtin_nontemporal_store(rv, &res[n + i]);
            sq += ru * ru + rv * rv;
        }
        SvS = Sv;
        SuvS = Suv;
        ays = ay;
        has_s = true;
    }
    block_sumsq(sq, partials + (size_t)by * nbx + bx);
}

// ||R||^2 from the per-block partials, in a fixed order (deterministic): 1024
// threads, each summing a strided slice with every load issued up front
// (independent accumulators), then an LDS tree.  (Round 4's 256-thread loop
// of dependent loads took 27 us at 8192^2 -- 16 384 partials -- 4.4 % of the
// residual; profiles/r05/r5base.)
constexpr int kSumThreads = 1024;
__global__ __launch_bounds__(kSumThreads) void sum_partials_kernel(const double *partials, int np,
                                                                   double *out)
{
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int i = threadIdx.x;
    for (; i + 3 * kSumThreads < np; i += 4 * kSumThreads) {
        a0 += partials[i];
        a1 += partials[i + kSumThreads];
        a2 += partials[i + 2 * kSumThreads];
        a3 += partials[i + 3 * kSumThreads];
    }
    for (; i < np; i += kSumThreads) a0 += partials[i];
    __shared__ double red[kSumThreads];
    red[threadIdx.x] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    for (int k = kSumThreads / 2; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = red[0];
}

// J(w) x: per cell the terms t1 = (ax u) xu, t2 = (0.5 ay) m, t3 = (ay v) xv,
// t4 = (0.5 ax) m with m = v xu + u xv; the west cell's t1, t4 and the
// south cell's t2, t3 enter with a minus sign (exact_jac2D, :2627-2656).
template <bool XCD, bool PF>
__global__ __launch_bounds__(kBlock) void jvp_kernel(Coeffs cf, const double *__restrict__ w,
                                                     const double *__restrict__ x,
                                                     double *__restrict__ y, int rows, int nbx,
                                                     int nb)
{
    int bx, by;
    block_of<XCD>(nbx, nb, bx, by);
    const int nx = cf.nx, ny = cf.ny;
    const size_t n = (size_t)nx * ny;
    const int c = bx * kBlock + threadIdx.x;
    const int r0 = by * rows;
    const int r1 = min(ny, r0 + rows);
    const bool colok = c < nx;
    const int cc = colok ? c : nx - 1;
    const bool lane0 = (threadIdx.x & (kWave - 1)) == 0;
    const bool west = c > 0;
    const double a = cf.alpha;
    const double ax = a * cf.inv_dx[cc];
    const double axw = west ? a * cf.inv_dx[cc - 1] : 0.0;
    const double *u = w, *v = w + n, *xu = x, *xv = x + n;
    const bool lw = lane0 && west;

    bool has_s = false;
    double t2S = 0.0, t3S = 0.0;
    if (r0 > 0) {
        const size_t j = (size_t)(r0 - 1) * nx + cc;
        const double ays = a * cf.inv_dy[r0 - 1];
        const double mS = v[j] * xu[j] + u[j] * xv[j];
        t2S = 0.5 * ays * mS;
        t3S = ays * v[j] * xv[j];
        has_s = true;
    }
    double nu = 0.0, nv = 0.0, nxu = 0.0, nxv = 0.0, wu = 0.0, wv = 0.0, wxu = 0.0, wxv = 0.0;
    auto load_row = [&](int r) {
        const size_t i = (size_t)r * nx + cc;
        nu = u[i], nv = v[i], nxu = xu[i], nxv = xv[i];
        if (lw) wu = u[i - 1], wv = v[i - 1], wxu = xu[i - 1], wxv = xv[i - 1];
    };
    if (PF && r0 < r1) load_row(r0);
    for (int r = r0; r < r1; ++r) {
        const size_t i = (size_t)r * nx + cc;
        if (!PF) load_row(r);
        const double ui = nu, vi = nv, xui = nxu, xvi = nxv;
        const double uj = wu, vj = wv, xuj = wxu, xvj = wxv;
        if (PF && r + 1 < r1) load_row(r + 1);
        double t1W0 = 0.0, t4W0 = 0.0;
        if (lw) {
            const double mW = vj * xuj + uj * xvj;
            t1W0 = axw * uj * xuj;
            t4W0 = 0.5 * axw * mW;
        }
        const double ay = a * cf.inv_dy[r];
        const double m = vi * xui + ui * xvi;
        const double t1 = ax * ui * xui;
        const double t2 = 0.5 * ay * m;
        const double t3 = ay * vi * xvi;
        const double t4 = 0.5 * ax * m;
        const double t1W = wave_shr1(t1W0, t1);
        const double t4W = wave_shr1(t4W0, t4);
        double yu = xui + t1 + t2;
        double yv = xvi + t3 + t4;
        if (west) {
            yu -= t1W;
            yv -= t4W;
        }
        if (has_s) {
            yu -= t2S;
            yv -= t3S;
        }
        if (colok) {
            __builtin_nontemporal_store(yu, &y[i]);
            __builtin_nontemporal_store(yv, &y[n + i]);
        }
        t2S = t2;
        t3S = t3;
        has_s = true;
    }
}

__global__ __launch_bounds__(kBlock) void axpy_neg_kernel(double *w, const double *d, size_t m)
{
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < m) w[i] = w[i] - d[i];
}

// Snapshot transpose: states[j][i] -> out[i*ldo + j], 64 x 64 tiles via LDS
// (coalesced reads along i, coalesced writes along j).
constexpr int kMaxStates = 64;
struct StatePtrs {
    const double *p[kMaxStates];
};

__global__ __launch_bounds__(256) void transpose_kernel(StatePtrs sp, int nstates, size_t m,
                                                        double *out, int ldo, size_t out_elems,
                                                        unsigned *flag)
{
    __shared__ double tile[64][65];
    const size_t i0 = (size_t)blockIdx.x * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
    for (int j = ty; j < nstates; j += 4) {
        const size_t i = i0 + tx;
        tile[j][tx] = i < m ? sp.p[j][i] : 0.0;
    }
    __syncthreads();
    for (int ii = ty; ii < 64; ii += 4) {
        const size_t i = i0 + ii;
        if (i < m && tx < nstates) {
            const size_t o = i * (size_t)ldo + tx;
            if (o < out_elems) out[o] = tile[tx][ii];
            else if (flag) atomicOr(flag, 2u);
        }
    }
}

}  // namespace

// Stencil variant (A/B knob BURG_STENCIL, bits: 1 XCD-aware block order, 2
// next-row prefetch, 4 resident layout: as many row blocks as the chip holds
// at once, so every block is in flight from the start and there is no tail;
// rows per block follow, e.g. 128 at 8192^2).  Every variant computes the same cells with the same op
// order: the results are bit-identical.  Measured at 8192^2 (round 4,
// profiles/r04/stencil_ab_v1): residual 0.635 / 0.636 / 0.640 / 0.640 ms,
// J.x 0.624 / 0.625 / 0.622 / 0.626 ms for variants 0 / 1 / 2 / 3 -- neither
// helps.  (Two columns per thread with 16-B loads and stores were 23 % slower,
// profiles/r04/stencil_ab_v2, and were removed.)
#ifndef BURG_STENCIL_DEFAULT
#define BURG_STENCIL_DEFAULT 0
#endif
int stencil_variant()
{
    static int v = -1;
    if (v < 0) {
        v = BURG_STENCIL_DEFAULT;
        if (const char *e = std::getenv("BURG_STENCIL")) v = std::atoi(e) & 7;
    }
    return v;
}

// Block layout of the stencils: column blocks of kBlock, rows per block: the
// tallest block (<= 64 rows) that still gives >= 16384 blocks, down to 8 rows.
// Round 4 (profiles/r04/stencil_ab_v3 .. v5, one box each): at 8192^2 the
// residual / J.x took 0.683 / 0.668 ms with 64-row blocks (4096 blocks, the
// rounds 1-3 rule), 0.625 / 0.603 with 32, 0.625 / 0.593 with 16, 0.654 /
// 0.595 with 8; at 4096^2 8 rows were best (0.177 / 0.159 ms).  More, shorter
// blocks keep more of them in flight per CU through the grid's tail; the
// south-row re-read they add (1 row in 16) costs less.  BURG_STENCIL_ROWS
// forces a height (A/B knob).
struct StencilLayout {
    int nbx, rows, nb;
};
// workgroups of `fn` resident on the whole GPU at once (0: unknown)
static int resident_blocks(const void *fn)
{
    int dev = 0, ncu = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kBlock, 0) != hipSuccess)
        return 0;
    return n * ncu;
}
static StencilLayout stencil_layout(const Coeffs &cf, const void *fn)
{
    static int force = -1;
    if (force < 0) {
        force = 0;
        if (const char *e = std::getenv("BURG_STENCIL_ROWS")) force = std::atoi(e);
    }
    StencilLayout l{};
    l.nbx = (cf.nx + kBlock - 1) / kBlock;
    l.rows = 64;
    while (l.rows > 8 && (long long)l.nbx * ((cf.ny + l.rows - 1) / l.rows) < 16384) l.rows >>= 1;
    if (stencil_variant() & 4) {
        const int cap = resident_blocks(fn);  // (per call: the current device's)
        if (cap > 0) {
            const int nby = std::max(1, cap / l.nbx);
            l.rows = (cf.ny + nby - 1) / nby;
        }
    }
    if (force >= 1 && force <= 1024) l.rows = force;
    l.nb = l.nbx * ((cf.ny + l.rows - 1) / l.rows);
    return l;
}

// the residual kernel of the current variant (its layout sizes the partials)
static const void *residual_fn()
{
    switch (stencil_variant() & 3) {
    case 0: return (const void *)residual_kernel<false, false>;
    case 1: return (const void *)residual_kernel<true, false>;
    case 2: return (const void *)residual_kernel<false, true>;
    default: return (const void *)residual_kernel<true, true>;
    }
}
static const void *jvp_fn()
{
    switch (stencil_variant() & 3) {
    case 0: return (const void *)jvp_kernel<false, false>;
    case 1: return (const void *)jvp_kernel<true, false>;
    case 2: return (const void *)jvp_kernel<false, true>;
    default: return (const void *)jvp_kernel<true, true>;
    }
}

int residual_partials_count(const Coeffs &cf) { return stencil_layout(cf, residual_fn()).nb; }

int launch_residual(const Coeffs &cf, const double *w, const double *wp, double *r,
                    double *partials, double *sumsq, const double *halo_w,
                    const double *halo_wp, hipStream_t st)
{
    const StencilLayout l = stencil_layout(cf, residual_fn());
    const int rows = l.rows, nbx = l.nbx, nb = l.nb;
    // (round 4: the final sum fused into the last block -- an agent-scope
    // ticket, sc1 partials -- measured the same as this second launch,
    // profiles/r04/stencil_ab_v4, and was not kept)
    switch (stencil_variant() & 3) {
    case 0: residual_kernel<false, false><<<nb, kBlock, 0, st>>>(cf, w, wp, r, partials, halo_w, halo_wp, rows, nbx, nb); break;
    case 1: residual_kernel<true, false><<<nb, kBlock, 0, st>>>(cf, w, wp, r, partials, halo_w, halo_wp, rows, nbx, nb); break;
    case 2: residual_kernel<false, true><<<nb, kBlock, 0, st>>>(cf, w, wp, r, partials, halo_w, halo_wp, rows, nbx, nb); break;
    default: residual_kernel<true, true><<<nb, kBlock, 0, st>>>(cf, w, wp, r, partials, halo_w, halo_wp, rows, nbx, nb); break;
    }
    if (sumsq) sum_partials_kernel<<<1, kSumThreads, 0, st>>>(partials, nb, sumsq);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_jvp(const Coeffs &cf, const double *w, const double *x, double *y, hipStream_t st)
{
    const StencilLayout l = stencil_layout(cf, jvp_fn());
    const int rows = l.rows, nbx = l.nbx, nb = l.nb;
    switch (stencil_variant() & 3) {
    case 0: jvp_kernel<false, false><<<nb, kBlock, 0, st>>>(cf, w, x, y, rows, nbx, nb); break;
    case 1: jvp_kernel<true, false><<<nb, kBlock, 0, st>>>(cf, w, x, y, rows, nbx, nb); break;
    case 2: jvp_kernel<false, true><<<nb, kBlock, 0, st>>>(cf, w, x, y, rows, nbx, nb); break;
    default: jvp_kernel<true, true><<<nb, kBlock, 0, st>>>(cf, w, x, y, rows, nbx, nb); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_axpy_neg(double *w, const double *d, size_t m, hipStream_t st)
{
    axpy_neg_kernel<<<(unsigned)((m + kBlock - 1) / kBlock), kBlock, 0, st>>>(w, d, m);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_transpose(const double *const *states, int nstates, size_t m, double *out,
                     int ldo, size_t out_elems, unsigned *flag, hipStream_t st)
{
    for (int j0 = 0; j0 < nstates; j0 += kMaxStates) {
        StatePtrs sp{};
        const int cnt = nstates - j0 < kMaxStates ? nstates - j0 : kMaxStates;
        for (int j = 0; j < cnt; ++j) sp.p[j] = states[j0 + j];
        if (out_elems < (size_t)j0) return -1;
        transpose_kernel<<<(unsigned)((m + 63) / 64), 256, 0, st>>>(sp, cnt, m, out + j0, ldo,
                                                                    out_elems - j0, flag);
        if (hipGetLastError() != hipSuccess) return -3;
    }
    return 0;
}

}  // namespace burg
