// stencil.hip -- fully parallel (HBM-bound) kernels of the FOM path:
//   residual  (K1)  inviscid_burgers_res2D_alt, C/hypernet2D.py:2512-2570,
//                   fused with the per-block sum of squares for ||R||
//   jvp       (K2)  inviscid_burgers_exact_jac2D(w) @ x, :2627-2656
//   axpy            x -= delta (newton_raphson update, :1854)
//   transpose       step-major device snapshots -> (2n, T+1) C-order columns
//                   of the reference's snaps matrix (:89-90, :126)
// Op order of residual/jvp mirrors oracle/burgers_oracle.c (compiled with
// -ffp-contract=off on both sides), so GPU == oracle bit for bit.
#include "burg_internal.h"

namespace burg {
namespace {

constexpr int kBlock = 256;

// Sum of squares of the two planes' cells this block owns, tree-reduced in
// a fixed order (deterministic).
__device__ __forceinline__ void block_sumsq(double x, double *partials)
{
    __shared__ double red[kBlock];
    red[threadIdx.x] = x;
    __syncthreads();
    for (int s = kBlock / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) partials[blockIdx.x] = red[0];
}

// halo_w / halo_wp: [u row | v row] of the row below this slab (nullptr =
// domain boundary).
__global__ __launch_bounds__(kBlock) void residual_kernel(Coeffs cf, const double *w,
                                                          const double *wp, double *res,
                                                          double *partials,
                                                          const double *halo_w,
                                                          const double *halo_wp)
{
    const int nx = cf.nx, ny = cf.ny;
    const size_t n = (size_t)nx * ny;
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    double sq = 0.0;
    if (i < n) {
        const int r = (int)(i / nx), c = (int)(i - (size_t)r * nx);
        const double a = cf.alpha;
        const double *u = w, *v = w + n, *up = wp, *vp = wp + n;
        const double ay = a * cf.inv_dy[r];
        const double ax = a * cf.inv_dx[c];
        const double Su = 0.5 * (u[i] * u[i]) + 0.5 * (up[i] * up[i]);
        const double Sv = 0.5 * (v[i] * v[i]) + 0.5 * (vp[i] * vp[i]);
        const double Suv = (0.5 * u[i]) * v[i] + (0.5 * up[i]) * vp[i];
        double dxu = ax * Su, dyuv = ay * Suv, dyv = ay * Sv, dxuv = cf.inv_dx[c] * Suv;
        if (c > 0) {
            const size_t j = i - 1;
            const double axw = a * cf.inv_dx[c - 1];
            const double SuW = 0.5 * (u[j] * u[j]) + 0.5 * (up[j] * up[j]);
            const double SuvW = (0.5 * u[j]) * v[j] + (0.5 * up[j]) * vp[j];
            dxu = dxu + (-axw) * SuW;
            dxuv = dxuv + (-cf.inv_dx[c - 1]) * SuvW;
        }
        if (r > 0 || halo_w != nullptr) {
            double uS, vS, upS, vpS;
            if (r > 0) {
                const size_t j = i - (size_t)nx;
                uS = u[j], vS = v[j], upS = up[j], vpS = vp[j];
            } else {
                uS = halo_w[c], vS = halo_w[nx + c], upS = halo_wp[c], vpS = halo_wp[nx + c];
            }
            const double ays = a * cf.inv_dy[r - 1];
            const double SvS = 0.5 * (vS * vS) + 0.5 * (vpS * vpS);
            const double SuvS = (0.5 * uS) * vS + (0.5 * upS) * vpS;
            dyuv = dyuv + (-ays) * SuvS;
            dyv = dyv + (-ays) * SvS;
        }
        double ru = u[i] - up[i];
        ru = ru + dxu;
        ru = ru + dyuv;
        ru = ru - cf.src[c];
        ru = ru - (c == 0 ? cf.lbc[r] : 0.0);
        double rv = v[i] - vp[i];
        rv = rv + dyv;
        rv = rv + a * dxuv;
        res[i] = ru;
        res[n + i] = rv;
        sq = ru * ru + rv * rv;
    }
    block_sumsq(sq, partials);
}

__global__ __launch_bounds__(kBlock) void sum_partials_kernel(const double *partials, int np,
                                                              double *out)
{
    double s = 0.0;
    for (int i = threadIdx.x; i < np; i += kBlock) s += partials[i];
    __shared__ double red[kBlock];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = kBlock / 2; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = red[0];
}

__global__ __launch_bounds__(kBlock) void jvp_kernel(Coeffs cf, const double *w,
                                                     const double *x, double *y)
{
    const int nx = cf.nx, ny = cf.ny;
    const size_t n = (size_t)nx * ny;
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int r = (int)(i / nx), c = (int)(i - (size_t)r * nx);
    const double a = cf.alpha;
    const double *u = w, *v = w + n, *xu = x, *xv = x + n;
    const double ax = a * cf.inv_dx[c], ay = a * cf.inv_dy[r];
    const double m = v[i] * xu[i] + u[i] * xv[i];
    double yu = xu[i] + ax * u[i] * xu[i] + 0.5 * ay * m;
    double yv = xv[i] + ay * v[i] * xv[i] + 0.5 * ax * m;
    if (c > 0) {
        const size_t j = i - 1;
        const double axw = a * cf.inv_dx[c - 1];
        const double mW = v[j] * xu[j] + u[j] * xv[j];
        yu -= axw * u[j] * xu[j];
        yv -= 0.5 * axw * mW;
    }
    if (r > 0) {
        const size_t j = i - (size_t)nx;
        const double ays = a * cf.inv_dy[r - 1];
        const double mS = v[j] * xu[j] + u[j] * xv[j];
        yu -= 0.5 * ays * mS;
        yv -= ays * v[j] * xv[j];
    }
    y[i] = yu;
    y[n + i] = yv;
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
                                                        double *out, int ldo)
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
        if (i < m && tx < nstates) out[i * (size_t)ldo + tx] = tile[tx][ii];
    }
}

}  // namespace

int residual_partials_count(const Coeffs &cf)
{
    const size_t n = (size_t)cf.nx * cf.ny;
    return (int)((n + kBlock - 1) / kBlock);
}

int launch_residual(const Coeffs &cf, const double *w, const double *wp, double *r,
                    double *partials, double *sumsq, const double *halo_w,
                    const double *halo_wp, hipStream_t st)
{
    const int nb = residual_partials_count(cf);
    residual_kernel<<<nb, kBlock, 0, st>>>(cf, w, wp, r, partials, halo_w, halo_wp);
    if (sumsq) sum_partials_kernel<<<1, kBlock, 0, st>>>(partials, nb, sumsq);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_jvp(const Coeffs &cf, const double *w, const double *x, double *y, hipStream_t st)
{
    const size_t n = (size_t)cf.nx * cf.ny;
    jvp_kernel<<<(unsigned)((n + kBlock - 1) / kBlock), kBlock, 0, st>>>(cf, w, x, y);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_axpy_neg(double *w, const double *d, size_t m, hipStream_t st)
{
    axpy_neg_kernel<<<(unsigned)((m + kBlock - 1) / kBlock), kBlock, 0, st>>>(w, d, m);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_transpose(const double *const *states, int nstates, size_t m, double *out,
                     int ldo, hipStream_t st)
{
    for (int j0 = 0; j0 < nstates; j0 += kMaxStates) {
        StatePtrs sp{};
        const int cnt = nstates - j0 < kMaxStates ? nstates - j0 : kMaxStates;
        for (int j = 0; j < cnt; ++j) sp.p[j] = states[j0 + j];
        transpose_kernel<<<(unsigned)((m + 63) / 64), 256, 0, st>>>(sp, cnt, m, out + j0, ldo);
        if (hipGetLastError() != hipSuccess) return -3;
    }
    return 0;
}

}  // namespace burg
