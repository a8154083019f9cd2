// lspg.hip -- LSPG PROM inner loop on the GPU:
// inviscid_burgers_implicit2D_LSPG + gauss_newton_LSPG, C/hypernet2D.py:133-200,
// 1859-1929.
//
// Per Gauss-Newton iteration the reference assembles J(w) as a CSR matrix,
// forms JV = J.dot(basis) (2n x npod, dense) and calls np.linalg.lstsq(JV, -f).
// Here one fused kernel builds the rows of [JV | -f] tile by tile in LDS and
// accumulates the augmented Gram matrix [JV | -f]^T [JV | -f] (its last
// column is JV^T(-f)), so JV never touches HBM; a one-workgroup kernel then
// solves the npod x npod normal equations by Cholesky and updates y.
//
// The LSPG Jacobian is NOT the FOM one: the driver permutes only the ROWS of
// kron(I, Dy) (:165-167; the FOM permutes rows and columns, :98-106), so its
// "y-derivative" reads the TRANSPOSED field:
//     (Y f)[r, c] = f[c, r] / dy_r - f[c, r-1] / dy_{r-1}      (nx == ny)
// and, with a = dt/2 and J = I + [[Dx a u + Y a v / 2, Y a u / 2],
//                                 [Dx a v / 2,        Y a v + Dx a u / 2]]
// (exact_jac2D, :2627-2656), column k of JV at cell (r, c) is
//   yu = xu + a(u xu/dx_c - u_W xu_W/dx_{c-1})
//           + a/2((vT xuT + uT xvT)/dy_r - (vT xuT + uT xvT)_S/dy_{r-1})
//   yv = xv + a((vT xvT)/dy_r - (vT xvT)_S/dy_{r-1})
//           + a/2((v xu + u xv)/dx_c - (v xu + u xv)_W/dx_{c-1})
// where T marks values read from the transposed planes (the state and the
// basis are kept in both layouts) and S the row below in the transposed plane.
#include "burg_internal.h"

#include <hip/hip_runtime.h>

namespace burg {
namespace {

constexpr int kLB = 256;   // threads per workgroup
constexpr int kGC = 16;    // cells per LDS tile (2 JV rows per cell)
constexpr int kGroups = 1024;

// w[i] = sum_k bt[k m + i] y[k]   (basis.dot(y), :191/:1924)
__global__ __launch_bounds__(kLB) void lspg_expand_kernel(const double *__restrict__ bt,
                                                          const double *__restrict__ y, int npod,
                                                          size_t m, double *__restrict__ w)
{
    __shared__ double ys[kLspgMaxPod];
    for (int k = threadIdx.x; k < npod; k += kLB) ys[k] = y[k];
    __syncthreads();
    for (size_t i = (size_t)blockIdx.x * kLB + threadIdx.x; i < m; i += (size_t)gridDim.x * kLB) {
        double s0 = 0.0, s1 = 0.0;
        int k = 0;
        for (; k + 1 < npod; k += 2) {
            s0 += bt[(size_t)k * m + i] * ys[k];
            s1 += bt[(size_t)(k + 1) * m + i] * ys[k + 1];
        }
        if (k < npod) s0 += bt[(size_t)k * m + i] * ys[k];
        w[i] = s0 + s1;
    }
}

// partial[k * nb + b] = sum over chunk b of bt[k m + i] x[i]   (basis.T.dot(w0), :157)
__global__ __launch_bounds__(kLB) void lspg_project_kernel(const double *__restrict__ bt,
                                                           const double *__restrict__ x, size_t m,
                                                           double *__restrict__ partial)
{
    const int k = blockIdx.y, nb = gridDim.x;
    const double *p = bt + (size_t)k * m;
    double s = 0.0;
    for (size_t i = (size_t)blockIdx.x * kLB + threadIdx.x; i < m; i += (size_t)nb * kLB)
        s += p[i] * x[i];
    __shared__ double red[kLB];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int h = kLB / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[(size_t)k * nb + blockIdx.x] = red[0];
}

// out[e] = sum_g partial[g * stride + e] (fixed order: deterministic)
__global__ __launch_bounds__(kLB) void lspg_sum_kernel(const double *__restrict__ partial,
                                                       int ng, size_t stride, int ne,
                                                       double *__restrict__ out)
{
    const int e = blockIdx.x * kLB + threadIdx.x;
    if (e >= ne) return;
    double s = 0.0;
    for (int g = 0; g < ng; ++g) s += partial[(size_t)g * stride + e];
    out[e] = s;
}

// per-k partial layout of the projection: out[k] = sum_b partial[k nb + b]
__global__ __launch_bounds__(kLB) void lspg_rowsum_kernel(const double *__restrict__ partial,
                                                          int nb, int npod,
                                                          double *__restrict__ out)
{
    const int k = blockIdx.x * kLB + threadIdx.x;
    if (k >= npod) return;
    double s = 0.0;
    for (int b = 0; b < nb; ++b) s += partial[(size_t)k * nb + b];
    out[k] = s;
}

// Fused JV + augmented Gram.  A workgroup walks tiles of kGC consecutive
// cells; per tile it fills A[2 kGC][P] in LDS (row 2j = u-equation of cell j,
// row 2j+1 = v-equation; column k < npod = JV[:, k], column npod = -R,
// columns above = 0), then thread (bi, bj) of a 16 x 16 grid accumulates the
// TB x TB block G[bi TB.., bj TB..] += A^T A.  Partials go to
// partial[group][P][P] (reduced by lspg_sum_kernel).
template <int TB>
__global__ __launch_bounds__(kLB) void lspg_gram_kernel(LspgArgs a, double *__restrict__ partial)
{
    constexpr int P = 16 * TB;
    constexpr int LD = P + 1;
    __shared__ double A[2 * kGC * LD];
    const int N = a.cf.nx;
    const size_t n = (size_t)N * N, m = 2 * n;
    const double al = a.cf.alpha;
    const int tid = threadIdx.x;
    const int bi = tid >> 4, bj = tid & 15;
    double acc[TB][TB];
#pragma unroll
    for (int p = 0; p < TB; ++p)
#pragma unroll
        for (int q = 0; q < TB; ++q) acc[p][q] = 0.0;

    const int j = tid % kGC, kg = tid / kGC;  // fill role: cell j, columns kg + 16 q
    const size_t ntiles = (n + kGC - 1) / kGC;
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const size_t i = t * kGC + j;
        const bool ok = i < n;
        const size_t ii = ok ? i : n - 1;
        const int r = (int)(ii / N), c = (int)(ii - (size_t)r * N);
        const bool west = c > 0, south = r > 0;
        const size_t iw = west ? ii - 1 : ii, is = south ? ii - N : ii;
        const double *u = a.w, *v = a.w + n, *uT = a.wT, *vT = a.wT + n;
        const double ui = u[ii], vi = v[ii], uW = u[iw], vW = v[iw];
        const double uTi = uT[ii], vTi = vT[ii], uTS = uT[is], vTS = vT[is];
        const double ax = al * a.cf.inv_dx[c], axw = west ? al * a.cf.inv_dx[c - 1] : 0.0;
        const double ay = al * a.cf.inv_dy[r], ays = south ? al * a.cf.inv_dy[r - 1] : 0.0;
        for (int k = kg; k < P; k += kLB / kGC) {
            double yu = 0.0, yv = 0.0;
            if (ok && k < a.npod) {
                const double *xu = a.bt + (size_t)k * m, *xv = xu + n;
                const double *xuT = a.btT + (size_t)k * m, *xvT = xuT + n;
                const double xui = xu[ii], xvi = xv[ii], xuw = xu[iw], xvw = xv[iw];
                const double xuTi = xuT[ii], xvTi = xvT[ii], xuTS = xuT[is], xvTS = xvT[is];
                const double mT = vTi * xuTi + uTi * xvTi;
                yu = xui + ax * (ui * xui) + 0.5 * ay * mT;
                yv = xvi + ay * (vTi * xvTi) + 0.5 * ax * (vi * xui + ui * xvi);
                if (west) {
                    yu -= axw * (uW * xuw);
                    yv -= 0.5 * axw * (vW * xuw + uW * xvw);
                }
                if (south) {
                    yu -= 0.5 * ays * (vTS * xuTS + uTS * xvTS);
                    yv -= ays * (vTS * xvTS);
                }
            } else if (ok && k == a.npod) {
                yu = -a.r[ii];
                yv = -a.r[n + ii];
            }
            A[(2 * j) * LD + k] = yu;
            A[(2 * j + 1) * LD + k] = yv;
        }
        __syncthreads();
#pragma unroll 2
        for (int row = 0; row < 2 * kGC; ++row) {
            double av[TB], bv[TB];
#pragma unroll
            for (int p = 0; p < TB; ++p) {
                av[p] = A[row * LD + bi * TB + p];
                bv[p] = A[row * LD + bj * TB + p];
            }
#pragma unroll
            for (int p = 0; p < TB; ++p)
#pragma unroll
                for (int q = 0; q < TB; ++q) acc[p][q] += av[p] * bv[q];
        }
        __syncthreads();
    }
    double *out = partial + (size_t)blockIdx.x * P * P;
#pragma unroll
    for (int p = 0; p < TB; ++p)
#pragma unroll
        for (int q = 0; q < TB; ++q) out[(bi * TB + p) * P + bj * TB + q] = acc[p][q];
}

// One workgroup: Cholesky of G[0:npod, 0:npod] (ld P), forward and back
// substitution against b = G[0:npod, npod], then y += dy.  err <- 1 when a
// pivot is not positive relative to its diagonal (rank-deficient JV).
__global__ __launch_bounds__(kLB) void lspg_solve_kernel(const double *__restrict__ G, int P,
                                                         int npod, double *__restrict__ y,
                                                         double *__restrict__ dy_out,
                                                         unsigned *__restrict__ err)
{
    extern __shared__ double L[];  // npod x (npod + 1), dynamic (up to 127 x 128 doubles)
    __shared__ double z[kLspgMaxPod], d0[kLspgMaxPod];
    __shared__ int bad;
    const int LD = npod + 1, tid = threadIdx.x;
    for (int e = tid; e < npod * npod; e += kLB) {
        const int i = e / npod, k = e - i * npod;
        L[i * LD + k] = G[(size_t)i * P + k];
    }
    for (int i = tid; i < npod; i += kLB) {
        z[i] = G[(size_t)i * P + npod];
        d0[i] = G[(size_t)i * P + i];
    }
    if (tid == 0) bad = 0;
    __syncthreads();
    for (int jj = 0; jj < npod; ++jj) {
        if (tid == 0) {
            const double d = L[jj * LD + jj];
            // a pivot that lost all but ~8 ulp of its column's norm: rank-deficient
            if (!(d > 0x1p-49 * d0[jj])) bad = 1;
            L[jj * LD + jj] = sqrt(d > 0.0 ? d : 1.0);
        }
        __syncthreads();
        const double piv = L[jj * LD + jj];
        for (int i = jj + 1 + tid; i < npod; i += kLB) L[i * LD + jj] /= piv;
        __syncthreads();
        const int rem = npod - jj - 1;
        for (int e = tid; e < rem * rem; e += kLB) {
            const int i = jj + 1 + e / rem, k = jj + 1 + e % rem;
            if (k <= i) L[i * LD + k] -= L[i * LD + jj] * L[k * LD + jj];
        }
        __syncthreads();
    }
    // L z' = b (in place in z), then L^T dy = z'
    for (int jj = 0; jj < npod; ++jj) {
        if (tid == 0) z[jj] /= L[jj * LD + jj];
        __syncthreads();
        for (int i = jj + 1 + tid; i < npod; i += kLB) z[i] -= L[i * LD + jj] * z[jj];
        __syncthreads();
    }
    for (int jj = npod - 1; jj >= 0; --jj) {
        if (tid == 0) z[jj] /= L[jj * LD + jj];
        __syncthreads();
        for (int i = tid; i < jj; i += kLB) z[i] -= L[jj * LD + i] * z[jj];
        __syncthreads();
    }
    for (int i = tid; i < npod; i += kLB) {
        y[i] += z[i];
        if (dy_out) dy_out[i] = z[i];
    }
    if (tid == 0 && bad) *err = 1u;
}

int groups_for(size_t n)
{
    const size_t tiles = (n + kGC - 1) / kGC;
    return (int)(tiles < (size_t)kGroups ? tiles : (size_t)kGroups);
}

}  // namespace

int lspg_cols(int npod)
{
    for (int tb = 2; tb <= 8; tb += 2)
        if (npod + 1 <= 16 * tb) return 16 * tb;
    return 0;
}

size_t lspg_partial_count(int nx, int npod)
{
    const int P = lspg_cols(npod);
    return (size_t)groups_for((size_t)nx * nx) * P * P + (size_t)npod * 256;
}

int launch_lspg_expand(const double *bt, const double *y, int npod, size_t m, double *w,
                       hipStream_t st)
{
    size_t g = (m + kLB - 1) / kLB;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(lspg_expand_kernel, dim3((unsigned)g), dim3(kLB), 0, st, bt, y, npod, m, w);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_lspg_project(const double *bt, const double *x, int npod, size_t m, double *scratch,
                        double *y, hipStream_t st)
{
    const int nb = 256;
    hipLaunchKernelGGL(lspg_project_kernel, dim3(nb, npod), dim3(kLB), 0, st, bt, x, m, scratch);
    hipLaunchKernelGGL(lspg_rowsum_kernel, dim3((npod + kLB - 1) / kLB), dim3(kLB), 0, st,
                       (const double *)scratch, nb, npod, y);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_lspg_gram(const LspgArgs &a, double *partial, double *G, hipStream_t st)
{
    const int P = lspg_cols(a.npod);
    const int ng = groups_for((size_t)a.cf.nx * a.cf.nx);
    switch (P) {
    case 32: hipLaunchKernelGGL(lspg_gram_kernel<2>, dim3(ng), dim3(kLB), 0, st, a, partial); break;
    case 64: hipLaunchKernelGGL(lspg_gram_kernel<4>, dim3(ng), dim3(kLB), 0, st, a, partial); break;
    case 96: hipLaunchKernelGGL(lspg_gram_kernel<6>, dim3(ng), dim3(kLB), 0, st, a, partial); break;
    case 128: hipLaunchKernelGGL(lspg_gram_kernel<8>, dim3(ng), dim3(kLB), 0, st, a, partial); break;
    default: return -1;
    }
    hipLaunchKernelGGL(lspg_sum_kernel, dim3((P * P + kLB - 1) / kLB), dim3(kLB), 0, st,
                       (const double *)partial, ng, (size_t)P * P, P * P, G);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_lspg_solve(const double *G, int npod, double *y, double *dy, unsigned *err,
                      hipStream_t st)
{
    static bool attr = false;
    const size_t lds = sizeof(double) * (size_t)npod * (npod + 1);
    if (!attr) {
        if (hipFuncSetAttribute((const void *)lspg_solve_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)(sizeof(double) * kLspgMaxPod * (kLspgMaxPod + 1))) !=
            hipSuccess)
            return -3;
        attr = true;
    }
    hipLaunchKernelGGL(lspg_solve_kernel, dim3(1), dim3(kLB), lds, st, G, lspg_cols(npod), npod,
                       y, dy, err);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace burg
