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

#include <cstdlib>
#include <cstring>

#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

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

// out[y * ne + e] = sum over groups g in slice y (= blockIdx.y of gridDim.y) of
// partial[g * stride + e]; fixed order, deterministic
__global__ __launch_bounds__(kLB) void lspg_sum_kernel(const double *__restrict__ partial,
                                                       int ng, size_t stride, int ne,
                                                       double *__restrict__ out)
{
    const int e = blockIdx.x * kLB + threadIdx.x;
    if (e >= ne) return;
    const int ns = gridDim.y, y = blockIdx.y;
    const int g0 = (int)((long long)ng * y / ns), g1 = (int)((long long)ng * (y + 1) / ns);
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int g = g0;
    for (; g + 3 < g1; g += 4) {
        s0 += partial[(size_t)g * stride + e];
        s1 += partial[(size_t)(g + 1) * stride + e];
        s2 += partial[(size_t)(g + 2) * stride + e];
        s3 += partial[(size_t)(g + 3) * stride + e];
    }
    for (; g < g1; ++g) s0 += partial[(size_t)g * stride + e];
    out[(size_t)y * ne + e] = (s0 + s1) + (s2 + s3);
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

// Fused JV + augmented Gram on the matrix cores (v_mfma_f64_16x16x4_f64).
// A tile = kMC consecutive cells = 2 kMC rows of X = [JV | -R] staged in LDS
// (u-rows 0..kMC-1, v-rows kMC..2kMC-1; filled with lane = cell, so every
// basis-plane load is a contiguous run of cells).  G = X^T X is symmetric:
// only the NB (NB + 1) / 2 upper 16 x 16 blocks are formed, block pair p owned
// by wave p % 4 for the whole launch (no cross-wave reduction).  Per 4-row
// step a lane feeds A = X[row 4s + (l >> 4)][16 b1 + (l & 15)] and the same
// for b2 (the f64 16x16x4 operand map: A[m = l & 15][k = l >> 4],
// B[k = l >> 4][n = l & 15]); D lane l register i = G[16 b1 + (l >> 4) + 4 i]
// [16 b2 + (l & 15)] (cdna_hip_programming.md, f64 MFMA layout).  The row
// stride LD = P + 17 doubles keeps both the fill stores (lane = row) and the
// operand reads (4 rows x 16 columns) free of LDS bank conflicts.
constexpr int kMC = 32;
typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int NB, int CH>
__global__ __launch_bounds__(kLB) void lspg_gram_mfma_kernel(LspgArgs a, double *__restrict__ partial)
{
    constexpr int P = 16 * NB;
    constexpr int LD = P + 17;
    constexpr int NPAIR = NB * (NB + 1) / 2;
    constexpr int NQ = (NPAIR + 3) / 4;
    __shared__ double X[2 * kMC * LD];
    const int N = a.cf.nx;
    const size_t n = (size_t)N * N, m = 2 * n;
    const double al = a.cf.alpha;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // this wave's block pairs (upper triangle, row-major enumeration)
    int pb1[NQ], pb2[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        int p = wv + 4 * q, b1 = 0;
        if (p >= NPAIR) p = -1;
        int rem = p;
        while (rem >= 0 && rem >= NB - b1) {
            rem -= NB - b1;
            ++b1;
        }
        pb1[q] = p < 0 ? -1 : b1;
        pb2[q] = p < 0 ? -1 : b1 + rem;
    }
    dbl4 acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = dbl4{0.0, 0.0, 0.0, 0.0};

    const int j = tid & (kMC - 1), kg = tid / kMC;  // fill role: cell j, columns kg + 8 q
    const int orow = lane >> 4, ocol = lane & 15;    // MFMA operand role
    const size_t ntiles = (n + kMC - 1) / kMC;
    // columns per filling thread, loaded in chunks of CH: every load of a
    // chunk is issued before the first LDS store (a store between two loads
    // would otherwise serialise them -- one memory latency per column)
    constexpr int KPT = P / (kLB / kMC);
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const size_t i = t * kMC + j;
        const bool ok = i < n;
        const size_t ii = ok ? i : n - 1;
        const int r = (int)(ii / N), c = (int)(ii - (size_t)r * N);
        const bool west = c > 0, south = r > 0;
        const size_t iw = west ? ii - 1 : ii, is = south ? ii - N : ii;
        const double *u = a.w, *v = a.w + n, *uT = a.wT, *vT = a.wT + n;
        const double ui = u[ii], vi = v[ii], uW = u[iw], vW = v[iw];
        const double uTi = uT[ii], vTi = vT[ii], uTS = uT[is], vTS = vT[is];
        const double rui = a.r[ii], rvi = a.r[n + ii];
        const double ax = al * a.cf.inv_dx[c], axw = west ? al * a.cf.inv_dx[c - 1] : 0.0;
        const double ay = al * a.cf.inv_dy[r], ays = south ? al * a.cf.inv_dy[r - 1] : 0.0;
#pragma unroll
        for (int q0 = 0; q0 < KPT; q0 += CH) {
            double xl[CH][8];
#pragma unroll
            for (int q = 0; q < CH; ++q) {
                const int k = kg + (kLB / kMC) * (q0 + q);
                const int kk = k < a.npod ? k : a.npod - 1;  // always a valid plane
                const double *xu = a.bt + (size_t)kk * m, *xv = xu + n;
                const double *xuT = a.btT + (size_t)kk * m, *xvT = xuT + n;
                xl[q][0] = xu[ii], xl[q][1] = xv[ii], xl[q][2] = xu[iw], xl[q][3] = xv[iw];
                xl[q][4] = xuT[ii], xl[q][5] = xvT[ii], xl[q][6] = xuT[is], xl[q][7] = xvT[is];
            }
#pragma unroll
            for (int q = 0; q < CH; ++q) {
                const int k = kg + (kLB / kMC) * (q0 + q);
                if (q0 + q >= KPT) break;
                const double xui = xl[q][0], xvi = xl[q][1], xuw = xl[q][2], xvw = xl[q][3];
                const double xuTi = xl[q][4], xvTi = xl[q][5], xuTS = xl[q][6], xvTS = xl[q][7];
                const double mT = vTi * xuTi + uTi * xvTi;
                double yu = xui + ax * (ui * xui) + 0.5 * ay * mT;
                double yv = xvi + ay * (vTi * xvTi) + 0.5 * ax * (vi * xui + ui * xvi);
                if (west) {
                    yu -= axw * (uW * xuw);
                    yv -= 0.5 * axw * (vW * xuw + uW * xvw);
                }
                if (south) {
                    yu -= 0.5 * ays * (vTS * xuTS + uTS * xvTS);
                    yv -= ays * (vTS * xvTS);
                }
                if (k == a.npod) {
                    yu = -rui;
                    yv = -rvi;
                } else if (k > a.npod) {
                    yu = 0.0;
                    yv = 0.0;
                }
                if (!ok) {
                    yu = 0.0;
                    yv = 0.0;
                }
                X[j * LD + k] = yu;
                X[(kMC + j) * LD + k] = yv;
            }
        }
        __syncthreads();
#pragma unroll 4
        for (int s4 = 0; s4 < 2 * kMC; s4 += 4) {
            const double *xr = X + (s4 + orow) * LD + ocol;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                if (pb1[q] < 0) continue;
                const double av = xr[16 * pb1[q]], bv = xr[16 * pb2[q]];
                acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[q], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    double *out = partial + (size_t)blockIdx.x * P * P;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        if (pb1[q] < 0) continue;
        const int r0 = 16 * pb1[q], c0 = 16 * pb2[q];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int rr = r0 + orow + 4 * e, cc = c0 + ocol;
            out[(size_t)rr * P + cc] = acc[q][e];
            if (pb1[q] != pb2[q]) out[(size_t)cc * P + rr] = acc[q][e];
        }
    }
}

// Warp-specialised variant (default for every P): waves 4..4+FW-1 fill the
// X tile of the NEXT tile while waves 0..3 run the MFMAs on the current one,
// through two LDS buffers and one barrier per tile.  A filling thread
// issues the loads of all its KPT basis columns (8 each) before its first
// LDS store (in two halves at P = 96: the register budget of two waves per
// SIMD), so a tile costs one or two memory latencies, not one per column;
// the products and the Gram blocks are those of lspg_gram_mfma_kernel.
template <int NB, int FW>
__global__ __launch_bounds__(kLB + FW * 64) void lspg_gram_ws_kernel(LspgArgs a, double *__restrict__ partial)
{
    constexpr int P = 16 * NB;
    constexpr int LD = P + 17;
    constexpr int NPAIR = NB * (NB + 1) / 2;
    constexpr int NQ = (NPAIR + 3) / 4;
    constexpr int XS = 2 * kMC * LD;       // doubles per buffer
    constexpr int KS = FW * 64 / kMC;      // column stride of the filling threads
    constexpr int KPT = P / KS;            // basis columns per filling thread
    constexpr int CH = KPT > 8 ? KPT / 2 : KPT;  // loaded together (register budget)
    extern __shared__ double gram_lds[];   // two buffers of XS (dynamic)
    const int N = a.cf.nx;
    const size_t n = (size_t)N * N;
    const double al = a.cf.alpha;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const size_t ntiles = (n + kMC - 1) / kMC, ng = gridDim.x;
    const size_t cnt = blockIdx.x < ntiles ? (ntiles - 1 - blockIdx.x) / ng + 1 : 0;

    if (wv >= 4) {
        // ---- fill role: cell j of the tile, basis columns kg + 8 q
        const int ft = tid - kLB;
        const int j = ft & (kMC - 1), kg = ft / kMC;  // columns kg + KS q
        for (size_t it = 0; it <= cnt; ++it) {
            if (it < cnt) {
                double *X = gram_lds + (it & 1) * XS;
                const size_t i = (blockIdx.x + it * ng) * kMC + j;
                const bool ok = i < n;
                const size_t ii = ok ? i : n - 1;
                const int r = (int)(ii / N), c = (int)(ii - (size_t)r * N);
                const bool west = c > 0, south = r > 0;
                const size_t iw = west ? ii - 1 : ii, is = south ? ii - N : ii;
                // blocked basis: the (u, v) pair of cell i, column k, plane s
                // (0 straight, 1 transposed) at ((i / 32 * npod + k) * 2 + s) *
                // 64 + (i % 32) * 2 -- one 16-B load per pair; a tile's values
                // for all columns are one contiguous run (few pages, full lines)
                const size_t np = (size_t)a.npod;
                const double *bi = a.bk + (ii / kMC) * np * 128 + (ii % kMC) * 2;
                const double *bw = a.bk + (iw / kMC) * np * 128 + (iw % kMC) * 2;
                const double *bs = a.bk + (is / kMC) * np * 128 + (is % kMC) * 2 + 64;
                const double *u = a.w, *v = a.w + n, *uT = a.wT, *vT = a.wT + n;
                const double ui = u[ii], vi = v[ii], uW = u[iw], vW = v[iw];
                const double uTi = uT[ii], vTi = vT[ii], uTS = uT[is], vTS = vT[is];
                const double rui = a.r[ii], rvi = a.r[n + ii];
                const double ax = al * a.cf.inv_dx[c], axw = west ? al * a.cf.inv_dx[c - 1] : 0.0;
                const double ay = al * a.cf.inv_dy[r], ays = south ? al * a.cf.inv_dy[r - 1] : 0.0;
#pragma unroll
                for (int q0 = 0; q0 < KPT; q0 += CH) {
                    double xl[CH][8];
#pragma unroll
                    for (int q = 0; q < CH; ++q) {
                        const int k = kg + KS * (q0 + q);
                        const size_t ko = (size_t)(k < a.npod ? k : a.npod - 1) * 128;  // valid column
                        const double2 pi = *(const double2 *)(bi + ko);
                        const double2 pw = *(const double2 *)(bw + ko);
                        const double2 pt = *(const double2 *)(bi + ko + 64);
                        const double2 ps = *(const double2 *)(bs + ko);
                        xl[q][0] = pi.x, xl[q][1] = pi.y, xl[q][2] = pw.x, xl[q][3] = pw.y;
                        xl[q][4] = pt.x, xl[q][5] = pt.y, xl[q][6] = ps.x, xl[q][7] = ps.y;
                    }
#pragma unroll
                    for (int q = 0; q < CH; ++q) {
                        const int k = kg + KS * (q0 + q);
                        const double xui = xl[q][0], xvi = xl[q][1], xuw = xl[q][2], xvw = xl[q][3];
                        const double xuTi = xl[q][4], xvTi = xl[q][5], xuTS = xl[q][6], xvTS = xl[q][7];
                        const double mT = vTi * xuTi + uTi * xvTi;
                        double yu = xui + ax * (ui * xui) + 0.5 * ay * mT;
                        double yv = xvi + ay * (vTi * xvTi) + 0.5 * ax * (vi * xui + ui * xvi);
                        if (west) {
                            yu -= axw * (uW * xuw);
                            yv -= 0.5 * axw * (vW * xuw + uW * xvw);
                        }
                        if (south) {
                            yu -= 0.5 * ays * (vTS * xuTS + uTS * xvTS);
                            yv -= ays * (vTS * xvTS);
                        }
                        if (k == a.npod) {
                            yu = -rui;
                            yv = -rvi;
                        } else if (k > a.npod) {
                            yu = 0.0;
                            yv = 0.0;
                        }
                        if (!ok) {
                            yu = 0.0;
                            yv = 0.0;
                        }
                        X[j * LD + k] = yu;
                        X[(kMC + j) * LD + k] = yv;
                    }
                }
            }
            __syncthreads();
        }
        return;
    }
    // ---- MFMA role: this wave's block pairs (upper triangle, row-major)
    int pb1[NQ], pb2[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        int p = wv + 4 * q, b1 = 0;
        if (p >= NPAIR) p = -1;
        int rem = p;
        while (rem >= 0 && rem >= NB - b1) {
            rem -= NB - b1;
            ++b1;
        }
        pb1[q] = p < 0 ? -1 : b1;
        pb2[q] = p < 0 ? -1 : b1 + rem;
    }
    dbl4 acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = dbl4{0.0, 0.0, 0.0, 0.0};
    const int orow = lane >> 4, ocol = lane & 15;
    for (size_t it = 0; it <= cnt; ++it) {
        if (it >= 1) {
            const double *X = gram_lds + ((it - 1) & 1) * XS;
#pragma unroll 4
            for (int s4 = 0; s4 < 2 * kMC; s4 += 4) {
                const double *xr = X + (s4 + orow) * LD + ocol;
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    if (pb1[q] < 0) continue;
                    const double av = xr[16 * pb1[q]], bv = xr[16 * pb2[q]];
                    acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[q], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    }
    double *out = partial + (size_t)blockIdx.x * P * P;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        if (pb1[q] < 0) continue;
        const int r0 = 16 * pb1[q], c0 = 16 * pb2[q];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int rr = r0 + orow + 4 * e, cc = c0 + ocol;
            out[(size_t)rr * P + cc] = acc[q][e];
            if (pb1[q] != pb2[q]) out[(size_t)cc * P + rr] = acc[q][e];
        }
    }
}

// Blocked basis for the warp-specialised Gram kernel: bk[((t npod + k) 2 + s)
// 64 + 2 j + e] = component e (u, v) of plane s (0: bt, 1: btT) of basis
// column k at cell 32 t + j (zero past the last cell): each cell's (u, v)
// pair is one 16-B load.  Built once per LSPG run from bt / btT.
__global__ __launch_bounds__(kLB) void lspg_block_basis_kernel(const double *__restrict__ bt,
                                                               const double *__restrict__ btT,
                                                               size_t n, int npod,
                                                               double *__restrict__ bk)
{
    const size_t ntiles = (n + kMC - 1) / kMC;
    const size_t total = ntiles * (size_t)npod * 128;
    const size_t m = 2 * n;
    for (size_t o = (size_t)blockIdx.x * kLB + threadIdx.x; o < total; o += (size_t)gridDim.x * kLB) {
        const int e = (int)(o & 1), j = (int)((o >> 1) & 31), sp = (int)((o >> 6) & 1);
        const size_t tk = o >> 7;
        const size_t t = tk / npod, k = tk - t * npod;
        const size_t i = t * kMC + j;
        double x = 0.0;
        if (i < n) {
            const double *src = (sp ? btT : bt) + k * m + (size_t)e * n;
            x = src[i];
        }
        bk[o] = x;
    }
}

// LDS row stride of the Cholesky factor: LD = 1 (mod 32) doubles, so a column
// (lane = row) spreads over all 64 banks and a row (lane = column) too
__host__ __device__ inline int lspg_solve_ld(int npod) { return npod + ((33 - npod % 32) % 32); }

// One workgroup: Cholesky of the augmented matrix [[G, b], [b^T, .]]
// (G = G[0:npod, 0:npod], b = G[0:npod, npod], ld P -- the Gram kernel's
// augmented column), so the factor's last row is L^-1 b and no forward
// substitution is needed; then L^T dy = L^-1 b and y += dy.  err <- 1 when a
// pivot is not positive relative to its diagonal (rank-deficient JV).
// One barrier per column: column jj is consumed unscaled (L_ij L_kj / d) by
// the trailing update and its scaled copy is written to the unused upper
// triangle (row jj), where the back substitution reads it.
__global__ __launch_bounds__(kLB) void lspg_solve_kernel(const double *__restrict__ G, int P,
                                                         int npod, double *__restrict__ y,
                                                         double *__restrict__ dy_out,
                                                         unsigned *__restrict__ err)
{
    extern __shared__ double L[];  // (npod + 1) x LD, dynamic (lspg_solve_ld)
    __shared__ double rdg[kLspgMaxPod], d0[kLspgMaxPod], dyv[kLspgMaxPod];
    __shared__ int bad;
    const int n1 = npod + 1;
    const int LD = lspg_solve_ld(n1), tid = threadIdx.x;
    for (int e = tid; e < n1 * n1; e += kLB) {
        const int i = e / n1, k = e - i * n1;
        L[i * LD + k] = G[(size_t)i * P + k];
    }
    for (int i = tid; i < npod; i += kLB) d0[i] = G[(size_t)i * P + i];
    if (tid == 0) bad = 0;
    __syncthreads();
    const int kk = tid & 127, half = tid >> 7;
    for (int jj = 0; jj < npod; ++jj) {
        const double d = L[jj * LD + jj];
        const double dd = d > 0.0 ? d : 1.0;
        const double rp = rsqrt(dd), rd = 1.0 / dd;
        if (tid == 0) {
            // a pivot that lost all but ~8 ulp of its column's norm: rank-deficient
            if (!(d > 0x1p-49 * d0[jj])) bad = 1;
            rdg[jj] = rp;
        }
        // scaled column jj (rows jj+1..npod) -> upper row jj
        for (int i = jj + 1 + tid; i <= npod; i += kLB) L[jj * LD + i] = L[i * LD + jj] * rp;
        const int k = jj + 1 + kk;
        if (k <= npod) {
            // rows i >= k of this half, 8 at a time: all loads issued before
            // the stores (the rows are distinct; one LDS latency per 8 rows)
            const double lk = L[k * LD + jj] * rd;
            const int i00 = k - ((k - (jj + 1 + half)) & 1);
            for (int i0 = i00; i0 <= npod; i0 += 16) {
                double li[8], lik[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int i = i0 + 2 * q;
                    const bool on = i <= npod && i >= k;
                    li[q] = on ? L[i * LD + jj] : 0.0;
                    lik[q] = on ? L[i * LD + k] : 0.0;
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int i = i0 + 2 * q;
                    if (i <= npod && i >= k) L[i * LD + k] = lik[q] - li[q] * lk;
                }
            }
        }
        __syncthreads();
    }
    // L^T dy = z, z_j = (L^-1 b)_j = upper row j, column npod; L^T row j = upper row j
    for (int jj = npod - 1; jj >= 0; --jj) {
        const double dj = L[jj * LD + npod] * rdg[jj];
        if (tid == 0) dyv[jj] = dj;
        for (int i = tid; i < jj; i += kLB) L[i * LD + npod] -= L[i * LD + jj] * dj;
        __syncthreads();
    }
    for (int i = tid; i < npod; i += kLB) {
        y[i] += dyv[i];
        if (dy_out) dy_out[i] = dyv[i];
    }
    if (tid == 0 && bad) *err = 1u;
}

// library solve (rocSOLVER potrf/potrs on G in place): the diagonal before
// the factorisation, then the rank check and y += dy (dy = G[npod*P..])
__global__ __launch_bounds__(kLB) void lspg_diag_kernel(const double *__restrict__ G, int P,
                                                        int npod, double *__restrict__ d0)
{
    const int k = blockIdx.x * kLB + threadIdx.x;
    if (k < npod) d0[k] = G[(size_t)k * P + k];
}

__global__ __launch_bounds__(kLB) void lspg_finish_kernel(const double *__restrict__ G, int P,
                                                          int npod, const double *__restrict__ d0,
                                                          const int *__restrict__ info,
                                                          double *__restrict__ y,
                                                          unsigned *__restrict__ err)
{
    const int k = blockIdx.x * kLB + threadIdx.x;
    if (k >= npod) return;
    const double l = G[(size_t)k * P + k];
    if (*info != 0 || !(l * l > 0x1p-49 * d0[k])) *err = 1u;
    y[k] += G[(size_t)npod * P + k];
}

constexpr int kMfmaGroups = 512;  // 2 per CU (57 KB of LDS each at P = 96)
constexpr int kSumSlices = 16;
constexpr size_t kMaxGramGroups = 1024;  // partial buffers are sized for this many

// basis columns per load chunk of the Gram kernel's fill (BURG_LSPG_CH: 3, 4
// or 6 at P = 96 -- a tuning knob; 4 by default)
int gram_chunk()
{
    static int v = 0;
    if (!v) {
        v = 4;
        if (const char *e = std::getenv("BURG_LSPG_CH")) {
            const int x = std::atoi(e);
            if (x == 3 || x == 6) v = x;
        }
    }
    return v;
}

// the one-role MFMA kernel (BURG_LSPG_GRAM=split) serves P <= 96 (npod <= 95);
// there P = 128 uses the vector kernel
bool use_mfma(int P) { return P <= 96; }

// BURG_LSPG_GRAM=split selects the one-role MFMA kernel (fill, then MFMA)
bool gram_ws()
{
    static int v = -1;
    if (v < 0) {
        const char *e = std::getenv("BURG_LSPG_GRAM");
        v = (e && std::strcmp(e, "split") == 0) ? 0 : 1;
    }
    return v == 1;
}

// fill waves of the P = 96 ws kernel: 8 (each filling thread loads its 6
// columns at once; 0.96 ms at 1024^2) or 4 (BURG_LSPG_FILL_WAVES=4: 12
// columns in two halves, 1.03 ms)
int gram_fill_waves()
{
    static int v = 0;
    if (!v) {
        const char *e = std::getenv("BURG_LSPG_FILL_WAVES");
        v = (e && std::atoi(e) == 4) ? 4 : 8;
    }
    return v;
}

size_t gram_ws_lds(int P) { return sizeof(double) * 2 * 2 * kMC * (size_t)(P + 17); }

const void *gram_fn(int P)
{
    if (gram_ws()) {
        switch (P) {
        case 32: return (const void *)lspg_gram_ws_kernel<2, 4>;
        case 64: return (const void *)lspg_gram_ws_kernel<4, 4>;
        case 96:
            return gram_fill_waves() == 8 ? (const void *)lspg_gram_ws_kernel<6, 8>
                                          : (const void *)lspg_gram_ws_kernel<6, 4>;
        case 128: return (const void *)lspg_gram_ws_kernel<8, 4>;  // (8 fill waves: spills)
        default: break;
        }
    }
    switch (P) {
    case 32: return (const void *)lspg_gram_mfma_kernel<2, 4>;
    case 64: return (const void *)lspg_gram_mfma_kernel<4, 4>;
    case 96:
        return gram_chunk() == 6   ? (const void *)lspg_gram_mfma_kernel<6, 6>
               : gram_chunk() == 3 ? (const void *)lspg_gram_mfma_kernel<6, 3>
                                   : (const void *)lspg_gram_mfma_kernel<6, 4>;
    case 128: return (const void *)lspg_gram_kernel<8>;
    default: return nullptr;
    }
}

bool is_ws(int P) { return gram_ws() && P <= 128; }
int gram_threads(int P) { return is_ws(P) ? kLB + 64 * (P == 96 ? gram_fill_waves() : 4) : kLB; }
size_t gram_dyn(int P) { return is_ws(P) ? gram_ws_lds(P) : 0; }
bool gram_prepare(const void *fn, int P)
{
    if (!is_ws(P)) return true;
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)gram_dyn(P)) ==
           hipSuccess;
}

// one resident wave of workgroups (occupancy x CUs; BURG_LSPG_GROUPS
// overrides), at most one per tile
int groups_for(size_t n, int P)
{
    const bool m = use_mfma(P) || is_ws(P);
    const size_t cells = m ? kMC : kGC;
    size_t cap = m ? kMfmaGroups : kGroups;
    int dev = 0, ncu = 0, per = 0;
    if (const void *fn = gram_fn(P))
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            gram_prepare(fn, P) &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, gram_threads(P), gram_dyn(P)) ==
                hipSuccess &&
            per > 0)
            cap = (size_t)per * ncu;
    if (const char *e = std::getenv("BURG_LSPG_GROUPS")) {
        const long v = std::atol(e);
        if (v > 0 && v <= 4096) cap = (size_t)v;
    }
    if (cap > kMaxGramGroups) cap = kMaxGramGroups;
    const size_t tiles = (n + cells - 1) / cells;
    return (int)(tiles < cap ? tiles : cap);
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
    return (size_t)(kMaxGramGroups + kSumSlices) * P * P + (size_t)npod * 256;
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

bool lspg_gram_blocked(int npod) { return is_ws(lspg_cols(npod)); }

size_t lspg_blocked_count(size_t n, int npod) { return (n + kMC - 1) / kMC * (size_t)npod * 128; }

int launch_lspg_block_basis(const double *bt, const double *btT, size_t n, int npod, double *bk,
                            hipStream_t st)
{
    const size_t total = lspg_blocked_count(n, npod);
    size_t g = (total + kLB - 1) / kLB;
    if (g > 65536) g = 65536;
    hipLaunchKernelGGL(lspg_block_basis_kernel, dim3((unsigned)g), dim3(kLB), 0, st, bt, btT, n,
                       npod, bk);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_lspg_gram(const LspgArgs &a, double *partial, double *G, hipStream_t st)
{
    const int P = lspg_cols(a.npod);
    const int ng = groups_for((size_t)a.cf.nx * a.cf.nx, P);
    const void *fn = gram_fn(P);
    if (!fn || !gram_prepare(fn, P) || (is_ws(P) && !a.bk)) return -1;
    LspgArgs args = a;
    void *kargs[] = {&args, &partial};
    if (hipLaunchKernel(fn, dim3(ng), dim3(gram_threads(P)), kargs, gram_dyn(P), st) != hipSuccess)
        return -3;
    // two-level deterministic reduction of the per-workgroup partials
    const int PP = P * P;
    double *mid = partial + (size_t)ng * PP;
    hipLaunchKernelGGL(lspg_sum_kernel, dim3((PP + kLB - 1) / kLB, kSumSlices), dim3(kLB), 0, st,
                       (const double *)partial, ng, (size_t)PP, PP, mid);
    hipLaunchKernelGGL(lspg_sum_kernel, dim3((PP + kLB - 1) / kLB, 1), dim3(kLB), 0, st,
                       (const double *)mid, kSumSlices, (size_t)PP, PP, G);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_lspg_solve_lib(void *handle, double *G, int npod, double *d0, int *info, double *y,
                          unsigned *err, hipStream_t st)
{
    // G is symmetric: its row-major (P x P) storage is the column-major one
    rocblas_handle h = (rocblas_handle)handle;
    const int P = lspg_cols(npod);
    hipLaunchKernelGGL(lspg_diag_kernel, dim3(1), dim3(kLB), 0, st, (const double *)G, P, npod, d0);
    if (rocsolver_dpotrf(h, rocblas_fill_lower, npod, G, P, info) != rocblas_status_success)
        return -3;
    if (rocsolver_dpotrs(h, rocblas_fill_lower, npod, 1, G, P, G + (size_t)npod * P, npod) !=
        rocblas_status_success)
        return -3;
    hipLaunchKernelGGL(lspg_finish_kernel, dim3(1), dim3(kLB), 0, st, (const double *)G, P, npod,
                       (const double *)d0, (const int *)info, y, err);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_lspg_solve(const double *G, int npod, double *y, double *dy, unsigned *err,
                      hipStream_t st)
{
    static bool attr = false;
    const size_t lds = sizeof(double) * (size_t)(npod + 1) * lspg_solve_ld(npod + 1);
    if (!attr) {
        if (hipFuncSetAttribute((const void *)lspg_solve_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)(sizeof(double) * (kLspgMaxPod + 1) *
                                      lspg_solve_ld(kLspgMaxPod + 1))) !=
            hipSuccess)
            return -3;
        attr = true;
    }
    hipLaunchKernelGGL(lspg_solve_kernel, dim3(1), dim3(kLB), lds, st, G, lspg_cols(npod), npod,
                       y, dy, err);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace burg
