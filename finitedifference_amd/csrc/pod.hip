// pod.hip -- POD of a snapshot matrix on the GPU (SURVEY.md section 8(f),
// row 4): POD(snaps, num_modes, method), C/hypernet2D.py:2670-2695, as called
// by C/run_prom.py:58-86 on the (2n, 9 x 501) training snapshot set.
//
// The reference calls np.linalg.svd (method 'svd') or sklearn's
// randomized_svd (method 'rsvd', unseeded).  Here: the exact thin SVD by
// Householder QR of the tall snapshot matrix and an SVD of its small R factor,
//     S = Q R,  R = U_R Sigma V^T,  U = Q [U_R; 0]
// all with rocSOLVER on the device (dgeqrf, dgesvd, dormqr), so the basis
// keeps LAPACK's backward stability (the method of snapshots, eig(S^T S),
// would square the condition number and lose the trailing modes).  The
// host's C-order (m x ns) matrix is a column-major (ns x m) one, so it is
// transposed once on the device (basis_transpose_kernel, ecsw.hip); the
// result is transposed back into C-order (m x k).  Signs: each column is
// flipped so that its largest-magnitude entry is positive (sklearn's
// svd_flip rule on U) -- LAPACK's signs are arbitrary.
#include "burg_internal.h"

#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace burg {
namespace {

constexpr int kPB = 256;

// R (upper triangle of the QR factor, column-major lda) -> dense ns x ns
__global__ __launch_bounds__(kPB) void triu_copy_kernel(const double *__restrict__ a, size_t lda,
                                                        int ns, double *__restrict__ r)
{
    const size_t e = (size_t)blockIdx.x * kPB + threadIdx.x;
    if (e >= (size_t)ns * ns) return;
    const int col = (int)(e / ns), row = (int)(e % ns);
    r[e] = row <= col ? a[(size_t)col * lda + row] : 0.0;
}

// C (m x k column-major, ldc = m) <- [U_R[:, :k]; 0]
__global__ __launch_bounds__(kPB) void embed_kernel(const double *__restrict__ ur, int ns, int k,
                                                    size_t m, double *__restrict__ c)
{
    const size_t e = (size_t)blockIdx.x * kPB + threadIdx.x;
    if (e >= m * k) return;
    const size_t col = e / m, row = e % m;
    c[e] = row < (size_t)ns ? ur[col * ns + row] : 0.0;
}

// per column of C (m x k column-major): sign of its largest-|.| entry
__global__ __launch_bounds__(kPB) void col_sign_kernel(const double *__restrict__ c, size_t m,
                                                       double *__restrict__ sgn)
{
    const double *p = c + (size_t)blockIdx.x * m;
    double best = -1.0, val = 0.0;
    for (size_t i = threadIdx.x; i < m; i += kPB) {
        const double a = fabs(p[i]);
        if (a > best) best = a, val = p[i];
    }
    __shared__ double bb[kPB], bv[kPB];
    bb[threadIdx.x] = best;
    bv[threadIdx.x] = val;
    __syncthreads();
    for (int h = kPB / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h && bb[threadIdx.x + h] > bb[threadIdx.x]) {
            bb[threadIdx.x] = bb[threadIdx.x + h];
            bv[threadIdx.x] = bv[threadIdx.x + h];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) sgn[blockIdx.x] = bv[0] < 0.0 ? -1.0 : 1.0;
}

__global__ __launch_bounds__(kPB) void col_scale_kernel(double *__restrict__ c, size_t m, int k,
                                                        const double *__restrict__ sgn)
{
    const size_t e = (size_t)blockIdx.x * kPB + threadIdx.x;
    if (e >= m * k) return;
    c[e] *= sgn[e / m];
}

unsigned blocks(size_t n) { return (unsigned)((n + kPB - 1) / kPB); }

// C (m x n, column-major, ldc) = sum over p < parts of W[p] (m x n, packed)
__global__ __launch_bounds__(kPB) void sum_parts_kernel(const double *__restrict__ w, int parts,
                                                        int m, int n, double *__restrict__ c,
                                                        int ldc)
{
    const size_t e = (size_t)blockIdx.x * kPB + threadIdx.x;
    const size_t mn = (size_t)m * n;
    if (e >= mn) return;
    double t = 0.0;
    for (int p = 0; p < parts; ++p) t += w[(size_t)p * mn + e];
    c[(e / m) * ldc + e % m] = t;
}

// C = A^T B for tall A (k x m) and B (k x n), column-major, k >> m, n: the
// reductions of the randomized SVD (Y^T Y, S^T Q, Q^T S).  rocBLAS tiles only
// the m x n output (a 105 x 105 Gram is ONE 128 x 192 macro tile: one
// workgroup walks all 125 000 rows, ~20 ms); here the k rows are split into
// `parts` chunks (one strided-batched dgemm, parts x tiles workgroups) whose
// partial products are summed by sum_parts_kernel.  The summation order
// differs from one dgemm's, within the same rounding bound.  work: parts x m
// x n doubles (+ m x n for the ragged tail).
rocblas_status gemm_tn_splitk(rocblas_handle h, hipStream_t st, rocblas_int m, rocblas_int n,
                              rocblas_int k, const double *a, rocblas_int lda, const double *b,
                              rocblas_int ldb, double *c, rocblas_int ldc, double *work, int parts)
{
    const double one = 1.0, zero = 0.0;
    if (parts <= 1 || k < 2 * parts)
        return rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_none, m, n, k, &one,
                             a, lda, b, ldb, &zero, c, ldc);
    const rocblas_int kp = k / parts, tail = k - kp * parts;
    const rocblas_stride mn = (rocblas_stride)m * n;
    rocblas_status s = rocblas_dgemm_strided_batched(
        h, rocblas_operation_transpose, rocblas_operation_none, m, n, kp, &one, a, lda, kp, b, ldb,
        kp, &zero, work, m, mn, parts);
    if (s != rocblas_status_success) return s;
    int np = parts;
    if (tail) {
        s = rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_none, m, n, tail, &one,
                          a + (size_t)kp * parts, lda, b + (size_t)kp * parts, ldb, &zero,
                          work + (size_t)parts * mn, m);
        if (s != rocblas_status_success) return s;
        ++np;
    }
    hipLaunchKernelGGL(sum_parts_kernel, dim3(blocks((size_t)mn)), dim3(kPB), 0, st,
                       (const double *)work, np, (int)m, (int)n, c, (int)ldc);
    return hipGetLastError() == hipSuccess ? rocblas_status_success : rocblas_status_internal_error;
}

// k-chunks for gemm_tn_splitk: enough (output tiles x chunks >= ~512
// workgroups) to fill the chip, each chunk >= 512 rows
int splitk_parts(rocblas_int m, rocblas_int n, rocblas_int k)
{
    const long tiles = (long)((m + 127) / 128) * ((n + 127) / 128);
    long p = (512 + tiles - 1) / tiles;
    p = std::min<long>(p, std::max<long>(1, k / 512));
    return (int)std::max<long>(1, std::min<long>(p, 256));
}

// G (R x R, column-major) += shift * I with shift = c * trace(G): the shifted
// first pass of CholeskyQR3 (Fukaya et al., "Shifted Cholesky QR for
// computing the QR factorization of ill-conditioned matrices", 2020):
// c = 11 (m R + R (R + 1)) u bounds ||Y||_2^2 <= trace(G) and keeps the
// Cholesky factorisation of G + shift I from breaking down for any
// cond(Y) < 1/u.  One workgroup.
__global__ __launch_bounds__(kPB) void shift_diag_kernel(double *__restrict__ g, int r, double c,
                                                         int ldg)
{
    __shared__ double part[kPB];
    double t = 0.0;
    for (int i = threadIdx.x; i < r; i += kPB) t += g[(size_t)i * ldg + i];
    part[threadIdx.x] = t;
    __syncthreads();
    for (int h = kPB / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) part[threadIdx.x] += part[threadIdx.x + h];
        __syncthreads();
    }
    const double shift = c * part[0];
    for (int i = threadIdx.x; i < r; i += kPB) g[(size_t)i * ldg + i] += shift;
}

// Orthonormal basis of the columns of Y (rows x r, column-major, in place):
// shifted CholeskyQR3 -- G = Y^T Y (one dgemm on the matrix cores), Cholesky
// G = R^T R, Y <- Y R^-1 (dtrsm); once with the shift, then twice plain --
// instead of Householder's r sequential panel steps (dgeqrf + dorgqr: ~100
// small gemv launches each).  Falls back to Householder if a Cholesky factor
// breaks down (info != 0: Y numerically rank deficient beyond the shift's
// reach).  Returns a rocblas_status (0 = success); *householder is set when
// the fallback ran.
rocblas_status orth_columns(rocblas_handle h, hipStream_t st, rocblas_int rows, rocblas_int r,
                            double *y, double *g, double *tau, rocblas_int *info, double *work,
                            bool *householder)
{
    const double one = 1.0;
    const double u = 0x1p-53;
    const double c = 11.0 * ((double)rows * r + (double)r * (r + 1)) * u;
    rocblas_status s;
    *householder = false;
    for (int pass = 0; pass < 3; ++pass) {
        if ((s = gemm_tn_splitk(h, st, r, r, rows, y, rows, y, rows, g, r, work,
                                splitk_parts(r, r, rows))) != rocblas_status_success)
            return s;
        if (pass == 0) hipLaunchKernelGGL(shift_diag_kernel, dim3(1), dim3(kPB), 0, st, g, (int)r, c, (int)r);
        if ((s = rocsolver_dpotrf(h, rocblas_fill_upper, r, g, r, info)) != rocblas_status_success)
            return s;
        rocblas_int hinfo = 0;
        if (hipMemcpyAsync(&hinfo, info, sizeof hinfo, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return rocblas_status_internal_error;
        if (hinfo != 0) {  // Y is left as the last successful pass made it: same span
            *householder = true;
            if ((s = rocsolver_dgeqrf(h, rows, r, y, rows, tau)) != rocblas_status_success) return s;
            return rocsolver_dorgqr(h, rows, r, r, y, rows, tau);
        }
        if ((s = rocblas_dtrsm(h, rocblas_side_right, rocblas_fill_upper, rocblas_operation_none,
                               rocblas_diagonal_non_unit, rows, r, &one, g, r, y, rows)) !=
            rocblas_status_success)
            return s;
    }
    return rocblas_status_success;
}

// ---- Tall-skinny products on the matrix cores ------------------------------
//
// The randomized SVD's work is its 16 products with the (m x ns) snapshot
// matrix S -- Y = S Z (m x R) and Z = S^T Y (ns x R), R = nrand = 105: 118
// GFLOP each at 250^2 x 9 mu (125 000 x 4 509), 26 flop per byte of S, so
// bound by the fp64 matrix rate (v_mfma_f64_16x16x4_f64; 78.6 TF/s peak, the
// same as fp64 VALU FMA) rather than by HBM.  The kernels below use S as it
// lies (C-order = row-major: no transposed copy), keep every thin operand
// row-major with its columns padded with zeros to Rp = 16 NB <= 128, stage
// the thin operand through LDS 32 reduction rows at a time (double-buffered,
// one barrier per chunk; its next chunk and the next A operands are loaded
// into registers before the MFMAs of the current one and stored to LDS
// after them), and give every wave a 32 x Rp block of the output in
// accumulators (2 x NB 16 x 16 tiles):
//  * gemm_nn_kernel: C (m x n) = A (m x K) B (K x n); a workgroup owns 128
//    rows of A (4 waves x 32) and the whole K reduction;
//  * gemm_tn_kernel: W_p (K x Rp) = A_p^T B_p over row part p; a workgroup
//    owns 128 columns of A and one part; sum_rows_kernel adds the parts in a
//    fixed order (deterministic).  Parts map to XCDs (blockIdx mod 8) so
//    that every column tile of a part runs on one XCD and reads B_p through
//    that XCD's L2.
// An MFMA's 4 k slots may carry any 4 reduction indices as long as A and B
// agree: slot s4 = lane >> 4 takes k = 8 s4 + s in the s-th of the 8 MFMAs
// of a chunk, so a lane's A operands of gemm_nn are 8 consecutive doubles of
// one row of S, and gemm_tn's 16 lanes of a slot read 128 contiguous bytes.
typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int kTK = 32;   // reduction rows per chunk
constexpr int kTW = 256;  // threads per workgroup (4 waves)

struct TsArgs {
    const double *a;  // row-major, row stride lda
    const double *b;  // row-major (reduction x n), row stride ldb
    double *c;        // nn: (m x n), row stride ldc; tn: parts x K x (16 NB) partials
    size_t lda, ldb, ldc;
    size_t m;         // rows of A (and of B for tn)
    int K;            // nn: columns of A = rows of B; tn: columns of A = output rows
    int n;            // valid columns of B and of the output
    int jtiles;       // tn: column tiles of 128
    size_t part_rows; // tn: rows per part
};

// LDS row stride of the staged thin operand: the rows the 4 k slots read in
// one instruction must fall in different bank halves (gemm_nn: slots 2 rows
// apart -> +8; gemm_tn: slots 8 rows apart -> +2)
template <int NB, bool NN>
constexpr int ts_ldb() { return 16 * NB + (NN ? 8 : 2); }

// reduction row of k slot s4 in MFMA step s (0..7) of a chunk: gemm_tn
// 8 s4 + s; gemm_nn 8 (s / 2) + 2 s4 + s % 2 (a lane's A operands are then
// 16-B pairs, and the 4 slots of a row read 64 contiguous bytes per load)
template <bool NN>
__device__ __forceinline__ int ts_krow(int s4, int s)
{
    return NN ? 8 * (s >> 1) + 2 * s4 + (s & 1) : 8 * s4 + s;
}

template <int NB, bool NN, int OCC>
__device__ __forceinline__ void ts_mfma_chunk(const double *bs, int cl, int s4,
                                              const double (&av)[2][8], dbl4 (&acc)[2][NB])
{
    constexpr int LDB = ts_ldb<NB, NN>();
    if constexpr (OCC == 2) {  // registers are scarce; the other workgroup covers the reads
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const double *brow = bs + ts_krow<NN>(s4, s) * LDB + cl;
#pragma unroll
            for (int cb = 0; cb < NB; ++cb) {
                const double bv = brow[16 * cb];
                acc[0][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[0][s], bv, acc[0][cb], 0, 0, 0);
                acc[1][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[1][s], bv, acc[1][cb], 0, 0, 0);
            }
        }
        return;
    }
    // the B operands of step s + 1 are read from LDS while the MFMAs of step s run
    double bv[2][NB];
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) bv[0][cb] = bs[ts_krow<NN>(s4, 0) * LDB + cl + 16 * cb];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        if (s < 7) {
            const double *brow = bs + ts_krow<NN>(s4, s + 1) * LDB + cl;
#pragma unroll
            for (int cb = 0; cb < NB; ++cb) bv[(s + 1) & 1][cb] = brow[16 * cb];
        }
#pragma unroll
        for (int cb = 0; cb < NB; ++cb) {
            acc[0][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[0][s], bv[s & 1][cb], acc[0][cb], 0, 0, 0);
            acc[1][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[1][s], bv[s & 1][cb], acc[1][cb], 0, 0, 0);
        }
    }
}

// this thread's share (2 NB doubles) of a kTK x 16 NB chunk of the thin
// operand: rows r0 .. r0 + kTK - 1 (valid below r_end), columns below n
template <int NB>
__device__ __forceinline__ void ts_load_b(const TsArgs &g, size_t r0, size_t r_end,
                                          double (&bn)[2 * NB])
{
    constexpr int NC = 16 * NB;
#pragma unroll
    for (int q = 0; q < 2 * NB; ++q) {
        const int e = threadIdx.x + kTW * q;
        const int kk = e / NC, cc = e % NC;
        const size_t r = r0 + kk;
        bn[q] = (r < r_end && cc < g.n) ? g.b[r * g.ldb + cc] : 0.0;
    }
}

template <int NB, bool NN>
__device__ __forceinline__ void ts_store_b(double *bs, const double (&bn)[2 * NB])
{
    constexpr int NC = 16 * NB, LDB = ts_ldb<NB, NN>();
#pragma unroll
    for (int q = 0; q < 2 * NB; ++q) {
        const int e = threadIdx.x + kTW * q;
        bs[(e / NC) * LDB + e % NC] = bn[q];
    }
}

typedef double dbl2u __attribute__((ext_vector_type(2), aligned(8)));

// OCC = 1: one workgroup per CU (208 VGPRs + 112 accumulator AGPRs), the
// next chunk's A operands prefetched into registers; OCC = 2: two per CU (<=
// 256 registers a wave), A loaded after the barrier -- the other
// workgroup's MFMAs cover the wait
template <int NB, int OCC>
__global__ __launch_bounds__(kTW, OCC) void gemm_nn_kernel(TsArgs g)
{
    constexpr int LDB = ts_ldb<NB, true>();
    __shared__ double bs[2][kTK * LDB];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int cl = lane & 15, s4 = lane >> 4;
    const size_t row0 = (size_t)blockIdx.x * 128 + (size_t)w * 32;
    const double *ap[2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
        const size_t r = row0 + 16 * rb + cl;
        ap[rb] = g.a + (r < g.m ? r : g.m - 1) * g.lda;  // rows past m: results dropped
    }
    dbl4 acc[2][NB];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int cb = 0; cb < NB; ++cb) acc[rb][cb] = dbl4{0.0, 0.0, 0.0, 0.0};
    const int nch = (g.K + kTK - 1) / kTK;
    double av[2][8], an[2][8], bn[2 * NB];
    auto load_a = [&](int ch, double (&an)[2][8]) {
        const int kb = ch * kTK + 2 * s4;  // + 8 q + e for the operand of step 2 q + e
        if (ch * kTK + kTK <= g.K) {        // whole chunk: 16-B loads (rows are 8-B aligned)
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const dbl2u v = *(const dbl2u *)(ap[rb] + kb + 8 * q);
                    an[rb][2 * q] = v.x;
                    an[rb][2 * q + 1] = v.y;
                }
        } else {
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    const int k = kb + 8 * (s >> 1) + (s & 1);
                    an[rb][s] = k < g.K ? ap[rb][k] : 0.0;
                }
        }
    };
    if constexpr (OCC == 1) load_a(0, an);
    ts_load_b<NB>(g, 0, (size_t)g.K, bn);
    ts_store_b<NB, true>(bs[0], bn);
    for (int ch = 0; ch < nch; ++ch) {
        __syncthreads();
        const bool more = ch + 1 < nch;
        if constexpr (OCC == 1) {
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
#pragma unroll
                for (int s = 0; s < 8; ++s) av[rb][s] = an[rb][s];
            if (more) load_a(ch + 1, an);
        } else {
            load_a(ch, av);
        }
        // OCC = 1: the next B chunk in flight during the MFMAs; OCC = 2: loaded after
        // them (registers: bn is not live across the MFMA block)
        if (OCC == 1 && more) ts_load_b<NB>(g, (size_t)(ch + 1) * kTK, (size_t)g.K, bn);
        ts_mfma_chunk<NB, true, OCC>(bs[ch & 1], cl, s4, av, acc);
        if (OCC == 2 && more) ts_load_b<NB>(g, (size_t)(ch + 1) * kTK, (size_t)g.K, bn);
        if (more) ts_store_b<NB, true>(bs[(ch + 1) & 1], bn);
    }
    // D layout of the f64 MFMA: column lane & 15, row (lane >> 4) + 4 q
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int cb = 0; cb < NB; ++cb)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const size_t r = row0 + 16 * rb + s4 + 4 * q;
                const int col = 16 * cb + cl;
                if (r < g.m && col < g.n) g.c[r * g.ldc + col] = acc[rb][cb][q];
            }
}

template <int NB, int OCC>
__global__ __launch_bounds__(kTW, OCC) void gemm_tn_kernel(TsArgs g)
{
    constexpr int NC = 16 * NB, LDB = ts_ldb<NB, false>();
    __shared__ double bs[2][kTK * LDB];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int cl = lane & 15, s4 = lane >> 4;
    const int x = blockIdx.x & 7, q8 = blockIdx.x >> 3;
    const int p = x + 8 * (q8 / g.jtiles), jt = q8 % g.jtiles;
    const size_t i_beg = std::min(g.m, (size_t)p * g.part_rows);
    const size_t i_end = std::min(g.m, i_beg + g.part_rows);
    const int j0 = jt * 128 + w * 32;
    const double *ap[2];
    bool jok[2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
        const int j = j0 + 16 * rb + cl;
        jok[rb] = j < g.K;
        ap[rb] = g.a + (jok[rb] ? j : 0);
    }
    dbl4 acc[2][NB];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int cb = 0; cb < NB; ++cb) acc[rb][cb] = dbl4{0.0, 0.0, 0.0, 0.0};
    const int nch = (int)((i_end - i_beg + kTK - 1) / kTK);
    double av[2][8], an[2][8], bn[2 * NB];
    auto load_a = [&](int ch, double (&an)[2][8]) {
        const size_t i0 = i_beg + (size_t)ch * kTK + 8 * s4;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const double *p = ap[rb] + i0 * g.lda;
#pragma unroll
            for (int s = 0; s < 8; ++s, p += g.lda)
                an[rb][s] = (jok[rb] && i0 + s < i_end) ? *p : 0.0;
        }
    };
    if (nch > 0) {
        if constexpr (OCC == 1) load_a(0, an);
        ts_load_b<NB>(g, i_beg, i_end, bn);
        ts_store_b<NB, false>(bs[0], bn);
    }
    for (int ch = 0; ch < nch; ++ch) {
        __syncthreads();
        const bool more = ch + 1 < nch;
        if constexpr (OCC == 1) {
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
#pragma unroll
                for (int s = 0; s < 8; ++s) av[rb][s] = an[rb][s];
            if (more) load_a(ch + 1, an);
        } else {
            load_a(ch, av);
        }
        // OCC = 1: the next B chunk in flight during the MFMAs; OCC = 2: loaded after
        // them (registers: bn is not live across the MFMA block)
        if (OCC == 1 && more) ts_load_b<NB>(g, i_beg + (size_t)(ch + 1) * kTK, i_end, bn);
        ts_mfma_chunk<NB, false, OCC>(bs[ch & 1], cl, s4, av, acc);
        if (OCC == 2 && more) ts_load_b<NB>(g, i_beg + (size_t)(ch + 1) * kTK, i_end, bn);
        if (more) ts_store_b<NB, false>(bs[(ch + 1) & 1], bn);
    }
    double *wp = g.c + (size_t)p * g.K * NC;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int cb = 0; cb < NB; ++cb)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = j0 + 16 * rb + s4 + 4 * q;
                if (j < g.K) wp[(size_t)j * NC + 16 * cb + cl] = acc[rb][cb][q];
            }
}

// out (K x n, row stride ldo) = sum over p < parts of W[p] (K x nc packed), in order
__global__ __launch_bounds__(kPB) void sum_rows_kernel(const double *__restrict__ w, int parts,
                                                       int K, int nc, int n,
                                                       double *__restrict__ out, int ldo)
{
    const size_t e = (size_t)blockIdx.x * kPB + threadIdx.x;
    if (e >= (size_t)K * n) return;
    const size_t j = e / n, c = e % n;
    const size_t kn = (size_t)K * nc;
    double t = 0.0;
    for (int p = 0; p < parts; ++p) t += w[p * kn + j * nc + c];
    out[j * ldo + c] = t;
}

// SVD of a small square matrix M (R x R, R <= 128) in one workgroup: one-sided
// Jacobi (Hestenes) on the columns of M held column-major in LDS -- cyclic
// round-robin sweeps, R/2 disjoint column pairs per step (16 waves, a pair
// per wave at a time, rows over the lanes), each pair rotated until
// |a_p . a_q| <= sqrt(R) eps ||a_p|| ||a_q||; then sigma_j = ||a_j|| and
// u_j = a_j / sigma_j, sorted by decreasing sigma.  Relative accuracy for
// every singular value (no bidiagonalisation): the small SVD of the
// randomized SVD (B = Q^T S) after B^T = Q_b R_b, replacing rocSOLVER's
// dgesvd of the wide 105 x 4 509 B (bidiagonalisation with one gemv pair per
// column and ~360 bdsqr launches: ~50 ms of the 250^2 POD).
// In: M[i][j] = src[j * lds + i] (column j of M = row j of a row-major
// source).  Out: U (R x R column-major, ld R), sigma (R), info (0, or 1 if
// the sweeps did not converge).
constexpr int kJT = 1024;
constexpr int kJacMaxSweeps = 60;
__global__ __launch_bounds__(kJT) void jacobi_svd_kernel(const double *__restrict__ src, int lds,
                                                         int R, double *__restrict__ u,
                                                         double *__restrict__ sigma,
                                                         int *__restrict__ info)
{
    extern __shared__ double jac_lds[];  // N columns of R (N = R rounded up to even)
    __shared__ int rotated;
    __shared__ double sg[128];
    const int N = R + (R & 1);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = kJT / 64;
    for (int e = threadIdx.x; e < N * R; e += kJT) {
        const int j = e / R, i = e % R;
        jac_lds[e] = j < R ? src[(size_t)j * lds + i] : 0.0;
    }
    const double tol = sqrt((double)R) * 0x1p-52;
    int sweep = 0;
    for (; sweep < kJacMaxSweeps; ++sweep) {
        if (threadIdx.x == 0) rotated = 0;
        __syncthreads();
        for (int st = 0; st < N - 1; ++st) {
            for (int pi = wv; pi < N / 2; pi += nw) {
                const int kp = pi, kq = N - 1 - pi;
                const int p = kp == 0 ? 0 : 1 + (kp - 1 + st) % (N - 1);
                const int q = 1 + (kq - 1 + st) % (N - 1);
                if (p >= R || q >= R) continue;  // the padding column
                double *ap = jac_lds + (size_t)p * R, *aq = jac_lds + (size_t)q * R;
                double x0 = lane < R ? ap[lane] : 0.0, y0 = lane < R ? aq[lane] : 0.0;
                double x1 = lane + 64 < R ? ap[lane + 64] : 0.0;
                double y1 = lane + 64 < R ? aq[lane + 64] : 0.0;
                double a = x0 * x0 + x1 * x1, b = y0 * y0 + y1 * y1, g = x0 * y0 + x1 * y1;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) {
                    a += __shfl_xor(a, o);
                    b += __shfl_xor(b, o);
                    g += __shfl_xor(g, o);
                }
                // the butterfly's lanes may differ in the last bit: take lane 0's
                // sums, so every lane takes the same decision and the same angle
                a = __shfl(a, 0), b = __shfl(b, 0), g = __shfl(g, 0);
                if (!(fabs(g) > tol * sqrt(a * b))) continue;  // wave-uniform
                const double z = (b - a) / (2.0 * g);
                const double t = (z >= 0.0 ? 1.0 : -1.0) / (fabs(z) + sqrt(1.0 + z * z));
                const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
                if (lane < R) {
                    ap[lane] = c * x0 - s * y0;
                    aq[lane] = s * x0 + c * y0;
                }
                if (lane + 64 < R) {
                    ap[lane + 64] = c * x1 - s * y1;
                    aq[lane + 64] = s * x1 + c * y1;
                }
                if (lane == 0) atomicAdd(&rotated, 1);
            }
            __syncthreads();
        }
        if (rotated == 0) break;
        __syncthreads();  // everyone has read `rotated` before it is reset
    }
    // sigma_j = ||a_j||, ranks by decreasing sigma (ties by index)
    for (int j = wv; j < R; j += nw) {
        const double *aj = jac_lds + (size_t)j * R;
        double x0 = lane < R ? aj[lane] : 0.0, x1 = lane + 64 < R ? aj[lane + 64] : 0.0;
        double a = x0 * x0 + x1 * x1;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) a += __shfl_xor(a, o);
        if (lane == 0) sg[j] = sqrt(a);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < R; j += kJT) {
        int rank = 0;
        for (int i = 0; i < R; ++i) rank += sg[i] > sg[j] || (sg[i] == sg[j] && i < j);
        sigma[rank] = sg[j];
        const double inv = sg[j] > 0.0 ? 1.0 / sg[j] : 0.0;
        for (int i = 0; i < R; ++i) u[(size_t)rank * R + i] = jac_lds[(size_t)j * R + i] * inv;
    }
    if (threadIdx.x == 0) *info = sweep < kJacMaxSweeps ? 0 : 1;
}

size_t jacobi_lds_bytes(int R) { return sizeof(double) * (size_t)(R + (R & 1)) * R; }

// out (K x n, row stride ldo) = sum over p < parts of W[p] (K x nc packed):
// groups of parts summed into tmp[g] (gridDim.y = groups), then the groups --
// a fixed order (deterministic), without one thread walking every part
__global__ __launch_bounds__(kPB) void sum_rows_group_kernel(const double *__restrict__ w,
                                                             int parts, int K, int nc, int n,
                                                             double *__restrict__ tmp)
{
    const size_t e = (size_t)blockIdx.x * kPB + threadIdx.x;
    if (e >= (size_t)K * n) return;
    const int G = gridDim.y, g = blockIdx.y;
    const int p0 = (int)((long)parts * g / G), p1 = (int)((long)parts * (g + 1) / G);
    const size_t j = e / n, c = e % n;
    const size_t kn = (size_t)K * nc;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int p = p0;
    for (; p + 3 < p1; p += 4) {
        s0 += w[p * kn + j * nc + c];
        s1 += w[(p + 1) * kn + j * nc + c];
        s2 += w[(p + 2) * kn + j * nc + c];
        s3 += w[(p + 3) * kn + j * nc + c];
    }
    for (; p < p1; ++p) s0 += w[p * kn + j * nc + c];
    tmp[(size_t)g * K * n + e] = (s0 + s1) + (s2 + s3);
}

// workgroups per CU of the tall-skinny products (BURG_POD_GEMM_OCC = 1 or 2)
int ts_occ()
{
    const char *e = std::getenv("BURG_POD_GEMM_OCC");  // read per launch (tests switch it)
    return e && std::atoi(e) == 1 ? 1 : 2;
}

template <void (*K1)(TsArgs), void (*K2)(TsArgs)>
void launch_ts(int occ, dim3 grid, hipStream_t st, const TsArgs &g)
{
    if (occ == 2)
        hipLaunchKernelGGL(K2, grid, dim3(kTW), 0, st, g);
    else
        hipLaunchKernelGGL(K1, grid, dim3(kTW), 0, st, g);
}

// C (m x n, ldc) = A (m x K, lda) B (K x n, ldb), all row-major, n <= 128
int ts_gemm_nn(hipStream_t st, const double *a, size_t lda, size_t m, int K, const double *b,
               size_t ldb, int n, double *c, size_t ldc)
{
    TsArgs g{a, b, c, lda, ldb, ldc, m, K, n, 0, 0};
    const dim3 grid((unsigned)((m + 127) / 128));
    const int occ = ts_occ();
    switch ((n + 15) / 16) {
    case 1: launch_ts<gemm_nn_kernel<1, 1>, gemm_nn_kernel<1, 2>>(occ, grid, st, g); break;
    case 2: launch_ts<gemm_nn_kernel<2, 1>, gemm_nn_kernel<2, 2>>(occ, grid, st, g); break;
    case 3: launch_ts<gemm_nn_kernel<3, 1>, gemm_nn_kernel<3, 2>>(occ, grid, st, g); break;
    case 4: launch_ts<gemm_nn_kernel<4, 1>, gemm_nn_kernel<4, 2>>(occ, grid, st, g); break;
    case 5: launch_ts<gemm_nn_kernel<5, 1>, gemm_nn_kernel<5, 2>>(occ, grid, st, g); break;
    case 6: launch_ts<gemm_nn_kernel<6, 1>, gemm_nn_kernel<6, 2>>(occ, grid, st, g); break;
    case 7: launch_ts<gemm_nn_kernel<7, 1>, gemm_nn_kernel<7, 2>>(occ, grid, st, g); break;
    case 8: launch_ts<gemm_nn_kernel<8, 1>, gemm_nn_kernel<8, 2>>(occ, grid, st, g); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// row parts of a tn product: a multiple of 8 (one set per XCD), ~4 000
// workgroups over the launch (~8 rounds at two per CU; at 250^2 x 9 mu: 112
// parts -- 68.8 ms per POD against 71.8-73.7 with 64 and 71.9 with 56,
// profiles/r04/pod/parts_ab.txt), >= 128 rows each, <= 512
int ts_tn_parts(size_t m, int K)
{
    const int jt = (K + 127) / 128;
    long p = 8L * ((4032 + 8L * jt - 1) / (8L * jt));
    if (const char *e = std::getenv("BURG_POD_TN_PARTS")) p = std::max(8L, 8L * (std::atol(e) / 8));
    while (p > 8 && (long)(m / (size_t)p) < 128) p -= 8;
    return (int)std::min(p, 512L);
}

// groups of parts in the first reduction pass: ~16 parts each
int ts_tn_groups(int parts) { return std::max(1, parts / 16); }

// out (K x n, ldo) = A^T B for A (m x K, lda) and B (m x n, ldb) row-major,
// n <= 128; work: ts_tn_work(m, K, n) doubles
int ts_gemm_tn(hipStream_t st, const double *a, size_t lda, size_t m, int K, const double *b,
               size_t ldb, int n, double *out, int ldo, double *work)
{
    const int NB = (n + 15) / 16;
    if (NB < 1 || NB > 8) return -1;
    const int parts = ts_tn_parts(m, K), jt = (K + 127) / 128;
    TsArgs g{a, b, work, lda, ldb, 0, m, K, n, jt, (m + parts - 1) / parts};
    const dim3 grid((unsigned)(parts * jt));
    const int occ = ts_occ();
    switch (NB) {
    case 1: launch_ts<gemm_tn_kernel<1, 1>, gemm_tn_kernel<1, 2>>(occ, grid, st, g); break;
    case 2: launch_ts<gemm_tn_kernel<2, 1>, gemm_tn_kernel<2, 2>>(occ, grid, st, g); break;
    case 3: launch_ts<gemm_tn_kernel<3, 1>, gemm_tn_kernel<3, 2>>(occ, grid, st, g); break;
    case 4: launch_ts<gemm_tn_kernel<4, 1>, gemm_tn_kernel<4, 2>>(occ, grid, st, g); break;
    case 5: launch_ts<gemm_tn_kernel<5, 1>, gemm_tn_kernel<5, 2>>(occ, grid, st, g); break;
    case 6: launch_ts<gemm_tn_kernel<6, 1>, gemm_tn_kernel<6, 2>>(occ, grid, st, g); break;
    case 7: launch_ts<gemm_tn_kernel<7, 1>, gemm_tn_kernel<7, 2>>(occ, grid, st, g); break;
    default: launch_ts<gemm_tn_kernel<8, 1>, gemm_tn_kernel<8, 2>>(occ, grid, st, g); break;
    }
    const int G = ts_tn_groups(parts);
    double *tmp = work + (size_t)parts * K * 16 * NB;
    hipLaunchKernelGGL(sum_rows_group_kernel, dim3(blocks((size_t)K * n), G), dim3(kPB), 0, st,
                       (const double *)work, parts, K, 16 * NB, n, tmp);
    hipLaunchKernelGGL(sum_rows_kernel, dim3(blocks((size_t)K * n)), dim3(kPB), 0, st,
                       (const double *)tmp, G, K, n, n, out, ldo);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

size_t ts_tn_work(size_t m, int K, int n)
{
    const int parts = ts_tn_parts(m, K);
    return (size_t)parts * K * 16 * ((n + 15) / 16) + (size_t)ts_tn_groups(parts) * K * n;
}

// dst (rows x ldd, row-major, columns >= cols zero) <- src (rows x cols column-major, lds)
__global__ __launch_bounds__(kPB) void cm_to_rm_pad_kernel(const double *__restrict__ src,
                                                           size_t lds, size_t rows, int cols,
                                                           double *__restrict__ dst, int ldd)
{
    const size_t e = (size_t)blockIdx.x * kPB + threadIdx.x;
    if (e >= rows * ldd) return;
    const size_t r = e / ldd;
    const int c = (int)(e % ldd);
    dst[e] = c < cols ? src[(size_t)c * lds + r] : 0.0;
}

// svd_flip on a row-major (m x k) U: per column the sign of its first
// largest-|.| entry; pass 1 per row chunk (thread = column), pass 2 over the
// chunks in order, pass 3 scales.
constexpr int kFlipRows = 1024;
__global__ __launch_bounds__(128) void rm_colmax_kernel(const double *__restrict__ u, size_t m,
                                                        int k, double *__restrict__ part)
{
    const int c = threadIdx.x;
    if (c >= k) return;
    const size_t r0 = (size_t)blockIdx.x * kFlipRows, r1 = std::min(m, r0 + kFlipRows);
    double best = -1.0, val = 0.0;
    for (size_t r = r0; r < r1; ++r) {
        const double v = u[r * k + c];
        if (fabs(v) > best) best = fabs(v), val = v;
    }
    part[((size_t)blockIdx.x * k + c) * 2] = best;
    part[((size_t)blockIdx.x * k + c) * 2 + 1] = val;
}

__global__ __launch_bounds__(128) void rm_colsign_kernel(const double *__restrict__ part,
                                                         int nparts, int k,
                                                         double *__restrict__ sgn)
{
    const int c = threadIdx.x;
    if (c >= k) return;
    double best = -1.0, val = 0.0;
    for (int p = 0; p < nparts; ++p) {
        const double b = part[((size_t)p * k + c) * 2];
        if (b > best) best = b, val = part[((size_t)p * k + c) * 2 + 1];
    }
    sgn[c] = val < 0.0 ? -1.0 : 1.0;
}

__global__ __launch_bounds__(kPB) void rm_colscale_kernel(double *__restrict__ u, size_t m, int k,
                                                          const double *__restrict__ sgn)
{
    const size_t e = (size_t)blockIdx.x * kPB + threadIdx.x;
    if (e >= m * k) return;
    u[e] *= sgn[e % k];
}

// U_B[:, :k] (R x R column-major, ld R) -> row-major (Rp x k), rows >= R zero
__global__ __launch_bounds__(kPB) void ub_rows_kernel(const double *__restrict__ ub, int R, int k,
                                                      int Rp, double *__restrict__ out)
{
    const size_t e = (size_t)blockIdx.x * kPB + threadIdx.x;
    if (e >= (size_t)Rp * k) return;
    const int r = (int)(e / k), c = (int)(e % k);
    out[e] = r < R ? ub[(size_t)c * R + r] : 0.0;
}

// Orthonormal basis of the columns of a row-major Y (rows x R, row stride
// Rp) in place: the shifted CholeskyQR3 of orth_columns with the Gram on
// gemm_tn_kernel and Y <- Y R^-1 as the transposed left solve on the
// column-major view Y^T (R x rows, ld Rp).  Householder fallback through a
// column-major copy (tmp: rows x Rp, allocated on demand).
rocblas_status orth_rows(rocblas_handle h, hipStream_t st, size_t rows, int R, int Rp, double *y,
                         double *g, double *tau, rocblas_int *info, double *work, double **tmp,
                         bool *householder)
{
    const double one = 1.0;
    const double u = 0x1p-53;
    const double c = 11.0 * ((double)rows * R + (double)R * (R + 1)) * u;
    rocblas_status s;
    *householder = false;
    for (int pass = 0; pass < 3; ++pass) {
        if (ts_gemm_tn(st, y, Rp, rows, Rp, y, Rp, Rp, g, Rp, work))
            return rocblas_status_internal_error;
        if (pass == 0)
            hipLaunchKernelGGL(shift_diag_kernel, dim3(1), dim3(kPB), 0, st, g, R, c, Rp);
        if ((s = rocsolver_dpotrf(h, rocblas_fill_upper, R, g, Rp, info)) != rocblas_status_success)
            return s;
        rocblas_int hinfo = 0;
        if (hipMemcpyAsync(&hinfo, info, sizeof hinfo, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return rocblas_status_internal_error;
        if (hinfo != 0) {  // Y is left as the last successful pass made it: same span
            *householder = true;
            if (!*tmp && hipMalloc(tmp, sizeof(double) * rows * Rp) != hipSuccess)
                return rocblas_status_memory_error;
            // row-major (rows x Rp) -> column-major (rows x Rp), QR, and back
            if (launch_basis_transpose(y, *tmp, rows, Rp, st)) return rocblas_status_internal_error;
            if ((s = rocsolver_dgeqrf(h, (rocblas_int)rows, R, *tmp, (rocblas_int)rows, tau)) !=
                    rocblas_status_success ||
                (s = rocsolver_dorgqr(h, (rocblas_int)rows, R, R, *tmp, (rocblas_int)rows, tau)) !=
                    rocblas_status_success)
                return s;
            if (launch_basis_transpose(*tmp, y, (size_t)Rp, (int)rows, st))
                return rocblas_status_internal_error;
            return rocblas_status_success;
        }
        if ((s = rocblas_dtrsm(h, rocblas_side_left, rocblas_fill_upper, rocblas_operation_transpose,
                               rocblas_diagonal_non_unit, R, (rocblas_int)rows, &one, g, Rp, y,
                               Rp)) != rocblas_status_success)
            return s;
    }
    return rocblas_status_success;
}

}  // namespace

int pod_rsvd_mfma(hipStream_t st, size_t m, int ns, const double *d_s, int k, int nrand,
                  int n_iter, const double *d_omega, double *d_u, double *d_sigma, char *msg,
                  size_t msglen);

int pod_device(hipStream_t st, size_t m, int ns, const double *d_s, int k, double *d_u,
               double *d_sigma, char *msg, size_t msglen)
{
    // d_s: C-order (m x ns) snapshots on the device; d_u: C-order (m x k) out
    auto err = [&](const char *what, int code) {
        snprintf(msg, msglen, "%s failed (%d)", what, code);
        return -3;
    };
    if (m < (size_t)ns) {
        snprintf(msg, msglen, "POD needs at least as many rows as snapshots (m=%zu < ns=%d)", m, ns);
        return -1;
    }
    if (m > 0x7fffffffULL) {
        snprintf(msg, msglen, "m=%zu exceeds rocSOLVER's 32-bit sizes", m);
        return -1;
    }
    double *a = nullptr, *tau = nullptr, *r = nullptr, *ur = nullptr, *e = nullptr, *c = nullptr,
           *sgn = nullptr, *sv = nullptr;
    rocblas_int *info = nullptr;
    rocblas_handle h = nullptr;
    int rc = 0;
    auto cleanup = [&]() {
        (void)hipStreamSynchronize(st);
        if (h) rocblas_destroy_handle(h);
        for (double *p : {a, tau, r, ur, e, c, sgn, sv})
            if (p) (void)hipFree(p);
        if (info) (void)hipFree(info);
    };
    const size_t nsz = (size_t)ns;
    if (hipMalloc(&a, sizeof(double) * m * nsz) != hipSuccess ||
        hipMalloc(&tau, sizeof(double) * nsz) != hipSuccess ||
        hipMalloc(&r, sizeof(double) * nsz * nsz) != hipSuccess ||
        hipMalloc(&ur, sizeof(double) * nsz * nsz) != hipSuccess ||
        hipMalloc(&e, sizeof(double) * nsz) != hipSuccess ||
        hipMalloc(&sv, sizeof(double) * nsz) != hipSuccess ||
        hipMalloc(&c, sizeof(double) * m * k) != hipSuccess ||
        hipMalloc(&sgn, sizeof(double) * k) != hipSuccess ||
        hipMalloc(&info, sizeof(rocblas_int)) != hipSuccess) {
        cleanup();
        snprintf(msg, msglen, "POD: hipMalloc of %zu MB failed",
                 (size_t)((sizeof(double) * (m * nsz + m * k + 2 * nsz * nsz)) >> 20));
        return -5;
    }
    if (rocblas_create_handle(&h) != rocblas_status_success) {
        cleanup();
        return err("rocblas_create_handle", 0);
    }
    rocblas_set_stream(h, st);
    // column-major (m x ns) copy of the snapshots
    if ((rc = launch_basis_transpose(d_s, a, m, ns, st))) {
        cleanup();
        return err("transpose", rc);
    }
    rocblas_status s;
    if ((s = rocsolver_dgeqrf(h, (rocblas_int)m, ns, a, (rocblas_int)m, tau)) !=
        rocblas_status_success) {
        cleanup();
        return err("rocsolver_dgeqrf", (int)s);
    }
    hipLaunchKernelGGL(triu_copy_kernel, dim3(blocks(nsz * nsz)), dim3(kPB), 0, st, a, m, ns, r);
    if ((s = rocsolver_dgesvd(h, rocblas_svect_singular, rocblas_svect_none, ns, ns, r, ns, sv, ur,
                              ns, nullptr, 1, e, rocblas_outofplace, info)) !=
        rocblas_status_success) {
        cleanup();
        return err("rocsolver_dgesvd", (int)s);
    }
    hipLaunchKernelGGL(embed_kernel, dim3(blocks(m * k)), dim3(kPB), 0, st, ur, ns, k, m, c);
    if ((s = rocsolver_dormqr(h, rocblas_side_left, rocblas_operation_none, (rocblas_int)m, k, ns,
                              a, (rocblas_int)m, tau, c, (rocblas_int)m)) !=
        rocblas_status_success) {
        cleanup();
        return err("rocsolver_dormqr", (int)s);
    }
    hipLaunchKernelGGL(col_sign_kernel, dim3(k), dim3(kPB), 0, st, c, m, sgn);
    hipLaunchKernelGGL(col_scale_kernel, dim3(blocks(m * k)), dim3(kPB), 0, st, c, m, k,
                       (const double *)sgn);
    // column-major (m x k) = C-order (k x m) -> C-order (m x k)
    if ((rc = launch_basis_transpose(c, d_u, (size_t)k, (int)m, st))) {
        cleanup();
        return err("transpose back", rc);
    }
    (void)hipMemcpyAsync(d_sigma, sv, sizeof(double) * k, hipMemcpyDeviceToDevice, st);
    rocblas_int hinfo = 0;
    (void)hipMemcpyAsync(&hinfo, info, sizeof hinfo, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) {
        cleanup();
        return err("POD stream", 0);
    }
    cleanup();
    if (hinfo != 0) {
        snprintf(msg, msglen, "rocsolver_dgesvd did not converge (info=%d)", (int)hinfo);
        return -6;
    }
    return 0;
}

// Randomized truncated SVD (the algorithm of sklearn's randomized_svd, which
// the reference's POD(method='rsvd') calls, C/hypernet2D.py:2688-2692):
// Y = S Omega, n_iter power iterations Y <- orth(S orth(S^T Y)), Q = orth(Y),
// B = Q^T S, B = U_B Sigma V^T, U = Q U_B[:, :k].  Orthonormalisation by
// shifted CholeskyQR3 (orth_columns; Householder QR as its fallback;
// sklearn's 'auto' normaliser is LU, which spans the same subspace).
// nrand <= 128 goes to pod_rsvd_mfma (our products, below); here, for wider
// sketches or BURG_POD_GEMM=rocblas, every product is a rocBLAS dgemm and
// the small SVD rocSOLVER's dgesvd.
// omega: (ns x nrand) column-major (host), k <= nrand <= ns.
int pod_rsvd_device(hipStream_t st, size_t m, int ns, const double *d_s, int k, int nrand,
                    int n_iter, const double *d_omega, double *d_u, double *d_sigma, char *msg,
                    size_t msglen)
{
    auto err = [&](const char *what, int code) {
        snprintf(msg, msglen, "%s failed (%d)", what, code);
        return -3;
    };
    if (m < (size_t)ns || m > 0x7fffffffULL || nrand < k || nrand > ns) {
        snprintf(msg, msglen, "rsvd: need ns <= m < 2^31 and k <= nrand <= ns");
        return -1;
    }
    const char *gemm = std::getenv("BURG_POD_GEMM");  // "rocblas": the library products below
    if (nrand <= 128 && !(gemm && std::strcmp(gemm, "rocblas") == 0))
        return pod_rsvd_mfma(st, m, ns, d_s, k, nrand, n_iter, d_omega, d_u, d_sigma, msg, msglen);
    const rocblas_int M = (rocblas_int)m, NS = ns, R = nrand;
    double *a = nullptr, *y = nullptr, *z = nullptr, *tau = nullptr, *b = nullptr, *ub = nullptr,
           *sv = nullptr, *e = nullptr, *c = nullptr, *sgn = nullptr, *g = nullptr,
           *work = nullptr;
    rocblas_int *info = nullptr;
    rocblas_handle h = nullptr;
    auto cleanup = [&]() {
        (void)hipStreamSynchronize(st);
        if (h) rocblas_destroy_handle(h);
        for (double *p : {a, y, z, tau, b, ub, sv, e, c, sgn, g, work})
            if (p) (void)hipFree(p);
        if (info) (void)hipFree(info);
    };
    const size_t nsz = (size_t)ns;
    // split-K partials of the tall products (gemm_tn_splitk): Y^T Y / Z^T Z,
    // S^T Q, Q^T S
    const size_t work_doubles = std::max(
        {(size_t)(splitk_parts(R, R, M) + 1) * R * R, (size_t)(splitk_parts(NS, R, M) + 1) * nsz * R,
         (size_t)(splitk_parts(R, NS, M) + 1) * nsz * R});
    if (hipMalloc(&a, sizeof(double) * m * nsz) != hipSuccess ||
        hipMalloc(&y, sizeof(double) * m * R) != hipSuccess ||
        hipMalloc(&z, sizeof(double) * nsz * R) != hipSuccess ||
        hipMalloc(&tau, sizeof(double) * R) != hipSuccess ||
        hipMalloc(&b, sizeof(double) * (size_t)R * nsz) != hipSuccess ||
        hipMalloc(&ub, sizeof(double) * (size_t)R * R) != hipSuccess ||
        hipMalloc(&sv, sizeof(double) * R) != hipSuccess ||
        hipMalloc(&e, sizeof(double) * R) != hipSuccess ||
        hipMalloc(&c, sizeof(double) * m * k) != hipSuccess ||
        hipMalloc(&sgn, sizeof(double) * k) != hipSuccess ||
        hipMalloc(&g, sizeof(double) * (size_t)R * R) != hipSuccess ||
        hipMalloc(&work, sizeof(double) * work_doubles) != hipSuccess ||
        hipMalloc(&info, sizeof(rocblas_int)) != hipSuccess) {
        cleanup();
        snprintf(msg, msglen, "rsvd: hipMalloc failed");
        return -5;
    }
    if (rocblas_create_handle(&h) != rocblas_status_success) {
        cleanup();
        return err("rocblas_create_handle", 0);
    }
    rocblas_set_stream(h, st);
    int rc = 0;
    if ((rc = launch_basis_transpose(d_s, a, m, ns, st))) {
        cleanup();
        return err("transpose", rc);
    }
    const double one = 1.0, zero = 0.0;
    rocblas_status s;
#define RS(call, what)                 \
    if ((s = (call)) != rocblas_status_success) { \
        cleanup();                     \
        return err(what, (int)s);      \
    }
    // Y = S Omega
    RS(rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, M, R, NS, &one, a, M,
                     d_omega, NS, &zero, y, M), "dgemm S.Omega");
    bool hh = false;
    int n_householder = 0;
    for (int it = 0; it < n_iter; ++it) {
        RS(orth_columns(h, st, M, R, y, g, tau, info, work, &hh), "orth Y");
        n_householder += hh;
        RS(gemm_tn_splitk(h, st, NS, R, M, a, M, y, M, z, NS, work, splitk_parts(NS, R, M)),
           "dgemm S^T.Q");
        RS(orth_columns(h, st, NS, R, z, g, tau, info, work, &hh), "orth Z");
        n_householder += hh;
        RS(rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, M, R, NS, &one, a, M,
                         z, NS, &zero, y, M), "dgemm S.Z");
    }
    RS(orth_columns(h, st, M, R, y, g, tau, info, work, &hh), "orth Q");
    n_householder += hh;
    if (std::getenv("BURG_POD_DEBUG"))  // diagnostics
        fprintf(stderr, "[pod] rsvd: %d of %d orthonormalisations fell back to Householder\n",
                n_householder, 2 * n_iter + 1);
    // B = Q^T S (R x ns), its SVD, U = Q U_B[:, :k]
    RS(gemm_tn_splitk(h, st, R, NS, M, y, M, a, M, b, R, work, splitk_parts(R, NS, M)),
       "dgemm Q^T.S");
    RS(rocsolver_dgesvd(h, rocblas_svect_singular, rocblas_svect_none, R, NS, b, R, sv, ub, R,
                        nullptr, 1, e, rocblas_outofplace, info), "dgesvd B");
    RS(rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, M, k, R, &one, y, M, ub, R,
                     &zero, c, M), "dgemm Q.U_B");
#undef RS
    hipLaunchKernelGGL(col_sign_kernel, dim3(k), dim3(kPB), 0, st, c, m, sgn);
    hipLaunchKernelGGL(col_scale_kernel, dim3(blocks(m * k)), dim3(kPB), 0, st, c, m, k,
                       (const double *)sgn);
    if ((rc = launch_basis_transpose(c, d_u, (size_t)k, (int)m, st))) {
        cleanup();
        return err("transpose back", rc);
    }
    (void)hipMemcpyAsync(d_sigma, sv, sizeof(double) * k, hipMemcpyDeviceToDevice, st);
    rocblas_int hinfo = 0;
    (void)hipMemcpyAsync(&hinfo, info, sizeof hinfo, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) {
        cleanup();
        return err("rsvd stream", 0);
    }
    cleanup();
    if (hinfo != 0) {
        snprintf(msg, msglen, "rocsolver_dgesvd did not converge (info=%d)", (int)hinfo);
        return -6;
    }
    return 0;
}

// The randomized SVD of pod_rsvd_device on the tall-skinny MFMA products
// (gemm_nn_kernel / gemm_tn_kernel): the same algorithm and the same
// CholeskyQR3 normaliser, with S read in place (C-order, no transposed copy)
// and every thin matrix row-major with Rp = 16 ceil(nrand / 16) columns (the
// padding columns are zero throughout):
//   Y = S Omega; n_iter x { Y = orth(Y); Z = orth(S^T Y); Y = S Z };
//   Q = orth(Y); B^T = S^T Q (ns x Rp row-major = B, R x ns column-major,
//   ld Rp); B = U_B Sigma V^T (rocSOLVER dgesvd); U = Q U_B[:, :k], written
//   straight into the C-order (m x k) result.
// nrand <= 128.
int pod_rsvd_mfma(hipStream_t st, size_t m, int ns, const double *d_s, int k, int nrand,
                  int n_iter, const double *d_omega, double *d_u, double *d_sigma, char *msg,
                  size_t msglen)
{
    auto err = [&](const char *what, int code) {
        snprintf(msg, msglen, "%s failed (%d)", what, code);
        return -3;
    };
    if (m < (size_t)ns || m > 0x7fffffffULL || nrand < k || nrand > ns || nrand > 128) {
        snprintf(msg, msglen, "rsvd: need ns <= m < 2^31 and k <= nrand <= min(ns, 128)");
        return -1;
    }
    const int R = nrand, Rp = 16 * ((R + 15) / 16);
    const size_t nsz = (size_t)ns;
    const size_t nflip = (m + kFlipRows - 1) / kFlipRows;
    const size_t work_doubles =
        std::max({ts_tn_work(m, ns, Rp), ts_tn_work(m, Rp, Rp), ts_tn_work(nsz, Rp, Rp),
                  2 * nflip * (size_t)k});
    double *y = nullptr, *z = nullptr, *om = nullptr, *tau = nullptr, *b = nullptr, *ub = nullptr,
           *ubk = nullptr, *sv = nullptr, *e = nullptr, *sgn = nullptr, *g = nullptr,
           *work = nullptr, *tmp = nullptr;
    rocblas_int *info = nullptr;
    rocblas_handle h = nullptr;
    auto cleanup = [&]() {
        (void)hipStreamSynchronize(st);
        if (h) rocblas_destroy_handle(h);
        for (double *p : {y, z, om, tau, b, ub, ubk, sv, e, sgn, g, work, tmp})
            if (p) (void)hipFree(p);
        if (info) (void)hipFree(info);
    };
    if (hipMalloc(&y, sizeof(double) * m * Rp) != hipSuccess ||
        hipMalloc(&z, sizeof(double) * nsz * Rp) != hipSuccess ||
        hipMalloc(&om, sizeof(double) * nsz * Rp) != hipSuccess ||
        hipMalloc(&tau, sizeof(double) * Rp) != hipSuccess ||
        hipMalloc(&b, sizeof(double) * nsz * Rp) != hipSuccess ||
        hipMalloc(&ub, sizeof(double) * (size_t)R * R) != hipSuccess ||
        hipMalloc(&ubk, sizeof(double) * (size_t)Rp * k) != hipSuccess ||
        hipMalloc(&sv, sizeof(double) * Rp) != hipSuccess ||
        hipMalloc(&e, sizeof(double) * Rp) != hipSuccess ||
        hipMalloc(&sgn, sizeof(double) * k) != hipSuccess ||
        hipMalloc(&g, sizeof(double) * (size_t)Rp * Rp) != hipSuccess ||
        hipMalloc(&work, sizeof(double) * work_doubles) != hipSuccess ||
        hipMalloc(&info, sizeof(rocblas_int)) != hipSuccess) {
        cleanup();
        snprintf(msg, msglen, "rsvd: hipMalloc failed");
        return -5;
    }
    if (rocblas_create_handle(&h) != rocblas_status_success) {
        cleanup();
        return err("rocblas_create_handle", 0);
    }
    rocblas_set_stream(h, st);
    rocblas_status s;
    bool hh = false;
    int n_householder = 0;
#define TS(call, what)                  \
    if ((call) != 0) {                  \
        cleanup();                      \
        return err(what, 0);            \
    }
#define RS(call, what)                                \
    if ((s = (call)) != rocblas_status_success) {     \
        cleanup();                                    \
        return err(what, (int)s);                     \
    }
    // Omega (ns x R column-major) -> row-major (ns x Rp)
    hipLaunchKernelGGL(cm_to_rm_pad_kernel, dim3(blocks(nsz * Rp)), dim3(kPB), 0, st, d_omega, nsz,
                       nsz, R, om, Rp);
    TS(ts_gemm_nn(st, d_s, nsz, m, ns, om, Rp, Rp, y, Rp), "S.Omega");
    for (int it = 0; it < n_iter; ++it) {
        RS(orth_rows(h, st, m, R, Rp, y, g, tau, info, work, &tmp, &hh), "orth Y");
        n_householder += hh;
        TS(ts_gemm_tn(st, d_s, nsz, m, ns, y, Rp, Rp, z, Rp, work), "S^T.Q");
        RS(orth_rows(h, st, nsz, R, Rp, z, g, tau, info, work, &tmp, &hh), "orth Z");
        n_householder += hh;
        TS(ts_gemm_nn(st, d_s, nsz, m, ns, z, Rp, Rp, y, Rp), "S.Z");
    }
    RS(orth_rows(h, st, m, R, Rp, y, g, tau, info, work, &tmp, &hh), "orth Q");
    n_householder += hh;
    if (std::getenv("BURG_POD_DEBUG"))
        fprintf(stderr, "[pod] rsvd (mfma): %d of %d orthonormalisations fell back to Householder\n",
                n_householder, 2 * n_iter + 1);
    // B^T = S^T Q (ns x Rp row-major) = B (R x ns column-major, ld Rp)
    TS(ts_gemm_tn(st, d_s, nsz, m, ns, y, Rp, Rp, b, Rp, work), "S^T.Q (B)");
    const char *ssvd = std::getenv("BURG_POD_SMALL_SVD");  // "rocsolver": dgesvd of B itself
    if (ssvd && std::strcmp(ssvd, "rocsolver") == 0) {
        RS(rocsolver_dgesvd(h, rocblas_svect_singular, rocblas_svect_none, R, ns, b, Rp, sv, ub, R,
                            nullptr, 1, e, rocblas_outofplace, info), "dgesvd B");
    } else {
        // B^T = Q_b R_b (CholeskyQR3 on a copy, R_b = Q_b^T B^T), so B = R_b^T Q_b^T and
        // U_B, sigma are the left singular vectors and values of R_b^T (Jacobi, one workgroup)
        if (hipMemcpyAsync(z, b, sizeof(double) * nsz * Rp, hipMemcpyDeviceToDevice, st) !=
            hipSuccess) {
            cleanup();
            return err("copy B", 0);
        }
        RS(orth_rows(h, st, nsz, R, Rp, z, g, tau, info, work, &tmp, &hh), "orth B^T");
        n_householder += hh;
        TS(ts_gemm_tn(st, z, Rp, nsz, Rp, b, Rp, Rp, g, Rp, work), "Q_b^T.B^T");
        // (set on every call: the attribute is per device, and a
        // function-local "done" flag is neither per device nor thread-safe)
        if (hipFuncSetAttribute((const void *)jacobi_svd_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)jacobi_lds_bytes(128)) != hipSuccess) {
            cleanup();
            return err("jacobi LDS", 0);
        }
        hipLaunchKernelGGL(jacobi_svd_kernel, dim3(1), dim3(kJT), jacobi_lds_bytes(R), st,
                           (const double *)g, Rp, R, ub, sv, (int *)info);
        TS(hipGetLastError() != hipSuccess, "jacobi svd");
    }
    // U = Q U_B[:, :k]: U_B (R x R column-major) -> row-major (Rp x k), rows >= R zero
    hipLaunchKernelGGL(ub_rows_kernel, dim3(blocks((size_t)Rp * k)), dim3(kPB), 0, st,
                       (const double *)ub, R, k, Rp, ubk);
    TS(ts_gemm_nn(st, y, Rp, m, Rp, ubk, k, k, d_u, k), "Q.U_B");
    hipLaunchKernelGGL(rm_colmax_kernel, dim3((unsigned)nflip), dim3(128), 0, st,
                       (const double *)d_u, m, k, work);
    hipLaunchKernelGGL(rm_colsign_kernel, dim3(1), dim3(128), 0, st, (const double *)work,
                       (int)nflip, k, sgn);
    hipLaunchKernelGGL(rm_colscale_kernel, dim3(blocks(m * k)), dim3(kPB), 0, st, d_u, m, k,
                       (const double *)sgn);
#undef TS
#undef RS
    (void)hipMemcpyAsync(d_sigma, sv, sizeof(double) * k, hipMemcpyDeviceToDevice, st);
    rocblas_int hinfo = 0;
    (void)hipMemcpyAsync(&hinfo, info, sizeof hinfo, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) {
        cleanup();
        return err("rsvd stream", 0);
    }
    cleanup();
    if (hinfo != 0) {
        if (ssvd && std::strcmp(ssvd, "rocsolver") == 0)
            snprintf(msg, msglen, "rocsolver_dgesvd did not converge (info=%d)", (int)hinfo);
        else
            snprintf(msg, msglen, "one-sided Jacobi SVD of the %d x %d sketch did not converge "
                     "within its sweep cap (info=%d)", R, R, (int)hinfo);
        return -6;
    }
    return 0;
}

}  // namespace burg
