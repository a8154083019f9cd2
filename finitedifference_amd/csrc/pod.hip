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
__global__ __launch_bounds__(kPB) void shift_diag_kernel(double *__restrict__ g, int r, double c)
{
    __shared__ double part[kPB];
    double t = 0.0;
    for (int i = threadIdx.x; i < r; i += kPB) t += g[(size_t)i * r + i];
    part[threadIdx.x] = t;
    __syncthreads();
    for (int h = kPB / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) part[threadIdx.x] += part[threadIdx.x + h];
        __syncthreads();
    }
    const double shift = c * part[0];
    for (int i = threadIdx.x; i < r; i += kPB) g[(size_t)i * r + i] += shift;
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
        if (pass == 0) hipLaunchKernelGGL(shift_diag_kernel, dim3(1), dim3(kPB), 0, st, g, (int)r, c);
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

}  // namespace

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
// sklearn's 'auto' normaliser is LU, which spans the same subspace).  Every
// product is a rocBLAS dgemm on the device.
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

}  // namespace burg
