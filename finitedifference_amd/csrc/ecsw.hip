// ecsw.hip -- ECSW hyper-reduction training matrix on the GPU (SURVEY.md
// section 8(f), row 2): compute_ECSW_training_matrix_2D, C/hypernet2D.py:2719-2740.
//
// Per snapshot (state w, previous state wp) and node i:
//   R      = residual(w; wp)                    (res2D_alt op order, :2512-2570)
//   W[:,k] = J(w) basis[:,k], k < npod           (exact_jac2D action, :2627-2656)
//   C[isnap*npod + k, i] = R_u[i] W_u[i,k] + R_v[i] W_v[i,k]        (:2737-2738)
// The reference assembles J as a CSR matrix, multiplies it into the basis and
// fills C in a Python loop over nodes; here one kernel does all of it, the
// basis read once per snapshot in a (npod, 2n) layout so every basis column
// is a coalesced plane, the C block written as npod coalesced planes.
// Op order per cell is that of stencil.hip / oracle/burgers_oracle.c
// (-ffp-contract=off): the product equals the oracle's restatement bit for bit.
#include "burg_internal.h"

namespace burg {
namespace {

constexpr int kEB = 256;

// (2n x npod) C-order basis -> (npod x 2n): 32 x 32 tiles through LDS
__global__ __launch_bounds__(256) void basis_transpose_kernel(const double *__restrict__ b,
                                                              double *__restrict__ bt, size_t m,
                                                              int npod)
{
    __shared__ double tile[32][33];
    const size_t i0 = (size_t)blockIdx.x * 32;
    const int k0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int r = ty; r < 32; r += 8) {
        const size_t i = i0 + r;
        const int k = k0 + tx;
        tile[r][tx] = (i < m && k < npod) ? b[i * npod + k] : 0.0;
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
        const int k = k0 + r;
        const size_t i = i0 + tx;
        if (k < npod && i < m) bt[(size_t)k * m + i] = tile[tx][r];
    }
}

// lane i <- lane i-1 (wave shift); lane 0 keeps `old0`
__device__ __forceinline__ double shr1(double old0, double x)
{
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old0), __double2loint(x), 0x138,
                                               0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old0), __double2hiint(x), 0x138,
                                               0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

// A workgroup: 256 columns x kER rows x one group of basis vectors
// (blockIdx.z; k = z, z + gridDim.z, ...).  The node's state, residual and
// neighbour states are computed once into registers; then per basis vector
// each cell loads only its own (xu, xv): the south pair is the previous
// row's (carried), the west pair the left lane's (DPP; lane 0 loads it).
constexpr int kER = 4;

__global__ __launch_bounds__(kEB) void ecsw_kernel(Coeffs cf, const double *__restrict__ w,
                                                   const double *__restrict__ wp,
                                                   const double *__restrict__ bt, int npod,
                                                   double *__restrict__ cblk)
{
    const int nx = cf.nx, ny = cf.ny;
    const size_t n = (size_t)nx * ny;
    const int c = blockIdx.x * kEB + threadIdx.x;
    const int r0 = blockIdx.y * kER;
    const int nr = min(kER, ny - r0);
    const bool colok = c < nx;
    const int cc = colok ? c : nx - 1;  // padding lanes mirror a real column, store nothing
    const bool lane0 = (threadIdx.x & (kWave - 1)) == 0;
    const bool west = c > 0;
    const double a = cf.alpha;
    const double ax = a * cf.inv_dx[cc];
    const double axw = west ? a * cf.inv_dx[cc - 1] : 0.0;
    const double *u = w, *v = w + n, *up = wp, *vp = wp + n;

    double U[kER], V[kER], UW[kER], VW[kER], US[kER], VS[kER], RU[kER], RV[kER], AY[kER],
        AYS[kER];
#pragma unroll
    for (int rr = 0; rr < kER; ++rr) {
        if (rr >= nr) break;
        const int r = r0 + rr;
        const size_t i = (size_t)r * nx + cc;
        const bool south = r > 0;
        const size_t iw = west ? i - 1 : i, is = south ? i - nx : i;
        const double ui = u[i], vi = v[i];
        const double uW = u[iw], vW = v[iw], uS = u[is], vS = v[is];
        const double ay = a * cf.inv_dy[r];
        const double ays = south ? a * cf.inv_dy[r - 1] : 0.0;
        // residual (stencil.hip residual_kernel / orc_residual op order)
        const double upi = up[i], vpi = vp[i];
        const double Su = 0.5 * (ui * ui) + 0.5 * (upi * upi);
        const double Sv = 0.5 * (vi * vi) + 0.5 * (vpi * vpi);
        const double Suv = (0.5 * ui) * vi + (0.5 * upi) * vpi;
        double dxu = ax * Su, dyuv = ay * Suv, dyv = ay * Sv, dxuv = cf.inv_dx[cc] * Suv;
        if (west) {
            const double upj = up[iw], vpj = vp[iw];
            const double SuW = 0.5 * (uW * uW) + 0.5 * (upj * upj);
            const double SuvW = (0.5 * uW) * vW + (0.5 * upj) * vpj;
            dxu = dxu + (-axw) * SuW;
            dxuv = dxuv + (-cf.inv_dx[cc - 1]) * SuvW;
        }
        if (south) {
            const double upS = up[is], vpS = vp[is];
            const double SvS = 0.5 * (vS * vS) + 0.5 * (vpS * vpS);
            const double SuvS = (0.5 * uS) * vS + (0.5 * upS) * vpS;
            dyuv = dyuv + (-ays) * SuvS;
            dyv = dyv + (-ays) * SvS;
        }
        double ru = ui - upi;
        ru = ru + dxu;
        ru = ru + dyuv;
        ru = ru - cf.src[cc];
        ru = ru - (c == 0 ? cf.lbc[r] : 0.0);
        double rv = vi - vpi;
        rv = rv + dyv;
        rv = rv + a * dxuv;
        U[rr] = ui, V[rr] = vi, UW[rr] = uW, VW[rr] = vW, US[rr] = uS, VS[rr] = vS;
        RU[rr] = ru, RV[rr] = rv, AY[rr] = ay, AYS[rr] = ays;
    }
    const bool wl = lane0 && west;
    for (int k = blockIdx.z; k < npod; k += gridDim.z) {
        const double *xu = bt + (size_t)k * 2 * n, *xv = xu + n;
        double xuS = 0.0, xvS = 0.0;
        if (r0 > 0) {
            const size_t is = (size_t)(r0 - 1) * nx + cc;
            xuS = xu[is], xvS = xv[is];
        }
        double XU[kER], XV[kER], XUW[kER], XVW[kER];
#pragma unroll
        for (int rr = 0; rr < kER; ++rr) {
            if (rr >= nr) break;
            const size_t i = (size_t)(r0 + rr) * nx + cc;
            const size_t j = wl ? i - 1 : i;
            XU[rr] = xu[i], XV[rr] = xv[i], XUW[rr] = xu[j], XVW[rr] = xv[j];
        }
#pragma unroll
        for (int rr = 0; rr < kER; ++rr) {
            if (rr >= nr) break;
            const int r = r0 + rr;
            const size_t i = (size_t)r * nx + cc;
            const double ui = U[rr], vi = V[rr], xui = XU[rr], xvi = XV[rr];
            const double xuj = shr1(XUW[rr], xui), xvj = shr1(XVW[rr], xvi);
            // J(w) basis_k at the node (stencil.hip jvp / orc_jvp op order)
            const double ay = AY[rr], ays = AYS[rr];
            const double m = vi * xui + ui * xvi;
            double yu = xui + ax * ui * xui + 0.5 * ay * m;
            double yv = xvi + ay * vi * xvi + 0.5 * ax * m;
            if (west) {
                const double uW = UW[rr], vW = VW[rr];
                const double mW = vW * xuj + uW * xvj;
                yu -= axw * uW * xuj;
                yv -= 0.5 * axw * mW;
            }
            if (r > 0) {
                const double uS = US[rr], vS = VS[rr];
                const double mS = vS * xuS + uS * xvS;
                yu -= 0.5 * ays * mS;
                yv -= ays * vS * xvS;
            }
            if (colok) __builtin_nontemporal_store(RU[rr] * yu + RV[rr] * yv, &cblk[(size_t)k * n + i]);
            xuS = xui;
            xvS = xvi;
        }
    }
}

}  // namespace

int launch_basis_transpose(const double *b, double *bt, size_t m, int npod, hipStream_t st)
{
    const dim3 grid((unsigned)((m + 31) / 32), (unsigned)((npod + 31) / 32));
    hipLaunchKernelGGL(basis_transpose_kernel, grid, dim3(256), 0, st, b, bt, m, npod);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_ecsw(const Coeffs &cf, const double *w, const double *wp, const double *bt, int npod,
                double *cblk, hipStream_t st)
{
    const unsigned gx = (unsigned)((cf.nx + kEB - 1) / kEB), gy = (unsigned)((cf.ny + kER - 1) / kER);
    // basis-vector groups: enough workgroups to fill the chip (>= 2048)
    unsigned gz = 1;
    while (gz < (unsigned)npod && (size_t)gx * gy * gz < 2048) gz *= 2;
    gz = gz > (unsigned)npod ? (unsigned)npod : gz;
    hipLaunchKernelGGL(ecsw_kernel, dim3(gx, gy, gz), dim3(kEB), 0, st, cf, w, wp, bt, npod, cblk);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace burg
