// march.hip -- the upwind tile engine: one implicit time step of the 2D
// inviscid Burgers FOM (MARCH cell) and the exact Newton linear solve
// J(w) delta = rhs (SOLVE cell), both as a skewed-wavefront sweep over
// 64-row tiles with block-Jacobi passes between tiles (DESIGN.md sections 3-4).
//
// Why a march: the reference residual (C/hypernet2D.py:2512-2570) couples a
// cell only to itself, its west (r, c-1) and south (r-1, c) neighbours, so
// R(w) = 0 is lower-triangular in (r, c) order and can be solved cell by
// cell.  Per cell the 2x2 system is u*s = Cu, v*s = Cv with the common factor
// s = 1 + hx*u + hy*v, hence s = 0.5 + sqrt(0.25 + hx*Cu + hy*Cv): the exact
// implicit step in closed form, replacing newton_raphson (:1811-1857) +
// spsolve (:1854).  The SOLVE cell is the same sweep for the linearised
// system (exact_jac2D, :2627-2656), used by the reference-faithful Newton mode.
//
// Op order of both cells is normative: oracle/burgers_oracle.c restates it
// (orc_march_step / orc_block_solve / orc_march_tiled_sim) and the GPU result
// is compared against it (bitwise for equal tiling and tolerance).
#include "burg_internal.h"

namespace burg {
namespace {

__device__ __forceinline__ double shr1(double x)
{
    // lane i <- lane i-1 (wave-wide DPP shift; lane 0 keeps 0)
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double readlane(double x, int l)
{
    const int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ bool moved(double a, double b, double tol)
{
    if (tol == 0.0) return a != b;
    return fabs(a - b) > tol * fmax(fabs(a), fabs(b));
}

// ---------------------------------------------------------------------------
// MARCH cell: inputs wp (up, vp); outputs w (u, v).
// Outflows: east (XF, XH) = ax*(F+Fp), ax*(H+Hp); north (YH, YG) = ay*(H+Hp),
// ay*(G+Gp), with F = u^2/2, G = v^2/2, H = u*v/2 (C/hypernet2D.py:2544-2547).
struct MarchCell {
    struct In {
        const double *p0;  // up plane (wp)
        const double *p1;  // vp plane
        double *o0;        // u plane (w)
        double *o1;        // v plane
    };
    struct Pre {
        double xfp, xhp, yhp, ygp, bu, bv;
    };
    __device__ static Pre pre(const Coeffs &cf, double ax, double ay, double sl, double pu,
                              double pv)
    {
        Pre p;
        const double hu = 0.5 * pu;
        p.xfp = ax * (hu * pu);
        p.xhp = ax * (hu * pv);
        p.yhp = ay * (hu * pv);
        p.ygp = ay * ((0.5 * pv) * pv);
        p.bu = ((pu - p.xfp) - p.yhp) + sl;
        p.bv = (pv - p.ygp) - p.xhp;
        return p;
    }
    // solve one cell given west (xf, xh) and south (yh, yg) inflow; returns
    // state and overwrites the inflow registers with this cell's outflow.
    __device__ static void step(const Pre &p, double hx, double hy, double &xf, double &xh,
                                double &yh, double &yg, double &nu, double &nv)
    {
        const double cu = (p.bu + xf) + yh;
        const double cv = (p.bv + yg) + xh;
        const double mm = fma(hx, cu, hy * cv);
        const double s = 0.5 + sqrt(0.25 + mm);
        const double rs = 1.0 / s;
        nu = cu * rs;
        nv = cv * rs;
        const double hxu = hx * nu;
        xf = fma(hxu, nu, p.xfp);
        xh = fma(hxu, nv, p.xhp);
        yh = fma(hy * nu, nv, p.yhp);
        yg = fma(hy * nv, nv, p.ygp);
    }
    // pass-1 guess of a neighbour's outflow: "the neighbour did not move"
    __device__ static void guess_e(double ax, double hx, double pu, double pv, double &xf,
                                   double &xh)
    {
        const double hu = 0.5 * pu;
        xf = fma(hx * pu, pu, ax * (hu * pu));
        xh = fma(hx * pu, pv, ax * (hu * pv));
    }
    __device__ static void guess_n(double ay, double hy, double pu, double pv, double &yh,
                                   double &yg)
    {
        const double hu = 0.5 * pu;
        yh = fma(hy * pu, pv, ay * (hu * pv));
        yg = fma(hy * pv, pv, ay * ((0.5 * pv) * pv));
    }
};

template <int TW>
__global__ __launch_bounds__(64) void march_pass_kernel(Coeffs cf, Engine eg,
                                                        MarchCell::In io, int pass)
{
    const int t = blockIdx.x;
    if (pass > 1 && eg.counters[pass - 1] == 0) return;  // converged: idempotent pass
    const int lane = threadIdx.x;
    const int I = t / eg.ntj, J = t - I * eg.ntj;
    const int nx = cf.nx, ny = cf.ny;
    const int r0 = I * kWave, c0 = J * TW;
    const int nrow = min(kWave, ny - r0), ncol = min(TW, nx - c0);
    const bool rowok = lane < nrow;
    const int r = r0 + (rowok ? lane : nrow - 1);
    const int cur = pass & 1, prv = cur ^ 1;
    constexpr int NQ = TW / kWave;  // S-edge columns held per lane
    const size_t nplane = (size_t)nx * ny;
    (void)nplane;

    // ---- inflow: west (per row) and south (per column, lane l holds l + 64q)
    double wxf = 0.0, wxh = 0.0;
    double sh[NQ], sg[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) sh[q] = sg[q] = 0.0;

    if (J > 0) {
        if (pass == 1) {
            const int c = c0 - 1;
            const size_t i = (size_t)r * nx + c;
            const double ax = cf.alpha * cf.inv_dx[c];
            MarchCell::guess_e(ax, 0.5 * ax, io.p0[i], io.p1[i], wxf, wxh);
        } else {
            const double *e = eg.eb[prv] + (size_t)(t - 1) * 2 * kWave;
            wxf = e[lane];
            wxh = e[kWave + lane];
        }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int col = lane + kWave * q;
        if (col >= ncol) continue;
        const int c = c0 + col;
        if (I > 0) {
            if (pass == 1) {
                const size_t i = (size_t)(r0 - 1) * nx + c;
                const double ay = cf.alpha * cf.inv_dy[r0 - 1];
                MarchCell::guess_n(ay, 0.5 * ay, io.p0[i], io.p1[i], sh[q], sg[q]);
            } else {
                const double *nn = eg.nb[prv] + (size_t)(t - eg.ntj) * 2 * TW;
                sh[q] = nn[col];
                sg[q] = nn[TW + col];
            }
        } else if (eg.halo_flux != nullptr) {
            if (pass == 1) {
                const double ay = cf.alpha * cf.inv_dy[-1];  // row below the slab
                MarchCell::guess_n(ay, 0.5 * ay, eg.halo_wp[c], eg.halo_wp[nx + c], sh[q],
                                   sg[q]);
            } else {
                sh[q] = eg.halo_flux[c];
                sg[q] = eg.halo_flux[nx + c];
            }
        }
    }

    // ---- skip test: re-march only if some inflow moved since last used
    double *wu = eg.wused + (size_t)t * 2 * kWave;
    double *su = eg.sused + (size_t)t * 2 * TW;
    if (pass > 1) {
        bool mv = rowok && (moved(wxf, wu[lane], eg.tol) || moved(wxh, wu[kWave + lane], eg.tol));
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int col = lane + kWave * q;
            if (col < ncol)
                mv = mv || moved(sh[q], su[col], eg.tol) || moved(sg[q], su[TW + col], eg.tol);
        }
        if (!__any(mv)) {
            // carry this tile's outflow into the current generation
            const double *ep = eg.eb[prv] + (size_t)t * 2 * kWave;
            double *ec = eg.eb[cur] + (size_t)t * 2 * kWave;
            ec[lane] = ep[lane];
            ec[kWave + lane] = ep[kWave + lane];
            const double *np_ = eg.nb[prv] + (size_t)t * 2 * TW;
            double *nc = eg.nb[cur] + (size_t)t * 2 * TW;
#pragma unroll
            for (int q = 0; q < 2 * NQ; ++q) nc[lane + kWave * q] = np_[lane + kWave * q];
            return;
        }
    }
    if (rowok) {
        wu[lane] = wxf;
        wu[kWave + lane] = wxh;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int col = lane + kWave * q;
        if (col < ncol) {
            su[col] = sh[q];
            su[TW + col] = sg[q];
        }
    }

    // ---- skewed sweep: lane l marches row r0+l, column j = s - l at step s
    const double ay = cf.alpha * cf.inv_dy[r];
    const double hy = 0.5 * ay;
    const double lb = cf.lbc[r];
    double xf = wxf, xh = wxh;      // running west inflow of my row
    double yho = 0.0, ygo = 0.0;    // my last north outflow (for lane + 1)
    double *nout = eg.nb[cur] + (size_t)t * 2 * TW;
    const int nsteps = ncol + nrow - 1;
    const size_t rowbase = (size_t)r * nx + c0;
    for (int s = 0; s < nsteps; ++s) {
        double yh = shr1(yho), yg = shr1(ygo);
        if (s < ncol) {  // lane 0 takes the tile's south edge for column s
            double eh, eg_;
            if constexpr (NQ == 1) {
                eh = readlane(sh[0], s);
                eg_ = readlane(sg[0], s);
            } else {
                const int q = s >> 6, l = s & 63;
                eh = q == 0 ? readlane(sh[0], l) : readlane(sh[NQ - 1], l);
                eg_ = q == 0 ? readlane(sg[0], l) : readlane(sg[NQ - 1], l);
            }
            if (lane == 0) {
                yh = eh;
                yg = eg_;
            }
        }
        const int j = s - lane;
        if (rowok && j >= 0 && j < ncol) {
            const int c = c0 + j;
            const size_t i = rowbase + j;
            const double pu = io.p0[i], pv = io.p1[i];
            const double ax = cf.alpha * cf.inv_dx[c];
            const double sl = c == 0 ? cf.src[0] + lb : cf.src[c];
            const MarchCell::Pre p = MarchCell::pre(cf, ax, ay, sl, pu, pv);
            double nu, nv;
            MarchCell::step(p, 0.5 * ax, hy, xf, xh, yh, yg, nu, nv);
            io.o0[i] = nu;
            io.o1[i] = nv;
            yho = yh;
            ygo = yg;
            if (lane == nrow - 1) {
                nout[j] = yh;
                nout[TW + j] = yg;
            }
        }
    }
    if (rowok) {
        double *ec = eg.eb[cur] + (size_t)t * 2 * kWave;
        ec[lane] = xf;
        ec[kWave + lane] = xh;
    }
    if (lane == 0) atomicAdd(&eg.counters[pass], 1);
}

// ---------------------------------------------------------------------------
// SOLVE cell: exact J(w) delta = rhs, J from exact_jac2D (C/hypernet2D.py:2627).
// Linearised outflows: east a = ax*u*du, b = 0.5*ax*(v*du + u*dv);
// north c = 0.5*ay*(v*du + u*dv), d = ay*v*dv.  Same op order as
// orc_block_solve.
template <int TW>
__global__ __launch_bounds__(64) void solve_pass_kernel(Coeffs cf, Engine eg,
                                                        const double *w, const double *rhs,
                                                        double *delta, int pass)
{
    const int t = blockIdx.x;
    if (pass > 1 && eg.counters[pass - 1] == 0) return;
    const int lane = threadIdx.x;
    const int I = t / eg.ntj, J = t - I * eg.ntj;
    const int nx = cf.nx, ny = cf.ny;
    const size_t n = (size_t)nx * ny;
    const int r0 = I * kWave, c0 = J * TW;
    const int nrow = min(kWave, ny - r0), ncol = min(TW, nx - c0);
    const bool rowok = lane < nrow;
    const int r = r0 + (rowok ? lane : nrow - 1);
    const int cur = pass & 1, prv = cur ^ 1;
    constexpr int NQ = TW / kWave;

    double wa = 0.0, wb = 0.0;  // west inflow (pass 1 guess: 0)
    double sc[NQ], sd[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) sc[q] = sd[q] = 0.0;
    if (pass > 1) {
        if (J > 0) {
            const double *e = eg.eb[prv] + (size_t)(t - 1) * 2 * kWave;
            wa = e[lane];
            wb = e[kWave + lane];
        }
        if (I > 0) {
            const double *nn = eg.nb[prv] + (size_t)(t - eg.ntj) * 2 * TW;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int col = lane + kWave * q;
                if (col < ncol) {
                    sc[q] = nn[col];
                    sd[q] = nn[TW + col];
                }
            }
        }
    }
    double *wu = eg.wused + (size_t)t * 2 * kWave;
    double *su = eg.sused + (size_t)t * 2 * TW;
    if (pass > 1) {
        bool mv = rowok && (moved(wa, wu[lane], eg.tol) || moved(wb, wu[kWave + lane], eg.tol));
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int col = lane + kWave * q;
            if (col < ncol)
                mv = mv || moved(sc[q], su[col], eg.tol) || moved(sd[q], su[TW + col], eg.tol);
        }
        if (!__any(mv)) {
            const double *ep = eg.eb[prv] + (size_t)t * 2 * kWave;
            double *ec = eg.eb[cur] + (size_t)t * 2 * kWave;
            ec[lane] = ep[lane];
            ec[kWave + lane] = ep[kWave + lane];
            const double *np_ = eg.nb[prv] + (size_t)t * 2 * TW;
            double *nc = eg.nb[cur] + (size_t)t * 2 * TW;
#pragma unroll
            for (int q = 0; q < 2 * NQ; ++q) nc[lane + kWave * q] = np_[lane + kWave * q];
            return;
        }
    }
    if (rowok) {
        wu[lane] = wa;
        wu[kWave + lane] = wb;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int col = lane + kWave * q;
        if (col < ncol) {
            su[col] = sc[q];
            su[TW + col] = sd[q];
        }
    }

    const double ay = cf.alpha * cf.inv_dy[r];
    double ea = wa, eb = wb;
    double nco = 0.0, ndo = 0.0;
    double *nout = eg.nb[cur] + (size_t)t * 2 * TW;
    const int nsteps = ncol + nrow - 1;
    const size_t rowbase = (size_t)r * nx + c0;
    for (int s = 0; s < nsteps; ++s) {
        double ic = shr1(nco), id = shr1(ndo);
        if (s < ncol) {
            double e0, e1;
            if constexpr (NQ == 1) {
                e0 = readlane(sc[0], s);
                e1 = readlane(sd[0], s);
            } else {
                const int q = s >> 6, l = s & 63;
                e0 = q == 0 ? readlane(sc[0], l) : readlane(sc[NQ - 1], l);
                e1 = q == 0 ? readlane(sd[0], l) : readlane(sd[NQ - 1], l);
            }
            if (lane == 0) {
                ic = e0;
                id = e1;
            }
        }
        const int j = s - lane;
        if (rowok && j >= 0 && j < ncol) {
            const int c = c0 + j;
            const size_t i = rowbase + j;
            const double u = w[i], v = w[n + i];
            const double ax = cf.alpha * cf.inv_dx[c];
            const double eu = (rhs[i] + ea) + ic;
            const double ev = (rhs[n + i] + eb) + id;
            const double a00 = (1.0 + ax * u) + (0.5 * ay) * v;
            const double a01 = (0.5 * ay) * u;
            const double a10 = (0.5 * ax) * v;
            const double a11 = (1.0 + ay * v) + (0.5 * ax) * u;
            const double det = a00 * a11 - a01 * a10;
            const double du = (a11 * eu - a01 * ev) / det;
            const double dv = (a00 * ev - a10 * eu) / det;
            delta[i] = du;
            delta[n + i] = dv;
            const double m = v * du + u * dv;
            ea = (ax * u) * du;
            eb = (0.5 * ax) * m;
            nco = (0.5 * ay) * m;
            ndo = (ay * v) * dv;
            if (lane == nrow - 1) {
                nout[j] = nco;
                nout[TW + j] = ndo;
            }
        }
    }
    if (rowok) {
        double *ec = eg.eb[cur] + (size_t)t * 2 * kWave;
        ec[lane] = ea;
        ec[kWave + lane] = eb;
    }
    if (lane == 0) atomicAdd(&eg.counters[pass], 1);
}

// One thread: fold the pass counters of the step into the run statistics and
// reset them for the next step.  Pass k "confirms" the step when it marched
// no tile; a step whose every allowed pass still marched tiles is counted as
// unconverged (only possible when max_passes is set below the guaranteed
// bound of #tile-anti-diagonals + 1).
__global__ void pass_epilogue_kernel(int *counters, int kmax, DevStats *stats)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    long long tiles = 0;
    int used = 0;
    for (int k = 1; k <= kmax; ++k) {
        const int ck = counters[k];
        tiles += ck;
        if (used == 0 && ck == 0) used = k;
        counters[k] = 0;
    }
    if (used == 0) {
        stats->unconverged_steps += 1;
        used = kmax;
    }
    stats->tile_marches += tiles;
    stats->steps += 1;
    stats->passes += used;
    if (used > stats->max_passes) stats->max_passes = used;
}

}  // namespace

int launch_march_pass(const Coeffs &cf, const Engine &eg, const double *wp, double *w,
                      int pass, hipStream_t st)
{
    const size_t n = (size_t)cf.nx * cf.ny;
    MarchCell::In io{wp, wp + n, w, w + n};
    const dim3 grid(eg.nti * eg.ntj), block(kWave);
    if (eg.tw == 64)
        march_pass_kernel<64><<<grid, block, 0, st>>>(cf, eg, io, pass);
    else if (eg.tw == 128)
        march_pass_kernel<128><<<grid, block, 0, st>>>(cf, eg, io, pass);
    else
        return -1;
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_solve_pass(const Coeffs &cf, const Engine &eg, const double *w,
                      const double *rhs, double *delta, int pass, hipStream_t st)
{
    const dim3 grid(eg.nti * eg.ntj), block(kWave);
    if (eg.tw == 64)
        solve_pass_kernel<64><<<grid, block, 0, st>>>(cf, eg, w, rhs, delta, pass);
    else if (eg.tw == 128)
        solve_pass_kernel<128><<<grid, block, 0, st>>>(cf, eg, w, rhs, delta, pass);
    else
        return -1;
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_pass_epilogue(const Engine &eg, int kmax, DevStats *stats, hipStream_t st)
{
    pass_epilogue_kernel<<<1, 64, 0, st>>>(eg.counters, kmax, stats);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace burg
