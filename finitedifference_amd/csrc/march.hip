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
//
// Schedule per step: passes 1..P are launched over all tiles (one wavefront
// per tile, block Jacobi between tiles); pass P+1 is the FINAL kernel: every
// tile checks its inflow, and the last workgroup to finish (arrival ticket,
// agent-scope release/acquire) runs any further passes itself until no tile
// moves -- so a step always ends at the fixed point, with no host round trip
// and no idle launches.  It also folds the step's statistics.
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
// MARCH cell: inputs wp = (up, vp); outputs w = (u, v).
// Outflows: east (XF, XH) = ax*(F+Fp), ax*(H+Hp); north (YH, YG) = ay*(H+Hp),
// ay*(G+Gp), with F = u^2/2, G = v^2/2, H = u*v/2 (C/hypernet2D.py:2544-2547).
struct MarchCell {
    static constexpr int NIN = 2;
    struct Io {
        const double *in[NIN];  // up, vp planes
        double *out[2];         // u, v planes
    };
    struct Row {
        double ay, hy, lb;
    };
    __device__ static Row row(const Coeffs &cf, int r)
    {
        Row w;
        w.ay = cf.alpha * cf.inv_dy[r];
        w.hy = 0.5 * w.ay;
        w.lb = cf.lbc[r];
        return w;
    }
    // solve cell (r, c) given west (e0=XF, e1=XH) and south (n0=YH, n1=YG)
    // inflow; the inflow registers are overwritten with this cell's outflow.
    __device__ static void cell(const Coeffs &cf, const Row &rw, const double (&x)[NIN],
                                double invdx, double srcc, int c, double &e0, double &e1,
                                double &n0, double &n1, double &o0, double &o1)
    {
        const double pu = x[0], pv = x[1];
        const double ax = cf.alpha * invdx;
        const double hx = 0.5 * ax;
        const double sl = c == 0 ? srcc + rw.lb : srcc;
        const double hu = 0.5 * pu;
        const double xfp = ax * (hu * pu);
        const double xhp = ax * (hu * pv);
        const double yhp = rw.ay * (hu * pv);
        const double ygp = rw.ay * ((0.5 * pv) * pv);
        const double bu = ((pu - xfp) - yhp) + sl;
        const double bv = (pv - ygp) - xhp;
        const double cu = (bu + e0) + n0;
        const double cv = (bv + n1) + e1;
        const double mm = fma(hx, cu, rw.hy * cv);
        const double s = 0.5 + sqrt(0.25 + mm);
        const double rs = 1.0 / s;
        const double nu = cu * rs, nv = cv * rs;
        const double hxu = hx * nu;
        e0 = fma(hxu, nu, xfp);
        e1 = fma(hxu, nv, xhp);
        n0 = fma(rw.hy * nu, nv, yhp);
        n1 = fma(rw.hy * nv, nv, ygp);
        o0 = nu;
        o1 = nv;
    }
    // pass-1 guesses of a neighbour's outflow: "the neighbour did not move"
    __device__ static void guess_e(const Coeffs &cf, const Io &io, int r, int c, double &e0,
                                   double &e1)
    {
        const size_t i = (size_t)r * cf.nx + c;
        const double pu = io.in[0][i], pv = io.in[1][i];
        const double ax = cf.alpha * cf.inv_dx[c], hx = 0.5 * ax;
        const double hu = 0.5 * pu;
        e0 = fma(hx * pu, pu, ax * (hu * pu));
        e1 = fma(hx * pu, pv, ax * (hu * pv));
    }
    __device__ static void guess_n_vals(double ay, double pu, double pv, double &n0, double &n1)
    {
        const double hy = 0.5 * ay, hu = 0.5 * pu;
        n0 = fma(hy * pu, pv, ay * (hu * pv));
        n1 = fma(hy * pv, pv, ay * ((0.5 * pv) * pv));
    }
    __device__ static void guess_n(const Coeffs &cf, const Io &io, int r, int c, double &n0,
                                   double &n1)
    {
        const size_t i = (size_t)r * cf.nx + c;
        guess_n_vals(cf.alpha * cf.inv_dy[r], io.in[0][i], io.in[1][i], n0, n1);
    }
    __device__ static void guess_halo(const Coeffs &cf, const Engine &eg, int c, double &n0,
                                      double &n1)
    {
        guess_n_vals(cf.alpha * cf.inv_dy[-1], eg.halo_wp[c], eg.halo_wp[cf.nx + c], n0, n1);
    }
};

// ---------------------------------------------------------------------------
// SOLVE cell: exact J(w) delta = rhs, J from exact_jac2D (C/hypernet2D.py:2627).
// Inputs (u, v, ru, rv); outputs (du, dv).  Linearised outflows: east
// a = ax*u*du, b = 0.5*ax*(v*du + u*dv); north c = 0.5*ay*(v*du + u*dv),
// d = ay*v*dv.  Same op order as orc_block_solve.  Pass-1 guess: zero.
struct SolveCell {
    static constexpr int NIN = 4;
    struct Io {
        const double *in[NIN];  // u, v, ru, rv planes
        double *out[2];         // du, dv planes
    };
    struct Row {
        double ay;
    };
    __device__ static Row row(const Coeffs &cf, int r) { return Row{cf.alpha * cf.inv_dy[r]}; }
    __device__ static void cell(const Coeffs &cf, const Row &rw, const double (&x)[NIN],
                                double invdx, double, int, double &e0, double &e1, double &n0,
                                double &n1, double &o0, double &o1)
    {
        const double u = x[0], v = x[1];
        const double ax = cf.alpha * invdx, ay = rw.ay;
        const double eu = (x[2] + e0) + n0;
        const double ev = (x[3] + e1) + n1;
        const double a00 = (1.0 + ax * u) + (0.5 * ay) * v;
        const double a01 = (0.5 * ay) * u;
        const double a10 = (0.5 * ax) * v;
        const double a11 = (1.0 + ay * v) + (0.5 * ax) * u;
        const double det = a00 * a11 - a01 * a10;
        const double du = (a11 * eu - a01 * ev) / det;
        const double dv = (a00 * ev - a10 * eu) / det;
        const double m = v * du + u * dv;
        e0 = (ax * u) * du;
        e1 = (0.5 * ax) * m;
        n0 = (0.5 * ay) * m;
        n1 = (ay * v) * dv;
        o0 = du;
        o1 = dv;
    }
    __device__ static void guess_e(const Coeffs &, const Io &, int, int, double &e0, double &e1)
    {
        e0 = e1 = 0.0;
    }
    __device__ static void guess_n(const Coeffs &, const Io &, int, int, double &n0, double &n1)
    {
        n0 = n1 = 0.0;
    }
    __device__ static void guess_halo(const Coeffs &, const Engine &, int, double &n0,
                                      double &n1)
    {
        n0 = n1 = 0.0;
    }
};

// ---------------------------------------------------------------------------
// One tile, one pass, one workgroup of kWaves wavefronts.  Wave 0 gathers the
// inflow, decides whether the tile must be marched and sweeps it; all waves
// stage the tile's inputs into LDS with coalesced row loads before the sweep
// and write the outputs back coalesced after it (the sweeping wave touches
// only LDS: lane l reads [l][s-l], conflict-free since the pitch TW-1 is odd).
// Returns true (uniform over the workgroup) if the tile was marched.
// Generation `cur` of the edge planes receives its outflow (marched or
// carried), generation `prv` holds the neighbours' outflow of the previous
// pass.
constexpr int kWaves = 4;
constexpr int kThreads = kWaves * kWave;

template <class C, int TW>
struct TileLds {
    double x[C::NIN][kWave * TW];  // staged inputs; planes 0/1 are overwritten by outputs
    double dx[TW], src[TW];        // per-column inv_dx, src of the tile
    double nout[2][TW];            // north outflow (top row), flushed after the sweep
    int need;
};

template <class C, int TW>
__device__ bool tile_pass(const Coeffs &cf, const Engine &eg, const typename C::Io &io, int t,
                          int pass, TileLds<C, TW> &sm)
{
    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & (kWave - 1);
    const int I = t / eg.ntj, J = t - I * eg.ntj;
    const int nx = cf.nx, ny = cf.ny;
    const int r0 = I * kWave, c0 = J * TW;
    const int nrow = min(kWave, ny - r0), ncol = min(TW, nx - c0);
    const bool rowok = lane < nrow;
    const int r = r0 + (rowok ? lane : nrow - 1);
    const int cur = pass & 1, prv = cur ^ 1;
    constexpr int NQ = TW / kWave;  // south-edge columns held per lane

    // ---- wave 0: inflow, west (per row) and south (per column, lane l holds l + 64q)
    double we0 = 0.0, we1 = 0.0;
    double sn0[NQ], sn1[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) sn0[q] = sn1[q] = 0.0;
    double *wu = eg.wused + (size_t)t * 2 * kWave;
    double *su = eg.sused + (size_t)t * 2 * TW;
    if (wave == 0) {
        if (J > 0) {
            if (pass == 1) {
                C::guess_e(cf, io, r, c0 - 1, we0, we1);
            } else {
                const double *e = eg.eb[prv] + (size_t)(t - 1) * 2 * kWave;
                we0 = e[lane];
                we1 = e[kWave + lane];
            }
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int col = lane + kWave * q;
            if (col >= ncol) continue;
            if (I > 0) {
                if (pass == 1) {
                    C::guess_n(cf, io, r0 - 1, c0 + col, sn0[q], sn1[q]);
                } else {
                    const double *nn = eg.nb[prv] + (size_t)(t - eg.ntj) * 2 * TW;
                    sn0[q] = nn[col];
                    sn1[q] = nn[TW + col];
                }
            } else if (eg.halo_flux != nullptr) {
                if (pass == 1) {
                    C::guess_halo(cf, eg, c0 + col, sn0[q], sn1[q]);
                } else {
                    sn0[q] = eg.halo_flux[c0 + col];
                    sn1[q] = eg.halo_flux[nx + c0 + col];
                }
            }
        }
        // skip test: march again only if some inflow moved since last used
        bool need = true;
        if (pass > 1) {
            bool mv = rowok &&
                      (moved(we0, wu[lane], eg.tol) || moved(we1, wu[kWave + lane], eg.tol));
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int col = lane + kWave * q;
                if (col < ncol)
                    mv = mv || moved(sn0[q], su[col], eg.tol) ||
                         moved(sn1[q], su[TW + col], eg.tol);
            }
            need = __any(mv);
        }
        if (lane == 0) sm.need = need;
    }
    __syncthreads();
    const bool need = sm.need;
    if (!need) {
        if (wave == 0) {  // carry this tile's outflow into the current generation
            const double *ep = eg.eb[prv] + (size_t)t * 2 * kWave;
            double *ec = eg.eb[cur] + (size_t)t * 2 * kWave;
            ec[lane] = ep[lane];
            ec[kWave + lane] = ep[kWave + lane];
            const double *np_ = eg.nb[prv] + (size_t)t * 2 * TW;
            double *nc = eg.nb[cur] + (size_t)t * 2 * TW;
#pragma unroll
            for (int q = 0; q < 2 * NQ; ++q) nc[lane + kWave * q] = np_[lane + kWave * q];
        }
        __syncthreads();  // sm reused by the next tile
        return false;
    }

    // ---- stage the tile's inputs: coalesced row segments -> LDS [row][col]
    const size_t tbase = (size_t)r0 * nx + c0;
    for (int e = tid; e < kWave * TW; e += kThreads) {
        const int rr = e / TW, cc = e - rr * TW;
        if (rr < nrow && cc < ncol) {
            const size_t g = tbase + (size_t)rr * nx + cc;
#pragma unroll
            for (int q = 0; q < C::NIN; ++q) sm.x[q][e] = io.in[q][g];
        }
    }
    for (int cc = tid; cc < TW; cc += kThreads) {
        const int c = c0 + min(cc, ncol - 1);
        sm.dx[cc] = cf.inv_dx[c];
        sm.src[cc] = cf.src[c];
    }
    if (wave == 0) {
        if (rowok) {
            wu[lane] = we0;
            wu[kWave + lane] = we1;
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int col = lane + kWave * q;
            if (col < ncol) {
                su[col] = sn0[q];
                su[TW + col] = sn1[q];
            }
        }
    }
    __syncthreads();

    // ---- wave 0: skewed sweep, lane l marches row r0+l, column j = s - l.
    // Only LDS and registers inside the loop; the next step's operands are
    // read one step ahead so the LDS latency hides under the cell's math.
    if (wave == 0) {
        const typename C::Row rw = C::row(cf, r);
        double e0 = we0, e1 = we1;    // running west inflow of my row
        double no0 = 0.0, no1 = 0.0;  // my last north outflow (for lane + 1)
        const int nsteps = ncol + nrow - 1;
        double *lrow[C::NIN];
#pragma unroll
        for (int q = 0; q < C::NIN; ++q) lrow[q] = sm.x[q] + lane * TW;
        double xn[C::NIN], dxn, scn;
        {
            const int jn = min(max(-lane, 0), ncol - 1);
#pragma unroll
            for (int q = 0; q < C::NIN; ++q) xn[q] = lrow[q][jn];
            dxn = sm.dx[jn];
            scn = sm.src[jn];
        }
        for (int s = 0; s < nsteps; ++s) {
            double xc[C::NIN];
#pragma unroll
            for (int q = 0; q < C::NIN; ++q) xc[q] = xn[q];
            const double dxc = dxn, scc = scn;
            {
                const int jn = min(max(s + 1 - lane, 0), ncol - 1);
#pragma unroll
                for (int q = 0; q < C::NIN; ++q) xn[q] = lrow[q][jn];
                dxn = sm.dx[jn];
                scn = sm.src[jn];
            }
            double n0 = shr1(no0), n1 = shr1(no1);
            if (s < ncol) {  // lane 0 takes the tile's south edge for column s
                double a, b;
                if constexpr (NQ == 1) {
                    a = readlane(sn0[0], s);
                    b = readlane(sn1[0], s);
                } else {
                    const int l = s & 63;
                    a = (s >> 6) == 0 ? readlane(sn0[0], l) : readlane(sn0[NQ - 1], l);
                    b = (s >> 6) == 0 ? readlane(sn1[0], l) : readlane(sn1[NQ - 1], l);
                }
                if (lane == 0) {
                    n0 = a;
                    n1 = b;
                }
            }
            const int j = s - lane;
            if (rowok && j >= 0 && j < ncol) {
                double o0, o1;
                C::cell(cf, rw, xc, dxc, scc, c0 + j, e0, e1, n0, n1, o0, o1);
                lrow[0][j] = o0;
                lrow[1][j] = o1;
                no0 = n0;
                no1 = n1;
                if (lane == nrow - 1) {
                    sm.nout[0][j] = n0;
                    sm.nout[1][j] = n1;
                }
            }
        }
        if (rowok) {
            double *ec = eg.eb[cur] + (size_t)t * 2 * kWave;
            ec[lane] = e0;
            ec[kWave + lane] = e1;
        }
    }
    __syncthreads();
    {
        double *nout = eg.nb[cur] + (size_t)t * 2 * TW;
        for (int cc = tid; cc < ncol; cc += kThreads) {
            nout[cc] = sm.nout[0][cc];
            nout[TW + cc] = sm.nout[1][cc];
        }
    }

    // ---- write the outputs back, coalesced
    for (int e = tid; e < kWave * TW; e += kThreads) {
        const int rr = e / TW, cc = e - rr * TW;
        if (rr < nrow && cc < ncol) {
            const size_t g = tbase + (size_t)rr * nx + cc;
            io.out[0][g] = sm.x[0][e];
            io.out[1][g] = sm.x[1][e];
        }
    }
    __syncthreads();  // sm reused by the next tile
    return true;
}

template <class C, int TW>
__global__ __launch_bounds__(kThreads) void pass_kernel(Coeffs cf, Engine eg, typename C::Io io,
                                                        int pass)
{
    __shared__ TileLds<C, TW> sm;
    if (pass > 1 && eg.counters[pass - 1] == 0) return;  // converged already
    if (tile_pass<C, TW>(cf, eg, io, blockIdx.x, pass, sm) && threadIdx.x == 0)
        atomicAdd(&eg.counters[pass], 1);
}

// FINAL pass (pass = P+1): all tiles check/march once; the last workgroup to
// arrive continues alone with passes P+2, P+3, ... until a pass marches
// nothing (the bound #tile anti-diagonals + 1 guarantees termination), then
// folds the step's counters into the run statistics and resets them.
template <class C, int TW>
__global__ __launch_bounds__(kThreads) void final_kernel(Coeffs cf, Engine eg, typename C::Io io,
                                                         int pass, DevStats *stats)
{
    __shared__ TileLds<C, TW> sm;
    const bool live = !(pass > 1 && eg.counters[pass - 1] == 0);
    if (live && tile_pass<C, TW>(cf, eg, io, blockIdx.x, pass, sm) && threadIdx.x == 0)
        atomicAdd(&eg.counters[pass], 1);
    // arrival: every storing wave drains, then one release and the ticket
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int last;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int tk = atomicAdd(eg.ticket, 1);
        last = (tk == (int)gridDim.x - 1);
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!last) return;

    const int ntiles = eg.nti * eg.ntj;
    int k = pass;
    int moved_last = live ? __hip_atomic_load(&eg.counters[k], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT)
                          : 0;
    int tail = 0;
    __shared__ int cnt;
    while (moved_last != 0 && k < eg.kbound) {
        ++k;
        ++tail;
        if (threadIdx.x == 0) cnt = 0;
        __syncthreads();
        for (int t = 0; t < ntiles; ++t)
            if (tile_pass<C, TW>(cf, eg, io, t, k, sm) && threadIdx.x == 0) ++cnt;
        // pass k's edges (stored by one lane, read by others next pass)
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __syncthreads();
        moved_last = cnt;
        if (threadIdx.x == 0) eg.counters[k] = cnt;
    }
    if (threadIdx.x == 0) {
        long long tiles = 0;
        int used = 0;
        for (int q = 1; q <= k; ++q) {
            const int cq = __hip_atomic_load(&eg.counters[q], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
            tiles += cq;
            if (used == 0 && cq == 0) used = q;
            eg.counters[q] = 0;
        }
        if (used == 0) {  // hit the bound (cannot happen: see DESIGN.md section 4)
            stats->unconverged_steps += 1;
            used = k;
        }
        stats->tile_marches += tiles;
        stats->steps += 1;
        stats->passes += used;
        stats->tail_passes += tail;
        if (used > stats->max_passes) stats->max_passes = used;
        // the engine keeps the generation parity of the final outflow
        *eg.ticket = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    }
}

template <class C>
int launch_pass(const Coeffs &cf, const Engine &eg, const typename C::Io &io, int pass,
                bool final, DevStats *stats, hipStream_t st)
{
    const dim3 grid(eg.nti * eg.ntj), block(kThreads);
    if (eg.tw == 64) {
        if (final)
            final_kernel<C, 64><<<grid, block, 0, st>>>(cf, eg, io, pass, stats);
        else
            pass_kernel<C, 64><<<grid, block, 0, st>>>(cf, eg, io, pass);
    } else if constexpr (C::NIN * 128 * kWave * 8 <= 160 * 1024) {
        if (eg.tw != 128) return -1;
        if (final)
            final_kernel<C, 128><<<grid, block, 0, st>>>(cf, eg, io, pass, stats);
        else
            pass_kernel<C, 128><<<grid, block, 0, st>>>(cf, eg, io, pass);
    } else {
        return -1;  // LDS budget: the 4-plane SOLVE cell needs tile_w = 64
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace

int launch_march_pass(const Coeffs &cf, const Engine &eg, const double *wp, double *w,
                      int pass, bool final, DevStats *stats, hipStream_t st)
{
    const size_t n = (size_t)cf.nx * cf.ny;
    MarchCell::Io io{{wp, wp + n}, {w, w + n}};
    return launch_pass<MarchCell>(cf, eg, io, pass, final, stats, st);
}

int launch_solve_pass(const Coeffs &cf, const Engine &eg, const double *w, const double *rhs,
                      double *delta, int pass, bool final, DevStats *stats, hipStream_t st)
{
    const size_t n = (size_t)cf.nx * cf.ny;
    SolveCell::Io io{{w, w + n, rhs, rhs + n}, {delta, delta + n}};
    return launch_pass<SolveCell>(cf, eg, io, pass, final, stats, st);
}

}  // namespace burg
