// march.hip -- the upwind tile engine: one implicit time step of the 2D
// inviscid Burgers FOM (MARCH cell) and the exact Newton linear solve
// J(w) delta = rhs (SOLVE cell), both as a skewed-wavefront sweep over
// 64-row tiles with block-Jacobi passes between tiles (DESIGN.md sections 3-5).
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
// Schedule per step: passes 1..P are launched over all tiles (one workgroup
// per tile, block Jacobi between tiles); pass P+1 is the FINAL kernel: every
// tile checks its inflow, and the last workgroup to finish (arrival ticket,
// agent-scope release/acquire) runs any further passes itself until no tile
// moves -- so a step always ends at the fixed point, with no host round trip
// and no idle launches.  It also folds the step's statistics.
//
// Inside a tile the critical path is the skewed sweep: 64 + 64 - 1 dependent
// steps of one wavefront.  A lone wave issues about one VALU instruction per
// 4-5 cycles whatever the instruction (measured), so the
// sweeping wave executes only the cell chain, the DPP hand-over and its
// commits; a helper wave on another SIMD precomputes the inflow-independent
// part of each cell into an LDS ring a few diagonals ahead.
#include "burg_internal.h"
#include "cell_math.h"

#ifdef BURG_STAMPS
__device__ long long burg_stamp[4];
#endif

namespace burg {
namespace {

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
    struct Pre {
        double ru, rv, a00, a01, a10, a11, det, axu, hax, hay, ayv, u, v;
    };
    static constexpr int NPRE = 13;
    __device__ static void pack(const Pre &p, double (&f)[NPRE])
    {
        f[0] = p.ru, f[1] = p.rv, f[2] = p.a00, f[3] = p.a01, f[4] = p.a10, f[5] = p.a11;
        f[6] = p.det, f[7] = p.axu, f[8] = p.hax, f[9] = p.hay, f[10] = p.ayv, f[11] = p.u;
        f[12] = p.v;
    }
    __device__ static Pre unpack(const double *f)
    {
        return Pre{f[0], f[1], f[2], f[3], f[4], f[5], f[6], f[7], f[8], f[9], f[10], f[11], f[12]};
    }
    __device__ static Pre pre(const Coeffs &cf, const Row &rw, const double *x, double invdx,
                              double, bool)
    {
        Pre p;
        const double u = x[0], v = x[1];
        const double ax = cf.alpha * invdx, ay = rw.ay;
        p.u = u;
        p.v = v;
        p.ru = x[2];
        p.rv = x[3];
        p.a00 = (1.0 + ax * u) + (0.5 * ay) * v;
        p.a01 = (0.5 * ay) * u;
        p.a10 = (0.5 * ax) * v;
        p.a11 = (1.0 + ay * v) + (0.5 * ax) * u;
        p.det = p.a00 * p.a11 - p.a01 * p.a10;
        p.axu = ax * u;
        p.hax = 0.5 * ax;
        p.hay = 0.5 * ay;
        p.ayv = ay * v;
        return p;
    }
    template <bool FAST>
    __device__ static void chain(const Pre &p, const Row &, double e0, double e1, double n0,
                                 double n1, double &oe0, double &oe1, double &on0, double &on1,
                                 double &o0, double &o1, bool &range_ok)
    {
        const double eu = (p.ru + e0) + n0;
        const double ev = (p.rv + e1) + n1;
        const double du = (p.a11 * eu - p.a01 * ev) / p.det;
        const double dv = (p.a00 * ev - p.a10 * eu) / p.det;
        const double m = p.v * du + p.u * dv;
        oe0 = p.axu * du;
        oe1 = p.hax * m;
        on0 = p.hay * m;
        on1 = p.ayv * dv;
        o0 = du;
        o1 = dv;
        range_ok = true;
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
// LDS image of one tile (one workgroup of kWaves wavefronts).
constexpr int kWaves = 4;
constexpr int kThreads = kWaves * kWave;
constexpr int kEp = kWaves - 1;  // sweep steps per epoch: one diagonal per helper wave
constexpr int kNE = 3;            // epochs held in the helper ring

template <class C>
constexpr int ring_pairs = (C::NPRE + 2 + 1) / 2;  // Pre fields + south inflow, as pairs

template <class C, bool HELPED>
struct Ring {
    // [epoch][step][field pair][lane][2]: Pre fields, then the lane's south
    // inflow (lane 0 only; +0.0 elsewhere); 16-byte pairs for b128 access
    double v[kNE][kEp][ring_pairs<C>][kWave][2];
};
template <class C>
struct Ring<C, false> {
};

// the helped sweep needs the tile (interleaved inputs) and the ring in LDS
template <class C, int TW>
constexpr bool helped_v = (size_t)C::NIN * TW * kWave * 8 +
                              sizeof(double) * kNE * kEp * ring_pairs<C> * 2 * kWave <=
                          150 * 1024;

template <class C, int TW>
struct TileLds {
    Ring<C, helped_v<C, TW>> ring;  // first: every ring access has an immediate offset
    double x[kWave * TW][C::NIN];   // inputs [row*TW + col][field]; fields 0/1 -> outputs
    double dx[TW], src[TW];         // per-column inv_dx, src of the tile
    double sedge[TW][2];            // south inflow of the tile
    double nout[TW][2];             // north outflow (top row), flushed after the sweep
    double trash[2][kWave][2];      // writes of lanes outside the tile this step
    int need;
};

// All waves: the tile's inputs, coalesced row segments -> LDS (missing cells
// of a partial tile read as 1.0: harmless operands for the idle lanes).
template <class C, int TW>
__device__ void stage_tile(const Coeffs &cf, const typename C::Io &io, TileLds<C, TW> &sm,
                           size_t tbase, int nrow, int ncol, int c0)
{
    const int tid = threadIdx.x;
    const int nx = cf.nx;
    constexpr int PER = kWave * TW / kThreads;  // elements per thread and plane
    double v[C::NIN][PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {  // all loads in flight before any LDS store
        const int e = tid + i * kThreads;
        const int rr = e / TW, cc = e - rr * TW;
        const bool ok = rr < nrow && cc < ncol;
        const size_t g = tbase + (size_t)(ok ? rr : 0) * nx + (ok ? cc : 0);
#pragma unroll
        for (int q = 0; q < C::NIN; ++q) v[q][i] = ok ? io.in[q][g] : 1.0;
    }
#pragma unroll
    for (int i = 0; i < PER; ++i)
#pragma unroll
        for (int q = 0; q < C::NIN; ++q) sm.x[tid + i * kThreads][q] = v[q][i];
    for (int cc = tid; cc < TW; cc += kThreads) {
        const int c = c0 + min(cc, ncol - 1);
        sm.dx[cc] = cf.inv_dx[c];
        sm.src[cc] = cf.src[c];
    }
}

// ---- generic sweep (one wave; SOLVE cell and 128-wide tiles): lane l
// marches row r0+l, column j = s - l at step s.  Branch-free steps: every
// lane evaluates a cell (idle lanes on clamped operands) and commits by
// select.  Returns false if a FAST-sequence operand left its range.
template <class C, int TW, bool FAST>
__device__ bool sweep_tile(const Coeffs &cf, const Engine &eg, TileLds<C, TW> &sm, int t, int cur,
                           int r, int nrow, int ncol, int c0, double we0, double we1)
{
    const int lane = threadIdx.x & (kWave - 1);
    const bool rowok = lane < nrow;
    bool all_ok = true;
    const typename C::Row rw = C::row(cf, r);
    double e0 = we0, e1 = we1;    // running west inflow of my row
    double no0 = 0.0, no1 = 0.0;  // my last north outflow (for lane + 1)
    const int nsteps = ncol + nrow - 1;
    const double(*xr)[C::NIN] = sm.x + lane * TW;
    for (int s = 0; s < nsteps; ++s) {
        const int jn = min(max(s - lane, 0), ncol - 1);
        const typename C::Pre pc =
            C::pre(cf, rw, xr[jn], sm.dx[jn], sm.src[jn], c0 + jn == 0);
        const int sc = min(s, ncol - 1);
        const double n0 = shr1(no0) + (lane == 0 ? sm.sedge[sc][0] : 0.0);
        const double n1 = shr1(no1) + (lane == 0 ? sm.sedge[sc][1] : 0.0);
        const int j = s - lane;
        const bool act = rowok && j >= 0 && j < ncol;
        double oe0, oe1, on0, on1, o0, o1;
        bool ok;
        C::template chain<FAST>(pc, rw, e0, e1, n0, n1, oe0, oe1, on0, on1, o0, o1, ok);
        all_ok = all_ok && (ok || !act);
        e0 = act ? oe0 : e0;
        e1 = act ? oe1 : e1;
        no0 = on0;
        no1 = on1;
        double *d = act ? sm.x[lane * TW + j] : sm.trash[0][lane];
        d[0] = o0;
        d[1] = o1;
        double *tn = act && lane == nrow - 1 ? sm.nout[j] : sm.trash[1][lane];
        tn[0] = on0;
        tn[1] = on1;
    }
    if (rowok) {
        double *ec = eg.eb[cur] + (size_t)t * 2 * kWave;
        ec[lane] = e0;
        ec[kWave + lane] = e1;
    }
    return !__any(!all_ok);
}

// ---- helped sweep (all waves call it): wave 0 runs only the cell chains,
// the DPP hand-over and its commits; waves 1..3 each precompute one diagonal
// of every epoch into the ring, two epochs ahead of the sweep.
template <class C, int TW, bool FAST>
__device__ bool sweep_tile_helped(const Coeffs &cf, const Engine &eg, TileLds<C, TW> &sm, int t,
                                  int cur, int r, int nrow, int ncol, int c0, double we0,
                                  double we1)
{
    constexpr int NF = C::NPRE;
    constexpr int NP = ring_pairs<C>;
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & (kWave - 1);
    const bool rowok = lane < nrow;
    const int nsteps = ncol + nrow - 1;
    const int nep = (nsteps + kEp - 1) / kEp;
    const typename C::Row rw = C::row(cf, r);
    // helper wave w (1..3) fills diagonal w-1 of epoch e
    auto produce = [&](int e) {
        const int i = wave - 1;
        const int d = e * kEp + i;
        const int jn = min(max(d - lane, 0), ncol - 1);
        double f[2 * NP];
        C::pack(C::pre(cf, rw, sm.x[lane * TW + jn], sm.dx[jn], sm.src[jn], c0 + jn == 0),
                *reinterpret_cast<double(*)[NF]>(f));
        const int sc = min(d, ncol - 1);
        f[NF] = lane == 0 ? sm.sedge[sc][0] : 0.0;
        f[NF + 1] = lane == 0 ? sm.sedge[sc][1] : 0.0;
        if constexpr (2 * NP > NF + 2) f[2 * NP - 1] = 0.0;
        double(*slot)[kWave][2] = sm.ring.v[e % kNE][i];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            slot[p][lane][0] = f[2 * p];
            slot[p][lane][1] = f[2 * p + 1];
        }
    };
    if (wave > 0) {
        produce(0);
        if (nep > 1) produce(1);
    }
    bool all_ok = true;
    double e0 = we0, e1 = we1;    // running west inflow of my row
    double no0 = 0.0, no1 = 0.0;  // my last north outflow (for lane + 1)
    // a lane outside the tile rows never sees 0 <= j < ncol
    const int jbase = rowok ? -lane : -(1 << 20);
    double fc[2 * NP];  // ring fields of the current step
#ifdef BURG_STAMPS
    unsigned long long st0 = 0, wait_acc = 0;
#endif
    for (int b = 0; b < nep; ++b) {
#ifdef BURG_STAMPS
        const unsigned long long wa = __builtin_amdgcn_s_memtime();
#endif
        __syncthreads();  // epochs b, b+1 are in the ring; slot (b+2)%kNE is free
#ifdef BURG_STAMPS
        wait_acc += __builtin_amdgcn_s_memtime() - wa;
#endif
        if (wave == 0) {
            const double(*cur_slots)[NP][kWave][2] = sm.ring.v[b % kNE];
            const double(*nxt_slots)[NP][kWave][2] = sm.ring.v[(b + 1) % kNE];
            if (b == 0) {
#ifdef BURG_STAMPS
                st0 = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    fc[2 * p] = cur_slots[0][p][lane][0];
                    fc[2 * p + 1] = cur_slots[0][p][lane][1];
                }
            }
#pragma unroll
            for (int i = 0; i < kEp; ++i) {
                const int s = b * kEp + i;
                // next step's fields first (the next epoch's slot is ready)
                double fn[2 * NP];
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    const double *src = i + 1 < kEp ? cur_slots[i + 1][p][lane]
                                                    : nxt_slots[0][p][lane];
                    fn[2 * p] = src[0];
                    fn[2 * p + 1] = src[1];
                }
                __builtin_amdgcn_sched_barrier(0);
                const typename C::Pre pc = C::unpack(fc);
                // lane l takes the outflow of lane l-1; lane 0 gets +0.0 + its
                // south inflow (exact: x + 0.0 == x)
                const double n0 = shr1(no0) + fc[NF];
                const double n1 = shr1(no1) + fc[NF + 1];
                const int j = s + jbase;
                const bool act = (unsigned)j < (unsigned)ncol;
                double oe0, oe1, on0, on1, o0, o1;
                bool ok;
                C::template chain<FAST>(pc, rw, e0, e1, n0, n1, oe0, oe1, on0, on1, o0, o1, ok);
                all_ok = all_ok && (ok || !act);
                e0 = act ? oe0 : e0;
                e1 = act ? oe1 : e1;
                no0 = on0;  // consumed by lane + 1 only when that lane is active,
                no1 = on1;  // i.e. exactly when this lane was active last step
                double *d = act ? sm.x[lane * TW + j] : sm.trash[0][lane];
                d[0] = o0;
                d[1] = o1;
                double *tn = act && lane == nrow - 1 ? sm.nout[j] : sm.trash[1][lane];
                tn[0] = on0;
                tn[1] = on1;
                // keep the next step's fields in registers (no re-read of LDS)
#pragma unroll
                for (int k = 0; k < 2 * NP; ++k) {
                    asm volatile("" : "+v"(fn[k]));
                    fc[k] = fn[k];
                }
            }
        } else if (b + 2 < nep) {
            produce(b + 2);
        }
    }
    if (wave == 0) {
#ifdef BURG_STAMPS
        const unsigned long long st1 = __builtin_amdgcn_s_memtime();
        if (lane == 0 && t == 0)
            burg_stamp[0] = (long long)(st1 - st0), burg_stamp[1] = nsteps,
            burg_stamp[2] = (long long)wait_acc;
#endif
        if (rowok) {
            double *ec = eg.eb[cur] + (size_t)t * 2 * kWave;
            ec[lane] = e0;
            ec[kWave + lane] = e1;
        }
    }
    return !__any(!all_ok);
}

// ---------------------------------------------------------------------------
// One tile, one pass, one workgroup.  Wave 0 gathers the inflow and decides
// whether the tile must be marched; all waves stage the tile into LDS and
// write the outputs back coalesced.  Returns true (workgroup-uniform) if the
// tile was marched.  Generation `cur` of the edge planes receives its outflow
// (marched or carried), generation `prv` holds the neighbours' outflow of the
// previous pass.
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

    // ---- stage the tile's inputs
    const size_t tbase = (size_t)r0 * nx + c0;
    stage_tile<C, TW>(cf, io, sm, tbase, nrow, ncol, c0);
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
            sm.sedge[col][0] = sn0[q];
            sm.sedge[col][1] = sn1[q];
        }
    }
    __syncthreads();

    // ---- the sweep with the short exact sequences; if an operand left their
    // range, restage and sweep again with the IEEE operators
    bool ok = true;
    if constexpr (helped_v<C, TW>) {
        ok = sweep_tile_helped<C, TW, true>(cf, eg, sm, t, cur, r, nrow, ncol, c0, we0, we1);
    } else {
        if (wave == 0)
            ok = sweep_tile<C, TW, true>(cf, eg, sm, t, cur, r, nrow, ncol, c0, we0, we1);
    }
    __syncthreads();
    if (wave == 0 && lane == 0) sm.need = ok;
    __syncthreads();
    if (!sm.need) {
        stage_tile<C, TW>(cf, io, sm, tbase, nrow, ncol, c0);
        __syncthreads();
        if (wave == 0) sweep_tile<C, TW, false>(cf, eg, sm, t, cur, r, nrow, ncol, c0, we0, we1);
    }
    __syncthreads();
    {
        double *nout = eg.nb[cur] + (size_t)t * 2 * TW;
        for (int cc = tid; cc < ncol; cc += kThreads) {
            nout[cc] = sm.nout[cc][0];
            nout[TW + cc] = sm.nout[cc][1];
        }
    }

    // ---- write the outputs back, coalesced
    for (int e = tid; e < kWave * TW; e += kThreads) {
        const int rr = e / TW, cc = e - rr * TW;
        if (rr < nrow && cc < ncol) {
            const size_t g = tbase + (size_t)rr * nx + cc;
            io.out[0][g] = sm.x[e][0];
            io.out[1][g] = sm.x[e][1];
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
    } else if constexpr (C::NIN * 128 * kWave * 8 <= 150 * 1024) {
        if (eg.tw != 128) return -1;
        if (final)
            final_kernel<C, 128><<<grid, block, 0, st>>>(cf, eg, io, pass, stats);
        else
            pass_kernel<C, 128><<<grid, block, 0, st>>>(cf, eg, io, pass);
    } else {
        return -1;  // LDS budget: the 4-input SOLVE cell needs tile_w = 64
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
