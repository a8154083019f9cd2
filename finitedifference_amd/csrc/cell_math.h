// cell_math.h -- the MARCH cell (closed-form implicit step of one cell) and
// the exact short fp64 sequences it uses; shared by the tile engine
// (march.hip) and the streaming engine (stream.hip).  Op order is normative:
// oracle/burgers_oracle.c (orc_march_step) restates it.
#pragma once

#include "burg_internal.h"

namespace burg {
namespace {

// lane i <- lane i-1 over the whole wave (DPP wave_shr:1); lane 0 gets +0.0
// (bound_ctrl).  Must run with every lane enabled: a DPP read from a
// disabled lane does not return that lane's register.
__device__ __forceinline__ double shr1(double x)
{
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), 0x138, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}

// Correctly rounded sqrt(q) for normal q, without the denormal/special-case
// range scaling of the compiler's expansion: the same v_rsq_f64 seed,
// Goldschmidt step and two Newton corrections (gfx950 ISA as emitted for
// sqrt()), hence bit-identical to IEEE sqrt on [2^-900, 2^900) (a negative
// q gives NaN, as sqrt does).
__device__ __forceinline__ double sqrt_normal(double q)
{
    const double y = __builtin_amdgcn_rsq(q);
    double g = q * y;
    double h = y * 0.5;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    double d = fma(-g, g, q);
    g = fma(d, h, g);
    d = fma(-g, g, q);
    return fma(d, h, g);
}

// a0/b and a1/b correctly rounded, sharing the reciprocal refinement: the
// compiler's division expansion (v_rcp_f64 seed, two Newton steps, one
// Markstein correction) without v_div_scale/fmas/fixup, which are identities
// for normal operands (b in [1, 2^900], a = 0 or |a| >= 2^-900).
__device__ __forceinline__ void div2_normal(double a0, double a1, double b, double &q0,
                                            double &q1)
{
    double r = __builtin_amdgcn_rcp(b);
    double e = fma(-b, r, 1.0);
    r = fma(r, e, r);
    e = fma(-b, r, 1.0);
    r = fma(r, e, r);
    const double t0 = a0 * r, t1 = a1 * r;
    const double m0 = fma(-b, t0, a0), m1 = fma(-b, t1, a1);
    q0 = fma(m0, r, t0);
    q1 = fma(m1, r, t1);
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
    // Inflow-independent part of a cell.
    struct Pre {
        double hx, xfp, xhp, yhp, ygp, bu, bv;
    };
    static constexpr int NPRE = 7;  // Pre fields as staged in the helper ring
    __device__ static void pack(const Pre &p, double (&f)[NPRE])
    {
        f[0] = p.hx, f[1] = p.xfp, f[2] = p.xhp, f[3] = p.yhp;
        f[4] = p.ygp, f[5] = p.bu, f[6] = p.bv;
    }
    __device__ static Pre unpack(const double *f)
    {
        return Pre{f[0], f[1], f[2], f[3], f[4], f[5], f[6]};
    }
    __device__ static Pre pre(const Coeffs &cf, const Row &rw, const double *x, double invdx,
                              double srcc, bool col0)
    {
        Pre p;
        const double pu = x[0], pv = x[1];
        const double ax = cf.alpha * invdx;
        p.hx = 0.5 * ax;
        const double sl = col0 ? srcc + rw.lb : srcc;
        const double hu = 0.5 * pu;
        p.xfp = ax * (hu * pu);
        p.xhp = ax * (hu * pv);
        p.yhp = rw.ay * (hu * pv);
        p.ygp = rw.ay * ((0.5 * pv) * pv);
        p.bu = ((pu - p.xfp) - p.yhp) + sl;
        p.bv = (pv - p.ygp) - p.xhp;
        return p;
    }
    // The cell's critical path: west (e0=XF, e1=XH) and south (n0=YH, n1=YG)
    // inflow -> state (o0, o1) and this cell's outflow.  FAST: the short exact
    // sequences (range_ok false if an operand is outside their range);
    // !FAST: the compiler's IEEE sqrt and division.
    template <bool FAST>
    __device__ static void chain(const Pre &p, const Row &rw, double e0, double e1, double n0,
                                 double n1, double &oe0, double &oe1, double &on0, double &on1,
                                 double &o0, double &o1, bool &range_ok)
    {
        const double cu = (p.bu + e0) + n0;
        const double cv = (p.bv + n1) + e1;
        const double mm = fma(p.hx, cu, rw.hy * cv);
        const double q = 0.25 + mm;
        double s, nu, nv;
        if constexpr (FAST) {
            // The fast window: Cu, Cv POSITIVE with magnitude in [2^-900,
            // 2^798), inside div2_normal's exact range.  Then q = 0.25 + h_x Cu
            // + h_y Cv is >= 0.25 (h_x, h_y > 0) and below 0.25 + 2^100 2^798
            // 2 < 2^900 (h_x, h_y < 2^100, checked by burg_set_problem), i.e.
            // inside sqrt_normal's exact range [2^-900, 2^900), and s = 0.5 +
            // sqrt(q) is in [1, 2^450]: no test of q is needed (round 4: the
            // window's top was 2^900, which let q reach 2^1001 for h near
            // 2^100 -- outside the range the sequences are verified on).
            // Tested on the high words: less 123 << 20, a positive operand's
            // word is below 1698 << 20 iff its biased exponent is in [123,
            // 1820] (a smaller one borrows past the top, a negative one has
            // the top bit set).  Zeros, negatives, denormals, Inf, NaN and
            // operands >= 2^798 take the IEEE path (which reports a NaN): the
            // reference regime's velocities are positive and O(1), and a
            // negative Cu / Cv is still computed exactly.  Two subtracts, a
            // max and a compare.
            const unsigned xu = (unsigned)__double2hiint(cu) - (123u << 20);
            const unsigned xv = (unsigned)__double2hiint(cv) - (123u << 20);
#ifdef BURG_AB_NOCHECK
            range_ok = true;  // (A/B probes only: the fast path for every operand -- wrong in general)
            (void)xu, (void)xv;
#else
            range_ok = max(xu, xv) < (1698u << 20);
#endif
            s = 0.5 + sqrt_normal(q);
            div2_normal(cu, cv, s, nu, nv);
        } else {
            range_ok = true;
            s = 0.5 + sqrt(q);
            nu = cu / s;
            nv = cv / s;
        }
        const double hxu = p.hx * nu;
        oe0 = fma(hxu, nu, p.xfp);
        oe1 = fma(hxu, nv, p.xhp);
        on0 = fma(rw.hy * nu, nv, p.yhp);
        on1 = fma(rw.hy * nv, nv, p.ygp);
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


}  // namespace
}  // namespace burg
