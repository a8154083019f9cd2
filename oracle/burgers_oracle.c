/*
 * burgers_oracle.c -- CPU restatement of the reference FOM hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: it may be
 * loaded only by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.  The product path (finitedifference_amd) never links,
 * imports or calls it and fails loudly if its HIP library is missing.
 *
 * Parity pinning: the restatement is checked against golden vectors made by
 * importing the Python reference in the build container
 * (tests/golden/make_golden.py) and against the author's pickled HDM slices
 * and SLURM Newton logs (tests/test_oracle_golden.py).
 *
 * Reference being restated (paths relative to /root/reference,
 * C/ = BurgersFD_CleanCoarse/):
 *   residual        C/hypernet2D.py:2512-2570  inviscid_burgers_res2D_alt
 *   Jacobian        C/hypernet2D.py:2627-2656  inviscid_burgers_exact_jac2D
 *   operators       C/hypernet2D.py:2410-2416  make_ddx (backward difference,
 *                   spdiags([-1/dx, 1/dx], [-1, 0])), :98-106 JDxec/JDyec
 *   Newton          C/hypernet2D.py:1811-1857  newton_raphson
 *   linear solve    C/hypernet2D.py:1854       scipy.sparse.linalg.spsolve
 *                   (SuperLU; third-party).  Restated as the exact 2x2-block
 *                   forward substitution: in cell-interleaved order the
 *                   Jacobian is block lower-triangular,
 *                   so LU of it has no fill and equals this sweep.
 *   time loop       C/hypernet2D.py:72-131     inviscid_burgers_implicit2D
 *
 * Layout (reference): w = [u.ravel(), v.ravel()], u row-major (ny, nx),
 * cell (r, c) at r*nx + c, v block offset n = nx*ny (C/run_fom.py:33-35).
 *
 * Host-side coefficient vectors are computed in Python exactly as NumPy does
 * in the reference and passed in:
 *   inv_dx[c] = 1/dx_c,  inv_dy[r] = 1/dy_r         (make_ddx, :2414)
 *   src[c]    = dt*0.02*exp(mu2*xc_c)               (:2550)
 *   lbc[r]    = 0.5*dt*mu1**2/dx[r]  (row-indexed quirk of :2553-2554)
 *
 * The closed-form march (orc_march_step) is NOT a reference function: it is
 * the build's own exact solver for the same implicit step
 * and is restated here op-for-op as the bitwise checker of the HIP march.
 */
#define _POSIX_C_SOURCE 200809L
#include <math.h>
#include <sched.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define IDX(r, c, nx) ((size_t)(r) * (size_t)(nx) + (size_t)(c))

/* ------------------------------------------------------------------------ */
/* Residual: mirror of inviscid_burgers_res2D_alt (C/hypernet2D.py:2512-2570),
 * keeping NumPy's operation order:
 *   ru = u - up + (a*JDx)@(Fu+Fpu) + (a*JDy)@(Fuv+Fpuv) - src ; ru -= lbc
 *   rv = v - vp + (a*JDy)@(Fv+Fpv) + a*(JDx@(Fuv+Fpuv))
 * with a = 0.5*dt.  A sparse row holds two entries, so the matvec sum is
 * order-independent: (D f)_i = k_i f_i - k_{i-1} f_{i-1}.                    */
void orc_residual(int nx, int ny, const double *inv_dx, const double *inv_dy,
                  const double *src, const double *lbc, double dt,
                  const double *w, const double *wp, double *res)
{
    const size_t n = (size_t)nx * ny;
    const double a = 0.5 * dt;
    const double *u = w, *v = w + n, *up = wp, *vp = wp + n;
    for (int r = 0; r < ny; ++r) {
        const double ay = a * inv_dy[r];
        const double ays = r > 0 ? a * inv_dy[r - 1] : 0.0;
        for (int c = 0; c < nx; ++c) {
            const size_t i = IDX(r, c, nx);
            const double ax = a * inv_dx[c];
            /* fluxes at this cell */
            const double Su = 0.5 * (u[i] * u[i]) + 0.5 * (up[i] * up[i]);
            const double Sv = 0.5 * (v[i] * v[i]) + 0.5 * (vp[i] * vp[i]);
            const double Suv = (0.5 * u[i]) * v[i] + (0.5 * up[i]) * vp[i];
            double dxu = ax * Su, dyuv = ay * Suv, dyv = ay * Sv, dxuv = inv_dx[c] * Suv;
            if (c > 0) {
                const size_t j = i - 1;
                const double axw = a * inv_dx[c - 1];
                const double SuW = 0.5 * (u[j] * u[j]) + 0.5 * (up[j] * up[j]);
                const double SuvW = (0.5 * u[j]) * v[j] + (0.5 * up[j]) * vp[j];
                dxu = dxu + (-axw) * SuW;
                dxuv = dxuv + (-inv_dx[c - 1]) * SuvW;
            }
            if (r > 0) {
                const size_t j = i - (size_t)nx;
                const double SvS = 0.5 * (v[j] * v[j]) + 0.5 * (vp[j] * vp[j]);
                const double SuvS = (0.5 * u[j]) * v[j] + (0.5 * up[j]) * vp[j];
                dyuv = dyuv + (-ays) * SuvS;
                dyv = dyv + (-ays) * SvS;
            }
            double ru = u[i] - up[i];
            ru = ru + dxu;
            ru = ru + dyuv;
            ru = ru - src[c];
            ru = ru - (c == 0 ? lbc[r] : 0.0);
            double rv = v[i] - vp[i];
            rv = rv + dyv;
            rv = rv + a * dxuv;
            res[i] = ru;
            res[n + i] = rv;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* Jacobian-vector product: J(w) x with J from inviscid_burgers_exact_jac2D
 * (C/hypernet2D.py:2627-2656):
 *   J = I + [[JDx D(au) + 0.5 JDy D(av), 0.5 JDy D(au)],
 *            [0.5 JDx D(av),            JDy D(av) + 0.5 JDx D(au)]]
 * Matrix-free, per cell with the linearised fluxes
 *   XFd = ax u xu,  XHd = 0.5 ax (v xu + u xv),
 *   YHd = 0.5 ay (v xu + u xv),  YGd = ay v xv,
 *   (Jx)_u = xu + XFd - XFd_W + YHd - YHd_S,
 *   (Jx)_v = xv + YGd - YGd_S + XHd - XHd_W.                                  */
void orc_jvp(int nx, int ny, const double *inv_dx, const double *inv_dy, double dt,
             const double *w, const double *x, double *y)
{
    const size_t n = (size_t)nx * ny;
    const double a = 0.5 * dt;
    const double *u = w, *v = w + n, *xu = x, *xv = x + n;
    for (int r = 0; r < ny; ++r) {
        for (int c = 0; c < nx; ++c) {
            const size_t i = IDX(r, c, nx);
            const double ax = a * inv_dx[c], ay = a * inv_dy[r];
            const double m = v[i] * xu[i] + u[i] * xv[i];
            double yu = xu[i] + ax * u[i] * xu[i] + 0.5 * ay * m;
            double yv = xv[i] + ay * v[i] * xv[i] + 0.5 * ax * m;
            if (c > 0) {
                const size_t j = i - 1;
                const double axw = a * inv_dx[c - 1];
                const double mW = v[j] * xu[j] + u[j] * xv[j];
                yu -= axw * u[j] * xu[j];
                yv -= 0.5 * axw * mW;
            }
            if (r > 0) {
                const size_t j = i - (size_t)nx;
                const double ays = a * inv_dy[r - 1];
                const double mS = v[j] * xu[j] + u[j] * xv[j];
                yu -= 0.5 * ays * mS;
                yv -= ays * v[j] * xv[j];
            }
            y[i] = yu;
            y[n + i] = yv;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* Exact solve J(w) delta = rhs: 2x2-block forward substitution in
 * lexicographic (r, c) order.  Replaces spsolve (C/hypernet2D.py:1854); the
 * Jacobian is block lower-triangular in cell order, so this is the LU solve
 * with zero fill.                                                            */
void orc_block_solve(int nx, int ny, const double *inv_dx, const double *inv_dy,
                     double dt, const double *w, const double *rhs, double *delta)
{
    const size_t n = (size_t)nx * ny;
    const double a = 0.5 * dt;
    const double *u = w, *v = w + n;
    double *du = delta, *dv = delta + n;
    for (int r = 0; r < ny; ++r) {
        for (int c = 0; c < nx; ++c) {
            const size_t i = IDX(r, c, nx);
            const double ax = a * inv_dx[c], ay = a * inv_dy[r];
            double eu = rhs[i], ev = rhs[n + i];
            if (c > 0) {
                const size_t j = i - 1;
                const double axw = a * inv_dx[c - 1];
                eu += axw * u[j] * du[j];
                ev += 0.5 * axw * (v[j] * du[j] + u[j] * dv[j]);
            }
            if (r > 0) {
                const size_t j = i - (size_t)nx;
                const double ays = a * inv_dy[r - 1];
                eu += 0.5 * ays * (v[j] * du[j] + u[j] * dv[j]);
                ev += ays * v[j] * dv[j];
            }
            const double a00 = 1.0 + ax * u[i] + 0.5 * ay * v[i];
            const double a01 = 0.5 * ay * u[i];
            const double a10 = 0.5 * ax * v[i];
            const double a11 = 1.0 + ay * v[i] + 0.5 * ax * u[i];
            const double det = a00 * a11 - a01 * a10;
            du[i] = (a11 * eu - a01 * ev) / det;
            dv[i] = (a00 * ev - a10 * eu) / det;
        }
    }
}

static double norm2(const double *x, size_t m)
{
    double s = 0.0;
    for (size_t i = 0; i < m; ++i) s += x[i] * x[i];
    return sqrt(s);
}

/* ------------------------------------------------------------------------ */
/* One implicit step by newton_raphson (C/hypernet2D.py:1811-1857):
 *   x = x0; init = ||R(x0)||; for i < max_its: rn = ||R(x)||;
 *   if rn/init < cutoff: break; x -= J(x)^{-1} R(x).
 * Returns the number of updates taken (the printed "i"); *final_rel gets the
 * last rn/init.  w_out may alias nothing; scratch is allocated here.         */
int orc_newton_step(int nx, int ny, const double *inv_dx, const double *inv_dy,
                    const double *src, const double *lbc, double dt,
                    const double *wp, double *w_out, int max_its, double cutoff,
                    double *final_rel)
{
    const size_t m = 2 * (size_t)nx * ny;
    double *res = (double *)malloc(m * sizeof(double));
    double *del = (double *)malloc(m * sizeof(double));
    memcpy(w_out, wp, m * sizeof(double));
    orc_residual(nx, ny, inv_dx, inv_dy, src, lbc, dt, wp, wp, res);
    const double init = norm2(res, m);
    int it = 0;
    double rel = NAN;
    for (it = 0; it < max_its; ++it) {
        orc_residual(nx, ny, inv_dx, inv_dy, src, lbc, dt, w_out, wp, res);
        rel = norm2(res, m) / init;
        if (rel < cutoff) break;
        orc_block_solve(nx, ny, inv_dx, inv_dy, dt, w_out, res, del);
        for (size_t i = 0; i < m; ++i) w_out[i] -= del[i];
    }
    if (final_rel) *final_rel = rel;
    free(res);
    free(del);
    return it;
}

/* ------------------------------------------------------------------------ */
/* Closed-form march (build's own exact solver; DESIGN.md section 3 "MARCH SPEC").
 * The implicit residual is lower-triangular in (r, c) and each cell's 2x2
 * system is u*s = Cu, v*s = Cv with the common factor s = 1 + hx u + hy v,
 * so s = 0.5 + sqrt(0.25 + hx Cu + hy Cv), u = Cu/s, v = Cv/s (IEEE sqrt and
 * division).  Op order is normative: the HIP march reproduces it bit for bit. */
void orc_march_step(int nx, int ny, const double *inv_dx, const double *inv_dy,
                    const double *src, const double *lbc, double dt,
                    const double *wp, double *w)
{
    const size_t n = (size_t)nx * ny;
    const double a = 0.5 * dt;
    const double *up = wp, *vp = wp + n;
    double *u = w, *v = w + n;
    /* outflows of the row below (YH, YG) and of the west cell (XF, XH) */
    double *yh = (double *)calloc((size_t)nx, sizeof(double));
    double *yg = (double *)calloc((size_t)nx, sizeof(double));
    for (int r = 0; r < ny; ++r) {
        const double ay = a * inv_dy[r];
        const double hy = 0.5 * ay;
        double xfw = 0.0, xhw = 0.0;
        for (int c = 0; c < nx; ++c) {
            const size_t i = IDX(r, c, nx);
            const double ax = a * inv_dx[c];
            const double hx = 0.5 * ax;
            const double sl = c == 0 ? src[0] + lbc[r] : src[c];
            const double pu = up[i], pv = vp[i];
            const double hu = 0.5 * pu;
            const double xfp = ax * (hu * pu);
            const double xhp = ax * (hu * pv);
            const double yhp = ay * (hu * pv);
            const double ygp = ay * ((0.5 * pv) * pv);
            const double bu = ((pu - xfp) - yhp) + sl;
            const double bv = (pv - ygp) - xhp;
            const double cu = (bu + xfw) + yh[c];
            const double cv = (bv + yg[c]) + xhw;
            const double mm = fma(hx, cu, hy * cv);
            const double s = 0.5 + sqrt(0.25 + mm);
            const double nu = cu / s, nv = cv / s;
            const double hxu = hx * nu;
            xfw = fma(hxu, nu, xfp);
            xhw = fma(hxu, nv, xhp);
            yh[c] = fma(hy * nu, nv, yhp);
            yg[c] = fma(hy * nv, nv, ygp);
            u[i] = nu;
            v[i] = nv;
        }
    }
    free(yh);
    free(yg);
}

/* ------------------------------------------------------------------------ */
/* CPU baseline (bench.py's cpu_baseline leg, not a parity checker): the
 * reference's snapshot generation over a mu set (C/run_prom.py:59-71 calls
 * load_or_compute_snaps once per mu) with the march above, one trajectory per
 * OpenMP thread -- the independent work the reference leaves on the table.
 * src_b[j*nx + c], lbc_b[j*ny + r]: trajectory j's coefficients; every
 * trajectory starts from w0 and runs num_steps steps (states ping-ponged, not
 * kept).  Returns the threads used.                                          */
int orc_march_sweep(int nx, int ny, const double *inv_dx, const double *inv_dy,
                    const double *src_b, const double *lbc_b, double dt, const double *w0,
                    int nmu, int num_steps, int threads)
{
    const size_t m = 2 * (size_t)nx * ny;
    int used = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
    for (int j = 0; j < nmu; ++j) {
#ifdef _OPENMP
        if (j == 0) used = omp_get_num_threads();
#endif
        double *a = (double *)malloc(m * sizeof(double));
        double *b = (double *)malloc(m * sizeof(double));
        memcpy(a, w0, m * sizeof(double));
        for (int i = 0; i < num_steps; ++i) {
            orc_march_step(nx, ny, inv_dx, inv_dy, src_b + (size_t)j * nx, lbc_b + (size_t)j * ny,
                           dt, a, b);
            double *t = a;
            a = b;
            b = t;
        }
        free(a);
        free(b);
    }
    return used;
}

/* ------------------------------------------------------------------------ */
/* The same march, rows pipelined over OpenMP threads (test support: the
 * checker for whole trajectories at the bench's sizes, 4096^2 x 500 steps,
 * where the serial step takes minutes).  Not a new algorithm: every cell runs
 * the loop body of orc_march_step with the same operands in the same order,
 * so the result is orc_march_step's bit for bit.  Row r's thread marches
 * columns [c0, c0 + 64) once row r-1 has published that it is past c0 + 64;
 * the north outflows live in one in-place array exactly as in the serial
 * version (row r overwrites yh[c] after reading it, row r+1 reads it after
 * row r's publish).  prog[r] = s*(nx+1) + columns done in step s (monotone,
 * never reset).  out: (num_steps/snap_every + 1) x 2n step-major (state after
 * j*snap_every steps in row j).  Returns the threads used.                   */
#define ORC_PAR_BLK 64
int orc_march_traj_par(int nx, int ny, const double *inv_dx, const double *inv_dy,
                       const double *src, const double *lbc, double dt, const double *w0,
                       int num_steps, int snap_every, double *out, int threads)
{
    const size_t n = (size_t)nx * ny, m = 2 * n;
    const double a = 0.5 * dt;
    double *A = (double *)malloc(m * sizeof(double));
    double *B = (double *)malloc(m * sizeof(double));
    double *yh = (double *)calloc((size_t)nx, sizeof(double));
    double *yg = (double *)calloc((size_t)nx, sizeof(double));
    int64_t *prog = (int64_t *)calloc((size_t)ny, sizeof(int64_t));
    memcpy(A, w0, m * sizeof(double));
    memcpy(out, w0, m * sizeof(double));
    int used = 1;
#pragma omp parallel num_threads(threads)
    {
        int t = 0, T = 1;
#ifdef _OPENMP
        t = omp_get_thread_num();
        T = omp_get_num_threads();
#endif
        if (t == 0) used = T;
        for (int s = 0; s < num_steps; ++s) {
            const double *up = (s & 1) ? B : A, *vp = up + n;
            double *u = (s & 1) ? A : B, *v = u + n;
            const int keep = (s + 1) % snap_every == 0;
            double *o = out + (size_t)((s + 1) / snap_every) * m;
            const int64_t base = (int64_t)s * (nx + 1);
            for (int r = t; r < ny; r += T) {
                const double ay = a * inv_dy[r];
                const double hy = 0.5 * ay;
                double xfw = 0.0, xhw = 0.0;
                for (int c0 = 0; c0 < nx; c0 += ORC_PAR_BLK) {
                    const int c1 = c0 + ORC_PAR_BLK < nx ? c0 + ORC_PAR_BLK : nx;
                    if (r > 0) {
                        unsigned spins = 0;
                        while (__atomic_load_n(&prog[r - 1], __ATOMIC_ACQUIRE) < base + c1)
                            if (++spins > 4096u) {
                                sched_yield();
                                spins = 0;
                            }
                    }
                    for (int c = c0; c < c1; ++c) {
                        const size_t i = IDX(r, c, nx);
                        const double ax = a * inv_dx[c];
                        const double hx = 0.5 * ax;
                        const double sl = c == 0 ? src[0] + lbc[r] : src[c];
                        const double pu = up[i], pv = vp[i];
                        const double hu = 0.5 * pu;
                        const double xfp = ax * (hu * pu);
                        const double xhp = ax * (hu * pv);
                        const double yhp = ay * (hu * pv);
                        const double ygp = ay * ((0.5 * pv) * pv);
                        const double bu = ((pu - xfp) - yhp) + sl;
                        const double bv = (pv - ygp) - xhp;
                        const double yin = r == 0 ? 0.0 : yh[c], gin = r == 0 ? 0.0 : yg[c];
                        const double cu = (bu + xfw) + yin;
                        const double cv = (bv + gin) + xhw;
                        const double mm = fma(hx, cu, hy * cv);
                        const double sq = 0.5 + sqrt(0.25 + mm);
                        const double nu = cu / sq, nv = cv / sq;
                        const double hxu = hx * nu;
                        xfw = fma(hxu, nu, xfp);
                        xhw = fma(hxu, nv, xhp);
                        yh[c] = fma(hy * nu, nv, yhp);
                        yg[c] = fma(hy * nv, nv, ygp);
                        u[i] = nu;
                        v[i] = nv;
                    }
                    __atomic_store_n(&prog[r], base + c1, __ATOMIC_RELEASE);
                }
                if (keep) {
                    memcpy(o + IDX(r, 0, nx), u + IDX(r, 0, nx), (size_t)nx * sizeof(double));
                    memcpy(o + n + IDX(r, 0, nx), v + IDX(r, 0, nx), (size_t)nx * sizeof(double));
                }
            }
#pragma omp barrier
        }
    }
    free(A);
    free(B);
    free(yh);
    free(yg);
    free(prog);
    return used;
}

/* ------------------------------------------------------------------------ */
/* Time loop (C/hypernet2D.py:72-131).  snaps is step-major:
 * (num_steps+1) x 2n, row j = state after j steps.  solver 0 = newton (the
 * reference algorithm), 1 = closed-form march.  newton_its[i] (may be NULL)
 * receives the Newton update count of step i.                                */
int orc_fom(int nx, int ny, const double *inv_dx, const double *inv_dy,
            const double *src, const double *lbc, double dt, const double *w0,
            int num_steps, int solver, int max_its, double cutoff,
            double *snaps, int *newton_its, double *final_rel)
{
    const size_t m = 2 * (size_t)nx * ny;
    memcpy(snaps, w0, m * sizeof(double));
    for (int i = 0; i < num_steps; ++i) {
        const double *wp = snaps + (size_t)i * m;
        double *w = snaps + (size_t)(i + 1) * m;
        if (solver == 0) {
            double rel = 0.0;
            int its = orc_newton_step(nx, ny, inv_dx, inv_dy, src, lbc, dt, wp, w,
                                      max_its, cutoff, &rel);
            if (newton_its) newton_its[i] = its;
            if (final_rel) final_rel[i] = rel;
        } else {
            orc_march_step(nx, ny, inv_dx, inv_dy, src, lbc, dt, wp, w);
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Schedule simulator for the HIP tile engine (test support, not a reference
 * restatement).  The grid is cut into th x tw tiles that are all marched in
 * parallel per iteration (block Jacobi over tiles).  Iteration 1 guesses each
 * interior tile inflow from wp ("the neighbour did not move"); iteration k>1
 * re-marches a tile only if one of its inflow values moved by more than
 * tol*|value| away from the inflow the tile last used.  Stops when no tile
 * was re-marched.  tol = 0 demands the bitwise fixed point, which equals the
 * sequential march but needs O(#tile rows) iterations in y-uniform regions
 * (1-ulp fixed points of the rounded recurrence); a few ulps suffice for
 * the iteration to stop after 2-4 passes.
 * Returns iterations run; *tiles_done = tiles marched.                      */
typedef struct {
    const double *inv_dx, *inv_dy, *src, *lbc;
    double a;
    int nx, ny;
} orc_grid;

static inline void cell_pre(const orc_grid *g, int r, int c, double pu, double pv,
                            double *bu, double *bv, double *xfp, double *xhp,
                            double *yhp, double *ygp)
{
    const double ax = g->a * g->inv_dx[c], ay = g->a * g->inv_dy[r];
    const double sl = c == 0 ? g->src[0] + g->lbc[r] : g->src[c];
    const double hu = 0.5 * pu;
    *xfp = ax * (hu * pu);
    *xhp = ax * (hu * pv);
    *yhp = ay * (hu * pv);
    *ygp = ay * ((0.5 * pv) * pv);
    *bu = ((pu - *xfp) - *yhp) + sl;
    *bv = (pv - *ygp) - *xhp;
}

static inline int moved(double a, double b, double tol)
{
    const double d = fabs(a - b), m = fmax(fabs(a), fabs(b));
    return tol == 0.0 ? a != b : d > tol * m;
}

int orc_march_tiled_sim(int nx, int ny, const double *inv_dx, const double *inv_dy,
                        const double *src, const double *lbc, double dt,
                        const double *wp, double *w, int th, int tw, int kmax,
                        double tol, long long *tiles_done)
{
    const size_t n = (size_t)nx * ny;
    const int nti = (ny + th - 1) / th, ntj = (nx + tw - 1) / tw;
    const size_t nt = (size_t)nti * ntj;
    orc_grid g = {inv_dx, inv_dy, src, lbc, 0.5 * dt, nx, ny};
    /* current outflow edges: E (xf, xh) per tile row, N (yh, yg) per tile column;
     * used inflows: W (xf, xh) and S (yh, yg) as last marched with            */
    double *E = (double *)calloc(nt * 2 * th, sizeof(double));
    double *Nn = (double *)calloc(nt * 2 * tw, sizeof(double));
    double *E2 = (double *)calloc(nt * 2 * th, sizeof(double));
    double *N2 = (double *)calloc(nt * 2 * tw, sizeof(double));
    double *Wu = (double *)calloc(nt * 2 * th, sizeof(double));
    double *Su = (double *)calloc(nt * 2 * tw, sizeof(double));
    double *yh = (double *)malloc(tw * sizeof(double)), *yg = (double *)malloc(tw * sizeof(double));
    double *win = (double *)malloc(2 * th * sizeof(double)), *sin_ = (double *)malloc(2 * tw * sizeof(double));
    long long done = 0;
    int k;
    for (k = 1; k <= kmax; ++k) {
        int any = 0;
        memcpy(E2, E, nt * 2 * th * sizeof(double));
        memcpy(N2, Nn, nt * 2 * tw * sizeof(double));
        for (int I = 0; I < nti; ++I)
            for (int J = 0; J < ntj; ++J) {
                const size_t t = (size_t)I * ntj + J;
                const int r0 = I * th, c0 = J * tw;
                const int r1 = r0 + th < ny ? r0 + th : ny, c1 = c0 + tw < nx ? c0 + tw : nx;
                /* gather inflow */
                for (int c = c0; c < c1; ++c) {
                    double sh = 0.0, sg = 0.0;
                    if (I > 0) {
                        if (k == 1) {
                            double bu, bv, xfp, xhp, yhp, ygp;
                            const size_t i = IDX(r0 - 1, c, nx);
                            const double pu = wp[i], pv = wp[n + i];
                            cell_pre(&g, r0 - 1, c, pu, pv, &bu, &bv, &xfp, &xhp, &yhp, &ygp);
                            const double hy = 0.5 * (g.a * inv_dy[r0 - 1]);
                            sh = fma(hy * pu, pv, yhp);
                            sg = fma(hy * pv, pv, ygp);
                        } else {
                            const double *sn = N2 + (t - ntj) * 2 * tw;
                            sh = sn[c - c0];
                            sg = sn[tw + c - c0];
                        }
                    }
                    sin_[c - c0] = sh;
                    sin_[tw + c - c0] = sg;
                }
                for (int r = r0; r < r1; ++r) {
                    double xf = 0.0, xh = 0.0;
                    if (J > 0) {
                        if (k == 1) {
                            double bu, bv, xfp, xhp, yhp, ygp;
                            const size_t i = IDX(r, c0 - 1, nx);
                            const double pu = wp[i], pv = wp[n + i];
                            cell_pre(&g, r, c0 - 1, pu, pv, &bu, &bv, &xfp, &xhp, &yhp, &ygp);
                            const double hx = 0.5 * (g.a * inv_dx[c0 - 1]);
                            xf = fma(hx * pu, pu, xfp);
                            xh = fma(hx * pu, pv, xhp);
                        } else {
                            const double *se = E2 + (t - 1) * 2 * th;
                            xf = se[r - r0];
                            xh = se[th + r - r0];
                        }
                    }
                    win[r - r0] = xf;
                    win[th + r - r0] = xh;
                }
                int need = (k == 1);
                if (!need) {
                    double *wu = Wu + t * 2 * th, *su = Su + t * 2 * tw;
                    for (int r = 0; r < r1 - r0 && !need; ++r)
                        need = moved(win[r], wu[r], tol) || moved(win[th + r], wu[th + r], tol);
                    for (int c = 0; c < c1 - c0 && !need; ++c)
                        need = moved(sin_[c], su[c], tol) || moved(sin_[tw + c], su[tw + c], tol);
                }
                if (!need) continue;
                any = 1;
                ++done;
                memcpy(Wu + t * 2 * th, win, 2 * th * sizeof(double));
                memcpy(Su + t * 2 * tw, sin_, 2 * tw * sizeof(double));
                for (int c = c0; c < c1; ++c) {
                    yh[c - c0] = sin_[c - c0];
                    yg[c - c0] = sin_[tw + c - c0];
                }
                double *eo = E + t * 2 * th, *no = Nn + t * 2 * tw;
                for (int r = r0; r < r1; ++r) {
                    double xfw = win[r - r0], xhw = win[th + r - r0];
                    const double ay = g.a * inv_dy[r], hy = 0.5 * ay;
                    for (int c = c0; c < c1; ++c) {
                        const size_t i = IDX(r, c, nx);
                        const double hx = 0.5 * (g.a * inv_dx[c]);
                        double bu, bv, xfp, xhp, yhp, ygp;
                        cell_pre(&g, r, c, wp[i], wp[n + i], &bu, &bv, &xfp, &xhp, &yhp, &ygp);
                        const double cu = (bu + xfw) + yh[c - c0];
                        const double cv = (bv + yg[c - c0]) + xhw;
                        const double mm = fma(hx, cu, hy * cv);
                        const double s = 0.5 + sqrt(0.25 + mm);
                        const double nu = cu / s, nv = cv / s;
                        const double hxu = hx * nu;
                        xfw = fma(hxu, nu, xfp);
                        xhw = fma(hxu, nv, xhp);
                        yh[c - c0] = fma(hy * nu, nv, yhp);
                        yg[c - c0] = fma(hy * nv, nv, ygp);
                        w[i] = nu;
                        w[n + i] = nv;
                    }
                    eo[r - r0] = xfw;
                    eo[th + r - r0] = xhw;
                }
                for (int c = c0; c < c1; ++c) {
                    no[c - c0] = yh[c - c0];
                    no[tw + c - c0] = yg[c - c0];
                }
            }
        if (!any) break;
    }
    free(E); free(Nn); free(E2); free(N2); free(Wu); free(Su);
    free(yh); free(yg); free(win); free(sin_);
    if (tiles_done) *tiles_done = done;
    return k;
}

/* Variant with a time-extrapolated pass-1 guess: g = 2*g_wp - e_prev, where
 * g_wp is the "neighbour did not move" outflow and e_prev the neighbour's
 * final outflow of the previous step (second-order in dt).  e_prev buffers
 * (E: nt*2*th, N: nt*2*tw) are read and then overwritten with this step's
 * final outflows; pass have_prev = 0 on the first step.                     */
int orc_march_tiled_sim2(int nx, int ny, const double *inv_dx, const double *inv_dy,
                         const double *src, const double *lbc, double dt,
                         const double *wp, double *w, int th, int tw, int kmax,
                         double tol, long long *tiles_done, double *eprev, double *nprev,
                         int have_prev, long long *pass_tiles)
{
    const size_t n = (size_t)nx * ny;
    const int nti = (ny + th - 1) / th, ntj = (nx + tw - 1) / tw;
    const size_t nt = (size_t)nti * ntj;
    orc_grid g = {inv_dx, inv_dy, src, lbc, 0.5 * dt, nx, ny};
    double *E = (double *)calloc(nt * 2 * th, sizeof(double));
    double *Nn = (double *)calloc(nt * 2 * tw, sizeof(double));
    double *E2 = (double *)calloc(nt * 2 * th, sizeof(double));
    double *N2 = (double *)calloc(nt * 2 * tw, sizeof(double));
    double *Wu = (double *)calloc(nt * 2 * th, sizeof(double));
    double *Su = (double *)calloc(nt * 2 * tw, sizeof(double));
    double *yh = (double *)malloc(tw * sizeof(double)), *yg = (double *)malloc(tw * sizeof(double));
    double *win = (double *)malloc(2 * th * sizeof(double)), *sin_ = (double *)malloc(2 * tw * sizeof(double));
    long long done = 0;
    int k;
    for (k = 1; k <= kmax; ++k) {
        int any = 0;
        long long pt = 0;
        memcpy(E2, E, nt * 2 * th * sizeof(double));
        memcpy(N2, Nn, nt * 2 * tw * sizeof(double));
        for (int I = 0; I < nti; ++I)
            for (int J = 0; J < ntj; ++J) {
                const size_t t = (size_t)I * ntj + J;
                const int r0 = I * th, c0 = J * tw;
                const int r1 = r0 + th < ny ? r0 + th : ny, c1 = c0 + tw < nx ? c0 + tw : nx;
                for (int c = c0; c < c1; ++c) {
                    double sh = 0.0, sg = 0.0;
                    if (I > 0) {
                        if (k == 1) {
                            double bu, bv, xfp, xhp, yhp, ygp;
                            const size_t i = IDX(r0 - 1, c, nx);
                            const double pu = wp[i], pv = wp[n + i];
                            cell_pre(&g, r0 - 1, c, pu, pv, &bu, &bv, &xfp, &xhp, &yhp, &ygp);
                            const double hy = 0.5 * (g.a * inv_dy[r0 - 1]);
                            sh = fma(hy * pu, pv, yhp);
                            sg = fma(hy * pv, pv, ygp);
                            if (have_prev) {
                                const double *pn = nprev + (t - ntj) * 2 * tw;
                                sh = 2.0 * sh - pn[c - c0];
                                sg = 2.0 * sg - pn[tw + c - c0];
                            }
                        } else {
                            const double *sn = N2 + (t - ntj) * 2 * tw;
                            sh = sn[c - c0];
                            sg = sn[tw + c - c0];
                        }
                    }
                    sin_[c - c0] = sh;
                    sin_[tw + c - c0] = sg;
                }
                for (int r = r0; r < r1; ++r) {
                    double xf = 0.0, xh = 0.0;
                    if (J > 0) {
                        if (k == 1) {
                            double bu, bv, xfp, xhp, yhp, ygp;
                            const size_t i = IDX(r, c0 - 1, nx);
                            const double pu = wp[i], pv = wp[n + i];
                            cell_pre(&g, r, c0 - 1, pu, pv, &bu, &bv, &xfp, &xhp, &yhp, &ygp);
                            const double hx = 0.5 * (g.a * inv_dx[c0 - 1]);
                            xf = fma(hx * pu, pu, xfp);
                            xh = fma(hx * pu, pv, xhp);
                            if (have_prev) {
                                const double *pe = eprev + (t - 1) * 2 * th;
                                xf = 2.0 * xf - pe[r - r0];
                                xh = 2.0 * xh - pe[th + r - r0];
                            }
                        } else {
                            const double *se = E2 + (t - 1) * 2 * th;
                            xf = se[r - r0];
                            xh = se[th + r - r0];
                        }
                    }
                    win[r - r0] = xf;
                    win[th + r - r0] = xh;
                }
                int need = (k == 1);
                if (!need) {
                    double *wu = Wu + t * 2 * th, *su = Su + t * 2 * tw;
                    for (int r = 0; r < r1 - r0 && !need; ++r)
                        need = moved(win[r], wu[r], tol) || moved(win[th + r], wu[th + r], tol);
                    for (int c = 0; c < c1 - c0 && !need; ++c)
                        need = moved(sin_[c], su[c], tol) || moved(sin_[tw + c], su[tw + c], tol);
                }
                if (!need) continue;
                any = 1;
                ++done;
                ++pt;
                memcpy(Wu + t * 2 * th, win, 2 * th * sizeof(double));
                memcpy(Su + t * 2 * tw, sin_, 2 * tw * sizeof(double));
                for (int c = c0; c < c1; ++c) {
                    yh[c - c0] = sin_[c - c0];
                    yg[c - c0] = sin_[tw + c - c0];
                }
                double *eo = E + t * 2 * th, *no = Nn + t * 2 * tw;
                for (int r = r0; r < r1; ++r) {
                    double xfw = win[r - r0], xhw = win[th + r - r0];
                    const double ay = g.a * inv_dy[r], hy = 0.5 * ay;
                    for (int c = c0; c < c1; ++c) {
                        const size_t i = IDX(r, c, nx);
                        const double hx = 0.5 * (g.a * inv_dx[c]);
                        double bu, bv, xfp, xhp, yhp, ygp;
                        cell_pre(&g, r, c, wp[i], wp[n + i], &bu, &bv, &xfp, &xhp, &yhp, &ygp);
                        const double cu = (bu + xfw) + yh[c - c0];
                        const double cv = (bv + yg[c - c0]) + xhw;
                        const double mm = fma(hx, cu, hy * cv);
                        const double s = 0.5 + sqrt(0.25 + mm);
                        const double nu = cu / s, nv = cv / s;
                        const double hxu = hx * nu;
                        xfw = fma(hxu, nu, xfp);
                        xhw = fma(hxu, nv, xhp);
                        yh[c - c0] = fma(hy * nu, nv, yhp);
                        yg[c - c0] = fma(hy * nv, nv, ygp);
                        w[i] = nu;
                        w[n + i] = nv;
                    }
                    eo[r - r0] = xfw;
                    eo[th + r - r0] = xhw;
                }
                for (int c = c0; c < c1; ++c) {
                    no[c - c0] = yh[c - c0];
                    no[tw + c - c0] = yg[c - c0];
                }
            }
        if (pass_tiles && k <= 16) pass_tiles[k - 1] = pt;
        if (!any) break;
    }
    memcpy(eprev, E, nt * 2 * th * sizeof(double));
    memcpy(nprev, Nn, nt * 2 * tw * sizeof(double));
    free(E); free(Nn); free(E2); free(N2); free(Wu); free(Su);
    free(yh); free(yg); free(win); free(sin_);
    if (tiles_done) *tiles_done = done;
    return k;
}
