/* sanitize_check.c -- host-side sanitizer run of the CPU oracle (test
 * infrastructure, like burgers_oracle.c itself): built with AddressSanitizer
 * and UndefinedBehaviorSanitizer by `make -C oracle sanitize` and run by
 * tests/test_oracle_golden.py::test_oracle_under_sanitizers.
 *
 * Exercises every entry point on a ragged grid (37 x 23: no dimension a
 * multiple of a tile) and checks the properties the parity tests rely on:
 *   - Newton (reference algorithm) and the closed-form march agree to 1e-12;
 *   - the tiled schedule simulator at tol = 0 is the march bit for bit;
 *   - the OpenMP sweep runs (2 threads) without touching memory it does not own;
 *   - residual of the march step is at round-off, J x and the block solve are
 *     inverse to each other.
 * Exit status 0 on success; any sanitizer report aborts the process.        */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void orc_residual(int nx, int ny, const double *inv_dx, const double *inv_dy, const double *src,
                  const double *lbc, double dt, const double *w, const double *wp, double *r);
void orc_jvp(int nx, int ny, const double *inv_dx, const double *inv_dy, double dt,
             const double *w, const double *x, double *y);
void orc_block_solve(int nx, int ny, const double *inv_dx, const double *inv_dy, double dt,
                     const double *w, const double *rhs, double *delta);
int orc_fom(int nx, int ny, const double *inv_dx, const double *inv_dy, const double *src,
            const double *lbc, double dt, const double *w0, int num_steps, int solver, int max_its,
            double cutoff, double *snaps, int *newton_its, double *final_rel);
int orc_march_sweep(int nx, int ny, const double *inv_dx, const double *inv_dy,
                    const double *src_b, const double *lbc_b, double dt, const double *w0, int nmu,
                    int num_steps, int threads);
int orc_march_tiled_sim(int nx, int ny, const double *inv_dx, const double *inv_dy,
                        const double *src, const double *lbc, double dt, const double *wp,
                        double *w, int th, int tw, int kmax, double tol, long long *tiles_done);

static double rel_l2(const double *a, const double *b, size_t m)
{
    double d = 0.0, s = 0.0;
    for (size_t i = 0; i < m; ++i) {
        d += (a[i] - b[i]) * (a[i] - b[i]);
        s += b[i] * b[i];
    }
    return sqrt(d / s);
}

int main(void)
{
    const int nx = 37, ny = 23, T = 4;
    const size_t n = (size_t)nx * ny, m = 2 * n;
    const double dt = 0.05, mu1 = 4.75, mu2 = 0.02, L = 100.0;
    double *inv_dx = malloc(nx * sizeof(double)), *inv_dy = malloc(ny * sizeof(double));
    double *src = malloc(nx * sizeof(double)), *lbc = malloc(ny * sizeof(double));
    const double dx = L / nx, dy = L / ny;
    for (int c = 0; c < nx; ++c) {
        inv_dx[c] = 1.0 / dx;
        src[c] = dt * 0.02 * exp(mu2 * (c + 0.5) * dx);
    }
    for (int r = 0; r < ny; ++r) {
        inv_dy[r] = 1.0 / dy;
        lbc[r] = 0.5 * dt * mu1 * mu1 / dx;
    }
    double *w0 = malloc(m * sizeof(double));
    for (size_t i = 0; i < m; ++i) w0[i] = 1.0;
    double *sn = malloc((T + 1) * m * sizeof(double)), *sm = malloc((T + 1) * m * sizeof(double));
    int its[T];
    double rel[T];
    orc_fom(nx, ny, inv_dx, inv_dy, src, lbc, dt, w0, T, 0, 100, 1e-12, sn, its, rel);
    orc_fom(nx, ny, inv_dx, inv_dy, src, lbc, dt, w0, T, 1, 0, 0.0, sm, NULL, NULL);
    const double e = rel_l2(sn + T * m, sm + T * m, m);
    printf("newton vs march after %d steps: %.3e (newton updates %d %d %d %d)\n", T, e, its[0],
           its[1], its[2], its[3]);
    if (!(e < 1e-12)) return 1;

    double *w = malloc(m * sizeof(double));
    long long tiles = 0;
    const int k = orc_march_tiled_sim(nx, ny, inv_dx, inv_dy, src, lbc, dt, sm + m, w, 8, 16, 64,
                                      0.0, &tiles);
    if (memcmp(w, sm + 2 * m, m * sizeof(double)) != 0) {
        printf("tiled simulator differs from the march\n");
        return 1;
    }
    printf("tiled simulator: %d passes, %lld tile marches, bitwise = march\n", k, tiles);

    double *srcb = malloc(3 * nx * sizeof(double)), *lbcb = malloc(3 * ny * sizeof(double));
    for (int j = 0; j < 3; ++j) {
        memcpy(srcb + j * nx, src, nx * sizeof(double));
        memcpy(lbcb + j * ny, lbc, ny * sizeof(double));
    }
    const int used = orc_march_sweep(nx, ny, inv_dx, inv_dy, srcb, lbcb, dt, w0, 3, T, 2);
    printf("sweep: %d threads\n", used);

    double *r = malloc(m * sizeof(double)), *r0 = malloc(m * sizeof(double));
    orc_residual(nx, ny, inv_dx, inv_dy, src, lbc, dt, sm + T * m, sm + (T - 1) * m, r);
    orc_residual(nx, ny, inv_dx, inv_dy, src, lbc, dt, sm + (T - 1) * m, sm + (T - 1) * m, r0);
    double nr = 0.0, n0 = 0.0;
    for (size_t i = 0; i < m; ++i) {
        nr += r[i] * r[i];
        n0 += r0[i] * r0[i];
    }
    printf("march residual ||R||/||R0|| = %.3e\n", sqrt(nr / n0));
    if (!(sqrt(nr / n0) < 1e-13)) return 1;

    double *x = malloc(m * sizeof(double)), *y = malloc(m * sizeof(double)),
           *z = malloc(m * sizeof(double));
    for (size_t i = 0; i < m; ++i) x[i] = sin(0.37 * (double)i) + 1.5;
    orc_jvp(nx, ny, inv_dx, inv_dy, dt, sm + T * m, x, y);
    orc_block_solve(nx, ny, inv_dx, inv_dy, dt, sm + T * m, y, z);
    const double ez = rel_l2(z, x, m);
    printf("block_solve(J x) vs x: %.3e\n", ez);
    if (!(ez < 1e-13)) return 1;

    free(inv_dx), free(inv_dy), free(src), free(lbc), free(w0), free(sn), free(sm), free(w);
    free(srcb), free(lbcb), free(r), free(r0), free(x), free(y), free(z);
    printf("sanitize_check ok\n");
    return 0;
}
