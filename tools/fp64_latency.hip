// fp64_latency.hip -- microbenchmark of dependent fp64 chains on gfx950
// (one wave, s_memtime cycles per iteration).  Used to size the march cell's
// critical path.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
#include <hip/hip_runtime.h>
#include <cstdio>

#define N_IT 4096

__device__ __forceinline__ unsigned long long clk() { return __builtin_amdgcn_s_memtime(); }

extern "C" __global__ void k_fma(double *o, double a, double b, long long *t) {
    double x = o[threadIdx.x];
    unsigned long long t0 = clk();
    for (int i = 0; i < N_IT; ++i) x = fma(x, a, b);
    unsigned long long t1 = clk();
    o[threadIdx.x] = x;
    if (threadIdx.x == 0) t[0] = (long long)(t1 - t0);
}
extern "C" __global__ void k_fma4(double *o, double a, double b, long long *t) {
    double x = o[threadIdx.x], y = x + 1, z = x + 2, w = x + 3;
    unsigned long long t0 = clk();
    for (int i = 0; i < N_IT; ++i) { x = fma(x, a, b); y = fma(y, a, b); z = fma(z, a, b); w = fma(w, a, b); }
    unsigned long long t1 = clk();
    o[threadIdx.x] = x + y + z + w;
    if (threadIdx.x == 0) t[0] = (long long)(t1 - t0);
}
extern "C" __global__ void k_sqrt(double *o, double a, double b, long long *t) {
    double x = o[threadIdx.x];
    unsigned long long t0 = clk();
    for (int i = 0; i < N_IT; ++i) x = sqrt(x) + b;
    unsigned long long t1 = clk();
    o[threadIdx.x] = x;
    if (threadIdx.x == 0) t[0] = (long long)(t1 - t0);
}
extern "C" __global__ void k_div(double *o, double a, double b, long long *t) {
    double x = o[threadIdx.x];
    unsigned long long t0 = clk();
    for (int i = 0; i < N_IT; ++i) x = a / x + b;
    unsigned long long t1 = clk();
    o[threadIdx.x] = x;
    if (threadIdx.x == 0) t[0] = (long long)(t1 - t0);
}
extern "C" __global__ void k_rcp(double *o, double a, double b, long long *t) {
    double x = o[threadIdx.x];
    unsigned long long t0 = clk();
    for (int i = 0; i < N_IT; ++i) x = __builtin_amdgcn_rcp(x) + b;
    unsigned long long t1 = clk();
    o[threadIdx.x] = x;
    if (threadIdx.x == 0) t[0] = (long long)(t1 - t0);
}
extern "C" __global__ void k_rsq(double *o, double a, double b, long long *t) {
    double x = o[threadIdx.x];
    unsigned long long t0 = clk();
    for (int i = 0; i < N_IT; ++i) x = __builtin_amdgcn_rsq(x) + b;
    unsigned long long t1 = clk();
    o[threadIdx.x] = x;
    if (threadIdx.x == 0) t[0] = (long long)(t1 - t0);
}
// the march cell chain: inflow -> outflow, closed form with IEEE sqrt/div
extern "C" __global__ void k_cell(double *o, double a, double b, long long *t) {
    double e0 = o[threadIdx.x & 63], e1 = 0.1, n0 = 0.2, n1 = 0.3;
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const double bu = 1.5, bv = 0.5, hx = 0.2, hy = 0.1, xfp = 0.3, xhp = 0.1, yhp = 0.05, ygp = 0.02;
    unsigned long long t0 = clk();
    for (int i = 0; i < N_IT; ++i) {
        const double cu = (bu + e0) + n0, cv = (bv + n1) + e1;
        const double mm = fma(hx, cu, hy * cv);
        const double s = 0.5 + sqrt(0.25 + mm);
        const double rs = 1.0 / s;
        const double nu = cu * rs, nv = cv * rs;
        const double hxu = hx * nu;
        e0 = fma(hxu, nu, xfp) * a; e1 = fma(hxu, nv, xhp) * a;
        n0 = fma(hy * nu, nv, yhp) * a; n1 = fma(hy * nv, nv, ygp) * a;
    }
    unsigned long long t1 = clk();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    o[threadIdx.x & 63] = e0 + e1 + n0 + n1;
    if (threadIdx.x == 0 && blockIdx.x == 0) { t[0] = (long long)(t1 - t0); t[1] = (long long)(r1 - r0); }
}
// same chain with hardware rcp/rsq + one Newton step each (not IEEE-exact)
extern "C" __global__ void k_cell_fast(double *o, double a, double b, long long *t) {
    double e0 = o[threadIdx.x], e1 = 0.1, n0 = 0.2, n1 = 0.3;
    const double bu = 1.5, bv = 0.5, hx = 0.2, hy = 0.1, xfp = 0.3, xhp = 0.1, yhp = 0.05, ygp = 0.02;
    unsigned long long t0 = clk();
    for (int i = 0; i < N_IT; ++i) {
        const double cu = (bu + e0) + n0, cv = (bv + n1) + e1;
        const double q = 0.25 + fma(hx, cu, hy * cv);
        double y = __builtin_amdgcn_rsq(q);
        y = y * fma(-0.5 * q * y, y, 1.5);
        const double s = fma(q, y, 0.5);
        double r = __builtin_amdgcn_rcp(s);
        r = fma(fma(-s, r, 1.0), r, r);
        const double nu = cu * r, nv = cv * r;
        const double hxu = hx * nu;
        e0 = fma(hxu, nu, xfp) * a; e1 = fma(hxu, nv, xhp) * a;
        n0 = fma(hy * nu, nv, yhp) * a; n1 = fma(hy * nv, nv, ygp) * a;
    }
    unsigned long long t1 = clk();
    o[threadIdx.x] = e0 + e1 + n0 + n1;
    if (threadIdx.x == 0) t[0] = (long long)(t1 - t0);
}

int main() {
    double *o; long long *t;
    hipMalloc(&o, 64 * sizeof(double)); hipMalloc(&t, 2 * sizeof(long long));
    double h[64]; for (int i = 0; i < 64; ++i) h[i] = 1.0 + i * 1e-3;
    struct { const char *n; void (*k)(double *, double, double, long long *); } ks[] = {
        {"fma dependent", k_fma}, {"fma x4 indep", k_fma4}, {"sqrt(+add)", k_sqrt},
        {"div(+add)", k_div}, {"rcp(+add)", k_rcp}, {"rsq(+add)", k_rsq},
        {"march cell (IEEE)", k_cell}, {"march cell (rcp/rsq+NR)", k_cell_fast}};
    for (auto &k : ks) {
        for (int rep = 0; rep < 2; ++rep) {
            hipMemcpy(o, h, sizeof h, hipMemcpyHostToDevice);
            hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, o, 0.999, 0.001, t);
            hipDeviceSynchronize();
        }
        long long c = 0; hipMemcpy(&c, t, sizeof c, hipMemcpyDeviceToHost);
        // s_memtime counts at the shader clock (MI355X_MICROARCH.md constants table)
        printf("%-26s %8.1f cycles/iter\n", k.n, (double)c / N_IT);
    }
    // in-kernel clock: s_memtime ticks / s_memrealtime (100 MHz) at 1 and 256 waves
    for (int blocks : {1, 256, 1024}) {
        for (int rep = 0; rep < 3; ++rep) {
            hipMemcpy(o, h, sizeof h, hipMemcpyHostToDevice);
            hipLaunchKernelGGL(k_cell, dim3(blocks), dim3(64), 0, 0, o, 0.999, 0.001, t);
            hipDeviceSynchronize();
        }
        long long c[2] = {0, 0}; hipMemcpy(c, t, sizeof c, hipMemcpyDeviceToHost);
        printf("cell chain, %4d waves: %8.1f ticks/iter, clock %.2f GHz\n", blocks,
               (double)c[0] / N_IT, c[1] ? (double)c[0] / (c[1] * 10.0) : 0.0);
    }
    return 0;
}
