// loop_bisect.hip -- which part of the march sweep step costs what (gfx950).
#include <hip/hip_runtime.h>
#include <cstdio>
#define N_IT 2048
__device__ __forceinline__ double shr1(double x) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
struct Pre { double hx, xfp, xhp, yhp, ygp, bu, bv; };
__device__ __forceinline__ Pre pre(double pu, double pv, double ax, double ay, double sl) {
    Pre p; p.hx = 0.5 * ax; const double hu = 0.5 * pu;
    p.xfp = ax * (hu * pu); p.xhp = ax * (hu * pv); p.yhp = ay * (hu * pv); p.ygp = ay * ((0.5 * pv) * pv);
    p.bu = ((pu - p.xfp) - p.yhp) + sl; p.bv = (pv - p.ygp) - p.xhp; return p;
}
template <int V>
__global__ void k(double *o, long long *t) {
    __shared__ double lds[2][64 * 64];
    __shared__ double trash[2][64];
    const int lane = threadIdx.x;
    for (int i = lane; i < 64 * 64; i += 64) { lds[0][i] = 1.0 + 1e-4 * i; lds[1][i] = 0.5 + 1e-4 * i; }
    __syncthreads();
    double e0 = o[lane], e1 = 0.1, n0 = 0.2, n1 = 0.3, no0 = 0.1, no1 = 0.2;
    const double ay = 0.256, hy = 0.128;
    Pre pc = pre(1.1, 0.9, 0.256, ay, 0.001);
    double rx0 = 1.0, rx1 = 0.5;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < N_IT; ++s) {
        if (V >= 2) { n0 = shr1(no0); n1 = shr1(no1); if (lane == 0) { n0 = 0.2; n1 = 0.3; } }
        Pre pn = pc;
        if (V >= 3) {
            pn = pre(rx0, rx1, 0.256, ay, 0.001);
            const int j = (s + 2 - lane) & 63;
            rx0 = lds[0][lane * 64 + j]; rx1 = lds[1][lane * 64 + j];
        }
        const double cu = (pc.bu + e0) + n0, cv = (pc.bv + n1) + e1;
        const double mm = fma(pc.hx, cu, hy * cv);
        const double sq = 0.5 + sqrt(0.25 + mm);
        const double rs = 1.0 / sq;
        const double nu = cu * rs, nv = cv * rs;
        const double hxu = pc.hx * nu;
        double oe0 = fma(hxu, nu, pc.xfp), oe1 = fma(hxu, nv, pc.xhp);
        double on0 = fma(hy * nu, nv, pc.yhp), on1 = fma(hy * nv, nv, pc.ygp);
        if (V >= 4) {
            const int j = s - lane;
            const bool act = j >= 0 && j < 64;
            e0 = act ? oe0 : e0; e1 = act ? oe1 : e1; no0 = act ? on0 : no0; no1 = act ? on1 : no1;
            double *d0 = act ? &lds[0][lane * 64 + (j & 63)] : &trash[0][lane];
            double *d1 = act ? &lds[1][lane * 64 + (j & 63)] : &trash[1][lane];
            *d0 = nu; *d1 = nv;
        } else {
            e0 = oe0 * 0.999; e1 = oe1 * 0.999; no0 = on0 * 0.999; no1 = on1 * 0.999;
            if (V < 2) { n0 = no0; n1 = no1; }
        }
        if (V >= 3) pc = pn;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    o[lane] = e0 + e1 + no0 + no1 + lds[0][lane];
    if (lane == 0) t[0] = (long long)(t1 - t0);
}
int main() {
    double *o; long long *t;
    (void)hipMalloc(&o, 64 * sizeof(double)); (void)hipMalloc(&t, sizeof(long long));
    double h[64]; for (int i = 0; i < 64; ++i) h[i] = 1.0 + i * 1e-3;
    void (*ks[])(double *, long long *) = {k<1>, k<2>, k<3>, k<4>};
    const char *nm[] = {"chain only", "+ DPP neighbour shift", "+ LDS operands + precompute", "+ select commit + LDS write"};
    for (int v = 0; v < 4; ++v) {
        long long c = 0;
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipMemcpy(o, h, sizeof h, hipMemcpyHostToDevice);
            hipLaunchKernelGGL(ks[v], dim3(1), dim3(64), 0, 0, o, t);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(&c, t, sizeof c, hipMemcpyDeviceToHost);
        }
        printf("%-32s %7.1f cycles/step\n", nm[v], (double)c / N_IT);
    }
    return 0;
}
