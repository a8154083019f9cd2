// issue_probe.hip -- issue cost of fp64 VALU and SALU on gfx950, for one and
// several waves per SIMD (s_memtime cycles per loop iteration, per wave).
// Sizes the pipe engine's per-diagonal budget.
// Build: hipcc --offload-arch=gfx950 -O3 issue_probe.hip -o issue_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define N_IT 2048

__device__ __forceinline__ unsigned long long clk() { return __builtin_amdgcn_s_memtime(); }

// 8 independent fp64 FMA chains
__global__ void k_f64(double *o, double a, double b, long long *t)
{
    double x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = o[threadIdx.x & 63] + j;
    __syncthreads();
    const unsigned long long t0 = clk();
    for (int i = 0; i < N_IT; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = fma(x[j], a, b);
    }
    const unsigned long long t1 = clk();
    double s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j];
    o[64 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) t[threadIdx.x >> 6] = (long long)(t1 - t0);
}

// the same, f32
__global__ void k_f32(double *o, double a, double b, long long *t)
{
    float x[8];
    const float af = (float)a, bf = (float)b;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (float)o[threadIdx.x & 63] + j;
    __syncthreads();
    const unsigned long long t0 = clk();
    for (int i = 0; i < N_IT; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = fmaf(x[j], af, bf);
    }
    const unsigned long long t1 = clk();
    float s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j];
    o[64 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) t[threadIdx.x >> 6] = (long long)(t1 - t0);
}

// 8 fp64 FMAs + 8 SALU adds per iteration (independent)
__global__ void k_mix(double *o, double a, double b, long long *t)
{
    double x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = o[threadIdx.x & 63] + j;
    unsigned s0 = 1, s1 = 2;
    __syncthreads();
    const unsigned long long t0 = clk();
    for (int i = 0; i < N_IT; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            x[j] = fma(x[j], a, b);
            asm volatile("s_add_u32 %0, %0, %1" : "+s"(s0) : "s"(s1));
        }
    }
    const unsigned long long t1 = clk();
    double s = s0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j];
    o[64 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) t[threadIdx.x >> 6] = (long long)(t1 - t0);
}

// 16 SALU adds per iteration only
__global__ void k_salu(double *o, double a, double b, long long *t)
{
    unsigned s0 = 1, s1 = 2;
    __syncthreads();
    const unsigned long long t0 = clk();
    for (int i = 0; i < N_IT; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) asm volatile("s_add_u32 %0, %0, %1" : "+s"(s0) : "s"(s1));
    }
    const unsigned long long t1 = clk();
    o[64 + threadIdx.x] = s0;
    if ((threadIdx.x & 63) == 0) t[threadIdx.x >> 6] = (long long)(t1 - t0);
}

// the pipe cell's fast chain (cell_math.h: sqrt_normal, div2_normal), NC
// independent cells per lane and iteration, each fed back into itself
template <int NC>
__global__ void k_cell(double *o, double a, double b, long long *t)
{
    double e0[NC], e1[NC], n0[NC], n1[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        e0[j] = o[threadIdx.x & 63] + j;
        e1[j] = 0.1;
        n0[j] = 0.2;
        n1[j] = 0.3;
    }
    const double bu = 1.5, bv = 0.5, hx = 0.2, hy = 0.1, xfp = 0.3, xhp = 0.1, yhp = 0.05, ygp = 0.02;
    __syncthreads();
    const unsigned long long t0 = clk();
    for (int i = 0; i < N_IT; ++i) {
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const double cu = (bu + e0[j]) + n0[j], cv = (bv + n1[j]) + e1[j];
            const double q = 0.25 + fma(hx, cu, hy * cv);
            const double y = __builtin_amdgcn_rsq(q);
            double g = q * y, h = y * 0.5;
            const double r = fma(-h, g, 0.5);
            g = fma(g, r, g);
            h = fma(h, r, h);
            double d = fma(-g, g, q);
            g = fma(d, h, g);
            d = fma(-g, g, q);
            const double s = 0.5 + fma(d, h, g);
            double rc = __builtin_amdgcn_rcp(s);
            double e = fma(-s, rc, 1.0);
            rc = fma(rc, e, rc);
            e = fma(-s, rc, 1.0);
            rc = fma(rc, e, rc);
            const double t0_ = cu * rc, t1_ = cv * rc;
            const double nu = fma(fma(-s, t0_, cu), rc, t0_), nv = fma(fma(-s, t1_, cv), rc, t1_);
            const double hxu = hx * nu;
            e0[j] = fma(hxu, nu, xfp) * a;
            e1[j] = fma(hxu, nv, xhp) * a;
            n0[j] = fma(hy * nu, nv, yhp) * a;
            n1[j] = fma(hy * nv, nv, ygp) * a;
        }
    }
    const unsigned long long t1 = clk();
    double s = 0;
#pragma unroll
    for (int j = 0; j < NC; ++j) s += e0[j] + e1[j] + n0[j] + n1[j];
    o[64 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) t[threadIdx.x >> 6] = (long long)(t1 - t0);
}

int main()
{
    double *o;
    long long *t;
    hipMalloc(&o, (64 + 1024) * sizeof(double));
    hipMalloc(&t, 16 * sizeof(long long));
    double h[64];
    for (int i = 0; i < 64; ++i) h[i] = 1.0 + i * 1e-3;
    hipMemcpy(o, h, sizeof h, hipMemcpyHostToDevice);
    struct {
        const char *n;
        void (*k)(double *, double, double, long long *);
        int per_it;  // instructions of interest per iteration
    } ks[] = {{"f64 fma x8", k_f64, 8}, {"f32 fma x8", k_f32, 8}, {"f64 fma x8 + salu x8", k_mix, 16},
              {"salu x16", k_salu, 16}, {"cell chain x1 (per cell)", k_cell<1>, 1},
              {"cell chains x2 (per cell)", k_cell<2>, 2}, {"cell chains x4 (per cell)", k_cell<4>, 4}};
    for (auto &k : ks) {
        for (int waves : {1, 4, 8, 16}) {
            long long c[16] = {};
            for (int rep = 0; rep < 2; ++rep) {
                hipLaunchKernelGGL(k.k, dim3(1), dim3(64 * waves), 0, 0, o, 0.999, 0.001, t);
                hipDeviceSynchronize();
            }
            hipMemcpy(c, t, waves * sizeof(long long), hipMemcpyDeviceToHost);
            long long mx = 0;
            for (int w = 0; w < waves; ++w) mx = c[w] > mx ? c[w] : mx;
            printf("%-22s waves/WG %2d (per SIMD %d): %6.2f cycles per instruction per wave\n", k.n, waves,
                   waves < 4 ? 1 : waves / 4, (double)mx / N_IT / k.per_it);
        }
    }
    return 0;
}
