// chain_probe.hip -- how many cycles a compute wave needs per diagonal for the
// march cell chain with ONE cell per lane (the pipe kernel today) against TWO
// independent cells per lane (a vertical tile pair: rows l and l + 64, the
// second set's south inflow from the first set's lane 63 by a wave rotate).
// The loop has the pipe kernel's per-diagonal skeleton without its hand-off
// protocol: the previous state from LDS, the cell (MarchCell::pre + chain with
// the range check, ballot and the IEEE redo branch), the DPP south carry, the
// east carry in registers, one ring store per cell.  s_memtime cycles per
// diagonal per wave, for 1 workgroup (isolated) and 256 workgroups (4 compute
// waves each, every SIMD busy).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I finitedifference_amd/csrc \
//        tools/probes/chain_probe.hip -o /tmp/chain_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#include "cell_math.h"

using namespace burg;

constexpr int kD = 4096;  // diagonals per run
constexpr int kW = 16;    // previous-state slots in LDS (narrow-tile style)

__device__ __forceinline__ double shr1_or(double old0, double x)
{
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old0), __double2loint(x), 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old0), __double2hiint(x), 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
// lane i <- lane i-1, lane 0 <- lane 63 (DPP wave_ror:1)
__device__ __forceinline__ double ror1(double x)
{
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), 0x13C, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), 0x13C, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

// MarchCell::chain<true> for two independent cells, statement by statement
// interleaved (same op order per cell: bit-identical results)
__device__ __forceinline__ void chain2_fast(const MarchCell::Pre &pa, const MarchCell::Pre &pb,
                                            const MarchCell::Row &rw, const double *e0, const double *e1,
                                            const double *n0, const double *n1, double *oe0, double *oe1,
                                            double *on0, double *on1, double *o0, double *o1, bool &ok)
{
    const MarchCell::Pre *p[2] = {&pa, &pb};
    double cu[2], cv[2], q[2], y[2], g[2], h[2], r[2], d[2], s[2], rc[2], e[2], t0[2], t1[2], m0[2],
        m1[2], nu[2], nv[2], hxu[2];
    unsigned bad = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) cu[k] = (p[k]->bu + e0[k]) + n0[k];
#pragma unroll
    for (int k = 0; k < 2; ++k) cv[k] = (p[k]->bv + n1[k]) + e1[k];
#pragma unroll
    for (int k = 0; k < 2; ++k) q[k] = 0.25 + fma(p[k]->hx, cu[k], rw.hy * cv[k]);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const unsigned hu = (unsigned)__double2hiint(cu[k]), hv = (unsigned)__double2hiint(cv[k]);
        const unsigned hq = (unsigned)__double2hiint(q[k]);
        const unsigned eu = ((hu - (123u << 20)) >> 20) & 0x7FFu;
        const unsigned ev = ((hv - (123u << 20)) >> 20) & 0x7FFu;
        const unsigned eq = (hq - (123u << 20)) >> 20;
        bad |= max(max(eu, ev), eq);
    }
    ok = bad < 1800u;
#pragma unroll
    for (int k = 0; k < 2; ++k) y[k] = __builtin_amdgcn_rsq(q[k]);
#pragma unroll
    for (int k = 0; k < 2; ++k) { g[k] = q[k] * y[k]; h[k] = y[k] * 0.5; }
#pragma unroll
    for (int k = 0; k < 2; ++k) r[k] = fma(-h[k], g[k], 0.5);
#pragma unroll
    for (int k = 0; k < 2; ++k) { g[k] = fma(g[k], r[k], g[k]); h[k] = fma(h[k], r[k], h[k]); }
#pragma unroll
    for (int k = 0; k < 2; ++k) d[k] = fma(-g[k], g[k], q[k]);
#pragma unroll
    for (int k = 0; k < 2; ++k) g[k] = fma(d[k], h[k], g[k]);
#pragma unroll
    for (int k = 0; k < 2; ++k) d[k] = fma(-g[k], g[k], q[k]);
#pragma unroll
    for (int k = 0; k < 2; ++k) s[k] = 0.5 + fma(d[k], h[k], g[k]);
#pragma unroll
    for (int k = 0; k < 2; ++k) rc[k] = __builtin_amdgcn_rcp(s[k]);
#pragma unroll
    for (int k = 0; k < 2; ++k) e[k] = fma(-s[k], rc[k], 1.0);
#pragma unroll
    for (int k = 0; k < 2; ++k) rc[k] = fma(rc[k], e[k], rc[k]);
#pragma unroll
    for (int k = 0; k < 2; ++k) e[k] = fma(-s[k], rc[k], 1.0);
#pragma unroll
    for (int k = 0; k < 2; ++k) rc[k] = fma(rc[k], e[k], rc[k]);
#pragma unroll
    for (int k = 0; k < 2; ++k) { t0[k] = cu[k] * rc[k]; t1[k] = cv[k] * rc[k]; }
#pragma unroll
    for (int k = 0; k < 2; ++k) { m0[k] = fma(-s[k], t0[k], cu[k]); m1[k] = fma(-s[k], t1[k], cv[k]); }
#pragma unroll
    for (int k = 0; k < 2; ++k) { nu[k] = fma(m0[k], rc[k], t0[k]); nv[k] = fma(m1[k], rc[k], t1[k]); }
#pragma unroll
    for (int k = 0; k < 2; ++k) hxu[k] = p[k]->hx * nu[k];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        oe0[k] = fma(hxu[k], nu[k], p[k]->xfp);
        oe1[k] = fma(hxu[k], nv[k], p[k]->xhp);
        on0[k] = fma(rw.hy * nu[k], nv[k], p[k]->yhp);
        on1[k] = fma(rw.hy * nv[k], nv[k], p[k]->ygp);
        o0[k] = nu[k];
        o1[k] = nv[k];
    }
}

struct Cell {
    double e0, e1, no0, no1;
};

template <int SETS, bool IL, int ST = 1>
__global__ __launch_bounds__(256) void chain_kernel(const double *cin, double2 *ring, long long *cyc,
                                                    long long *ieee)
{
    __shared__ double2 st[4][SETS][kW][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const double alpha = 0.025, invdx = 10.24;
    const double ay = alpha * invdx, hy = 0.5 * ay;
    const MarchCell::Row rw{ay, hy, 0.0};
    for (int k = 0; k < SETS; ++k)
        for (int c = 0; c < kW; ++c) st[wave][k][c][lane] = make_double2(1.0 + 0.001 * c, 1.0);
    Cell cs[SETS];
    for (int k = 0; k < SETS; ++k) cs[k] = Cell{0.0, 0.0, 0.0, 0.0};
    double2 *my = ring + ((size_t)blockIdx.x * 4 + wave) * (size_t)SETS * kD * 64;
    long long nieee = 0;
    const double idx = invdx * cin[0];  // (hoisted: no global load in the loop)
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < kD; ++s) {
        double o0[SETS], o1[SETS], oe0[SETS], oe1[SETS], on0[SETS], on1[SETS];
        MarchCell::Pre p[SETS];
        double n0[SETS], n1[SETS];
        bool ok[SETS];
#pragma unroll
        for (int k = 0; k < SETS; ++k) {
            const double2 x = st[wave][k][s & (kW - 1)][lane];
            const double xs[2] = {x.x, x.y};
            p[k] = MarchCell::pre(Coeffs{0, 0, 0, 0, alpha, 0, 0}, rw, xs, idx, 0.001, false);
        }
        // south inflows: set 0 lane 0 from the boundary (0), set k > 0 lane 0
        // from set k-1's lane 63 (the vertical pair)
        n0[0] = shr1_or(0.0, cs[0].no0);
        n1[0] = shr1_or(0.0, cs[0].no1);
#pragma unroll
        for (int k = 1; k < SETS; ++k) {
            n0[k] = shr1_or(ror1(cs[k - 1].no0), cs[k].no0);
            n1[k] = shr1_or(ror1(cs[k - 1].no1), cs[k].no1);
        }
        if constexpr (SETS == 2 && IL) {
            const double e0[2] = {cs[0].e0, cs[1].e0}, e1[2] = {cs[0].e1, cs[1].e1};
            chain2_fast(p[0], p[1], rw, e0, e1, n0, n1, oe0, oe1, on0, on1, o0, o1, ok[0]);
            ok[1] = ok[0];
        } else {
#pragma unroll
            for (int k = 0; k < SETS; ++k)
                MarchCell::chain<true>(p[k], rw, cs[k].e0, cs[k].e1, n0[k], n1[k], oe0[k], oe1[k], on0[k],
                                       on1[k], o0[k], o1[k], ok[k]);
        }
        bool allok = true;
#pragma unroll
        for (int k = 0; k < SETS; ++k) allok = allok && ok[k];
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(!allok) != 0, 0)) {
#pragma unroll
            for (int k = 0; k < SETS; ++k)
                MarchCell::chain<false>(p[k], rw, cs[k].e0, cs[k].e1, n0[k], n1[k], oe0[k], oe1[k],
                                        on0[k], on1[k], o0[k], o1[k], ok[k]);
            ++nieee;
        }
#pragma unroll
        for (int k = 0; k < SETS; ++k) {
            cs[k] = Cell{(s & (kW - 1)) == kW - 1 ? 0.0 : oe0[k], (s & (kW - 1)) == kW - 1 ? 0.0 : oe1[k],
                         on0[k], on1[k]};
            st[wave][k][s & (kW - 1)][lane] = make_double2(o0[k], o1[k]);
            if constexpr (ST == 1) {
                __builtin_nontemporal_store(o0[k], &my[((size_t)k * kD + s) * 64 + lane].x);
                __builtin_nontemporal_store(o1[k], &my[((size_t)k * kD + s) * 64 + lane].y);
            } else if constexpr (ST == 2) {  // plain (cached) stores
                my[((size_t)k * kD + s) * 64 + lane] = make_double2(o0[k], o1[k]);
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        cyc[blockIdx.x * 4 + wave] = (long long)(t1 - t0);
        ieee[blockIdx.x * 4 + wave] = nieee;
    }
}

template <int SETS, bool IL = false, int ST = 1>
void run(int blocks, double *d_in, double2 *d_ring, long long *d_cyc, long long *d_ieee)
{
    std::vector<long long> cyc(blocks * 4), ie(blocks * 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL((chain_kernel<SETS, IL, ST>), dim3(blocks), dim3(256), 0, 0, d_in, d_ring, d_cyc, d_ieee);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipMemcpy(cyc.data(), d_cyc, cyc.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(ie.data(), d_ieee, ie.size() * 8, hipMemcpyDeviceToHost);
    double avg = 0;
    for (long long c : cyc) avg += (double)c;
    avg /= cyc.size();
    // s_memtime ticks at 100 MHz on gfx950? report ns per diagonal from events too
    printf("sets=%d%s store=%d blocks=%d: %.1f memtime ticks per diagonal per wave, %.1f ns per diagonal "
           "(events), cells per ns chip-wide %.2f, ieee=%lld\n",
           SETS, IL ? " interleaved" : "", ST, blocks, avg / kD, ms * 1e6 / kD, (double)blocks * 4 * 64 * SETS * kD / (ms * 1e6),
           ie[0]);
}

int main()
{
    const int maxb = 256;
    double *d_in;
    double2 *d_ring;
    long long *d_cyc, *d_ieee;
    (void)hipMalloc(&d_in, 64);
    double one = 1.0;
    (void)hipMemcpy(d_in, &one, 8, hipMemcpyHostToDevice);
    (void)hipMalloc(&d_ring, (size_t)maxb * 4 * 2 * kD * 64 * sizeof(double2));
    (void)hipMalloc(&d_cyc, maxb * 4 * 8);
    (void)hipMalloc(&d_ieee, maxb * 4 * 8);
    for (int blocks : {1, 256}) {
        run<1>(blocks, d_in, d_ring, d_cyc, d_ieee);
        run<2>(blocks, d_in, d_ring, d_cyc, d_ieee);
        run<2, true>(blocks, d_in, d_ring, d_cyc, d_ieee);
        run<1, false, 0>(blocks, d_in, d_ring, d_cyc, d_ieee);
        run<1, false, 2>(blocks, d_in, d_ring, d_cyc, d_ieee);
    }
    return 0;
}
