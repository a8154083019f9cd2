// march_stamp.hip -- diagnostic build of the march engine with s_memtime
// stamps around the skewed sweep of tile 0 (not part of the library).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -DBURG_STAMPS march_stamp.hip
#include "../finitedifference_amd/csrc/march.hip"

#include <cstdio>
#include <vector>

int main()
{
    using namespace burg;
    const int nx = 64, ny = 64, tw = 64;
    const size_t n = (size_t)nx * ny;
    std::vector<double> h(2 * n, 1.0), idx(nx, 10.24), src(nx, 0.001), lbc(ny, 0.3);
    double *d_w, *d_wp, *d_idx, *d_idy, *d_src, *d_lbc, *d_e;
    int *d_cnt;
    DevStats *d_st;
    hipMalloc(&d_w, 2 * n * 8); hipMalloc(&d_wp, 2 * n * 8);
    hipMalloc(&d_idx, nx * 8); hipMalloc(&d_idy, ny * 8); hipMalloc(&d_src, nx * 8); hipMalloc(&d_lbc, ny * 8);
    hipMalloc(&d_e, 8 * 1024 * 8); hipMalloc(&d_cnt, 64 * 4); hipMalloc(&d_st, sizeof(DevStats));
    hipMemset(d_e, 0, 8 * 1024 * 8); hipMemset(d_cnt, 0, 256); hipMemset(d_st, 0, sizeof(DevStats));
    hipMemcpy(d_wp, h.data(), 2 * n * 8, hipMemcpyHostToDevice);
    hipMemcpy(d_idx, idx.data(), nx * 8, hipMemcpyHostToDevice);
    hipMemcpy(d_idy, idx.data(), ny * 8, hipMemcpyHostToDevice);
    hipMemcpy(d_src, src.data(), nx * 8, hipMemcpyHostToDevice);
    hipMemcpy(d_lbc, lbc.data(), ny * 8, hipMemcpyHostToDevice);
    Coeffs cf{d_idx, d_idy, d_src, d_lbc, 0.025, nx, ny};
    Engine eg{};
    eg.eb[0] = d_e; eg.eb[1] = d_e + 1024; eg.nb[0] = d_e + 2048; eg.nb[1] = d_e + 3072;
    eg.wused = d_e + 4096; eg.sused = d_e + 5120; eg.counters = d_cnt; eg.ticket = d_cnt + 60;
    eg.kbound = 2; eg.tol = 0x1p-50; eg.nti = 1; eg.ntj = 1; eg.tw = tw;
    for (int rep = 0; rep < 3; ++rep) {
        launch_march_pass(cf, eg, d_wp, d_w, 1, false, d_st, 0);
        hipDeviceSynchronize();
        long long st[4];
        hipMemcpyFromSymbol(st, HIP_SYMBOL(burg_stamp), sizeof st);
        printf("sweep: %lld ticks over %lld steps = %.1f ticks/step; barrier wait sweeper %lld, helper %lld (unused)\n",
               st[0], st[1], (double)st[0] / st[1], st[2], st[3]);
    }
    return 0;
}
