// Timing probe of lspg_solve_kernel alone (npod scaling), by including the
// kernel source.  hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I finitedifference_amd/csrc tools/solve_probe.hip -o tools/solve_probe
#include "../finitedifference_amd/csrc/lspg.hip"
#include <cstdio>
#include <vector>
#include <cmath>
using namespace burg;
int main()
{
    for (int npod : {8, 16, 32, 64, 95, 127}) {
        const int P = lspg_cols(npod);
        std::vector<double> G((size_t)P * P, 0.0);
        for (int i = 0; i < npod; ++i) {
            for (int k = 0; k < npod; ++k) G[i * P + k] = (i == k ? 2.0 : 0.0) + 1.0 / (1.0 + i + k);
            G[i * P + npod] = 1.0;
        }
        double *dG, *dy;
        unsigned *derr;
        hipMalloc(&dG, sizeof(double) * P * P);
        hipMalloc(&dy, sizeof(double) * 128);
        hipMalloc(&derr, 4);
        hipMemcpy(dG, G.data(), sizeof(double) * P * P, hipMemcpyHostToDevice);
        hipMemset(dy, 0, sizeof(double) * 128);
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        launch_lspg_solve(dG, npod, dy, nullptr, derr, 0);
        hipDeviceSynchronize();
        hipEventRecord(a, 0);
        const int reps = 20;
        for (int r = 0; r < reps; ++r) launch_lspg_solve(dG, npod, dy, nullptr, derr, 0);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        printf("npod %3d: %.1f us per solve (%s)\n", npod, 1000.0 * ms / reps,
               hipGetErrorString(hipGetLastError()));
        hipFree(dG), hipFree(dy), hipFree(derr);
    }
    return 0;
}
