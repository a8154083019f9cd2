// lds_occ.hip -- how many workgroups of a given LDS size are co-resident per
// CU on this GPU (census: each workgroup counts itself in, then waits up to
// ~20 ms for the whole grid; the count reached is what was resident at once).
// Build: hipcc --offload-arch=gfx950 -O2 lds_occ.hip -o lds_occ
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void census(unsigned *cnt, unsigned *seen, int waves)
{
    extern __shared__ int dyn[];
    if (threadIdx.x == 0) {
        dyn[0] = 1;
        atomicAdd(cnt, 1u);
        const long long t0 = __builtin_amdgcn_s_memrealtime();
        unsigned n = 0;
        for (;;) {
            n = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (n >= gridDim.x) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000) break;  // 100 MHz ticks: 20 ms
            __builtin_amdgcn_s_sleep(8);
        }
        atomicMin(seen, n);  // the first to give up saw only the resident ones
    }
    __syncthreads();
}

template <int SZ>
__global__ void census_static(unsigned *cnt, unsigned *seen, int waves)
{
    __shared__ int buf[SZ / 4];
    if (threadIdx.x == 0) {
        buf[SZ / 4 - 1] = 1;
        atomicAdd(cnt, 1u);
        const long long t0 = __builtin_amdgcn_s_memrealtime();
        unsigned n = 0;
        for (;;) {
            n = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (n >= gridDim.x) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000) break;
            __builtin_amdgcn_s_sleep(8);
        }
        atomicMin(seen, n + (buf[SZ / 4 - 1] - 1));
    }
    __syncthreads();
}

template <int SZ>
void run_static(unsigned *d, int cus)
{
    for (int th : {320, 384}) {
        for (int per = 1; per <= 2; ++per) {
            hipMemset(d, 0, 4);
            hipMemset(d + 1, 0xff, 4);
            hipLaunchKernelGGL(census_static<SZ>, dim3(cus * per), dim3(th), 0, 0, d, d + 1, th / 64);
            hipDeviceSynchronize();
            unsigned h[2];
            hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
            printf("static threads %d lds %6d grid %4d: resident %4u%s\n", th, SZ, cus * per, h[1],
                   h[1] >= (unsigned)(cus * per) ? "" : "  <-- not all");
        }
    }
}

int main(int argc, char **argv)
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *d;
    hipMalloc(&d, 8);
    {
        int c0 = 0;
        hipDeviceGetAttribute(&c0, hipDeviceAttributeMultiprocessorCount, 0);
        unsigned *d0;
        hipMalloc(&d0, 8);
        run_static<49152>(d0, c0);
        run_static<55296>(d0, c0);
        run_static<57344>(d0, c0);
        run_static<61440>(d0, c0);
        run_static<62992>(d0, c0);
        run_static<65536>(d0, c0);
        run_static<81920>(d0, c0);
        if (argc > 1) return 0;
    }
    const int sizes[] = {16384, 32768, 40960, 49152, 53248, 55296, 57344, 59392, 61440, 63488, 65536, 81920};
    const int threads[] = {320, 384, 640};
    for (int th : threads) {
        hipFuncSetAttribute((const void *)census, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        for (int sz : sizes) {
            int occ = 0;
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, census, th, sz);
            for (int per = 1; per <= 3; ++per) {
                hipMemset(d, 0, 4); hipMemset(d + 1, 0xff, 4);
                hipLaunchKernelGGL(census, dim3(cus * per), dim3(th), sz, 0, d, d + 1, th / 64);
                hipDeviceSynchronize();
                unsigned h[2];
                hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
                printf("threads %d lds %6d occ_api %d  grid %4d: resident %4u%s\n", th, sz, occ, cus * per, h[1],
                       h[1] >= (unsigned)(cus * per) ? "" : "  <-- not all");
            }
        }
    }
    return 0;
}
