// Cross-wave LDS-DMA visibility probe: wave 0 DMAs 4 rows (64 x 16 B) into
// LDS, waits vmcnt(0), then publishes a flag in LDS; wave 1 polls the flag
// and checks every word.  Reports mismatches over many rounds.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) int lds_i32;
typedef __attribute__((address_space(3))) v4u lds_v4u;
__global__ void probe(const v4u *src, unsigned *bad, int rounds, int rows_src)
{
    __shared__ v4u win[4][64];
    __shared__ int flag, ack;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) { flag = -1; ack = -1; }
    __syncthreads();
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)src, 0, rows_src * 1024, 0x00020000);
    unsigned nb = 0;
    for (int it = 0; it < rounds; ++it) {
        if (wave == 0) {
            while (*(volatile lds_i32 *)&ack != it - 1) __builtin_amdgcn_s_sleep(1);
            for (int r = 0; r < 4; ++r)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void *)&win[r][0], 16,
                    (unsigned)((it * 4 + r) % rows_src) * 1024u + lane * 16u, 0, 0, 16);
            __builtin_amdgcn_s_waitcnt(0);
            if (lane == 0) *(volatile lds_i32 *)&flag = it;
        } else {
            while (*(volatile lds_i32 *)&flag != it) __builtin_amdgcn_s_sleep(1);
            for (int r = 0; r < 4; ++r) {
                const v4u g = src[((it * 4 + r) % rows_src) * 64 + lane];
                const v4u l = *(volatile lds_v4u *)&win[r][lane];
                nb += (g.x != l.x) + (g.y != l.y) + (g.z != l.z) + (g.w != l.w);
            }
            __builtin_amdgcn_s_waitcnt(0);
            if (lane == 0) *(volatile lds_i32 *)&ack = it;
        }
    }
    if (wave == 1) atomicAdd(bad, nb);
}
int main()
{
    const int rows = 4096;
    std::vector<unsigned> h(rows * 256);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0x9E3779B9u * (unsigned)(i + 1);
    v4u *d; unsigned *b;
    (void)hipMalloc(&d, rows * 1024); (void)hipMalloc(&b, 4); (void)hipMemset(b, 0, 4);
    (void)hipMemcpy(d, h.data(), rows * 1024, hipMemcpyHostToDevice);
    probe<<<256, 128>>>(d, b, 2000, rows);
    unsigned nb = 0; (void)hipMemcpy(&nb, b, 4, hipMemcpyDeviceToHost);
    printf("dma_xwave_probe: %u mismatched words (256 blocks x 2000 rounds x 4096 words)\n", nb);
    return 0;
}
