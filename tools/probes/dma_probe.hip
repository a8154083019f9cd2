// LDS-DMA layout probe: one wave DMAs 16 rows of 64 x 16 B (buffer_load_dwordx4
// ... lds, M0 = row * 1 KB) and checks every word against the source.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned v4u __attribute__((ext_vector_type(4)));
__global__ void probe(const v4u *src, unsigned *bad, int L)
{
    __shared__ v4u win[16][64];
    const int lane = threadIdx.x;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)src, 0, L * 1024, 0x00020000);
    for (int r = 0; r < 16; ++r)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void *)&win[r][0], 16, (unsigned)(r + 3) * 1024u + lane * 16u, 0, 0, 16);
    __builtin_amdgcn_s_waitcnt(0);
    unsigned nb = 0;
    for (int r = 0; r < 16; ++r) {
        v4u g = src[(r + 3) * 64 + lane], l = win[r][lane];
        nb += (g.x != l.x) + (g.y != l.y) + (g.z != l.z) + (g.w != l.w);
    }
    atomicAdd(bad, nb);
}
int main()
{
    const int L = 32;
    std::vector<unsigned> h(L * 256);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0x1000u + (unsigned)i;
    v4u *d; unsigned *b;
    hipMalloc(&d, L * 1024); hipMalloc(&b, 4); hipMemset(b, 0, 4);
    hipMemcpy(d, h.data(), L * 1024, hipMemcpyHostToDevice);
    probe<<<1, 64>>>(d, b, L);
    unsigned nb = 0; hipMemcpy(&nb, b, 4, hipMemcpyDeviceToHost);
    printf("dma_probe: %u mismatched words of %d\n", nb, 16 * 64 * 4);
    return nb != 0;
}
