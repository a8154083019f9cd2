// LDS-DMA above 64 KB: one wave DMAs 1 KB rows (buffer_load_dwordx4 ... lds)
// into a dynamic LDS image at offsets 0 .. 160 KB (the whole CU) and checks
// every word --
// does the pipe engine's wide-tile window have to sit below 64 KB?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned v4u __attribute__((ext_vector_type(4)));
extern __shared__ __attribute__((aligned(16))) unsigned char img[];
__global__ void probe(const v4u *src, unsigned *bad, int rows)
{
    typedef __attribute__((address_space(3))) v4u lv4u;
    lv4u *win = (lv4u *)img;
    const int lane = threadIdx.x;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)src, 0, rows * 1024, 0x00020000);
    for (int r = 0; r < rows; ++r)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *)&win[r * 64], 16,
                                                 (unsigned)r * 1024u + lane * 16u, 0, 0, 16);
    __builtin_amdgcn_s_waitcnt(0);
    unsigned nb = 0, first = 0xFFFFFFFFu;
    for (int r = 0; r < rows; ++r) {
        v4u g = src[r * 64 + lane], l = win[r * 64 + lane];
        unsigned e = (g.x != l.x) + (g.y != l.y) + (g.z != l.z) + (g.w != l.w);
        if (e && first == 0xFFFFFFFFu) first = r;
        nb += e;
    }
    atomicAdd(bad, nb);
    atomicMin(bad + 1, first);
}
int main()
{
    const int rows = 160;  // 160 KB: the whole LDS of a CU
    std::vector<unsigned> h(rows * 256);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0x1000u + (unsigned)i;
    v4u *d; unsigned *b;
    (void)hipMalloc(&d, rows * 1024); (void)hipMalloc(&b, 8);
    unsigned init[2] = {0, 0xFFFFFFFFu};
    (void)hipMemcpy(b, init, 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(d, h.data(), rows * 1024, hipMemcpyHostToDevice);
    (void)hipFuncSetAttribute((const void *)probe, hipFuncAttributeMaxDynamicSharedMemorySize, rows * 1024);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), rows * 1024, 0, d, b, rows);
    unsigned r[2];
    (void)hipMemcpy(r, b, 8, hipMemcpyDeviceToHost);
    printf("dma_high_probe: %d rows (%d KB): %u bad words, first bad row %d (%s)\n", rows, rows, r[0],
           (int)r[1], r[0] ? "rows at or above that KB are not reachable" : "all reachable");
    return 0;
}
