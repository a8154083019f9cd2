// hostxfer.hip -- every copy between CALLER host memory (numpy arrays, std::
// vectors: pageable) and the device goes through pinned bounce buffers that
// the library allocates once per device and never frees (DESIGN.md section 6,
// "host transfers"), as plain 1-D copies.
//
// Why (round 4's two intermittent hipErrorIllegalAddress reports, VERDICT r04
// item 1): both surfaced at a host-memory copy (burg_download_state into a
// fresh np.empty; the side-by-side sweep's upload from a per-call std::vector)
// right after calls that had (a) hipHostRegister'ed a caller's snapshot matrix
// and copied into it with hipMemcpy2DAsync, and (b) handed pageable memory to
// hipMemcpy*, which the runtime may pin on the fly and cache by host address --
// Python frees and re-allocates same-sized arrays at the same address all the
// time.  Every kernel before them had completed cleanly and the ring indices
// of every kernel are proven in range (burg_ring_audit), so these runtime
// paths were the remaining suspects.  They are gone: the runtime only ever
// sees pinned memory the library owns for the life of the process and 1-D
// device <-> pinned copies; the CPU moves the bytes between the caller's
// array and the bounce buffer (double-buffered against the DMA) and does any
// striding.
//
// Every function here is synchronous: when it returns, the caller's buffer
// may be reused or freed (h2d) or holds the data (d2h).
#include <algorithm>
#include <cstring>
#include <mutex>

#include "burg_internal.h"

namespace burg {
namespace {

constexpr size_t kBounceBytes = (size_t)8 << 20;  // per buffer; two per device
constexpr int kMaxDevices = 64;

struct Bounce {
    std::mutex mu;
    char *buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool ready = false;
};

Bounce g_bounce[kMaxDevices];

// the calling thread's current device's bounce pair, created on first use
hipError_t bounce_acquire(Bounce **out)
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
    Bounce &b = g_bounce[dev];
    b.mu.lock();
    if (!b.ready) {
        for (int i = 0; i < 2; ++i) {
            if (!b.buf[i] && (e = hipHostMalloc((void **)&b.buf[i], kBounceBytes, hipHostMallocDefault)) != hipSuccess) {
                b.buf[i] = nullptr;
                b.mu.unlock();
                return e;
            }
            if (!b.ev[i] && (e = hipEventCreateWithFlags(&b.ev[i], hipEventDisableTiming)) != hipSuccess) {
                b.ev[i] = nullptr;
                b.mu.unlock();
                return e;
            }
        }
        b.ready = true;
    }
    // (a call that returned early on an error may have left a copy in flight)
    for (int i = 0; i < 2; ++i) (void)hipEventSynchronize(b.ev[i]);
    *out = &b;
    return hipSuccess;
}

struct BounceLock {
    Bounce *b = nullptr;
    ~BounceLock()
    {
        if (b) b->mu.unlock();
    }
};

}  // namespace

hipError_t h2d(void *dst, const void *src, size_t bytes, hipStream_t st)
{
    if (bytes == 0) return hipSuccess;
    BounceLock lk;
    hipError_t e = bounce_acquire(&lk.b);
    if (e != hipSuccess) return e;
    Bounce &b = *lk.b;
    bool pending[2] = {false, false};
    int i = 0;
    for (size_t off = 0; off < bytes; off += kBounceBytes, i ^= 1) {
        const size_t n = std::min(kBounceBytes, bytes - off);
        if (pending[i] && (e = hipEventSynchronize(b.ev[i])) != hipSuccess) return e;
        std::memcpy(b.buf[i], (const char *)src + off, n);
        if ((e = hipMemcpyAsync((char *)dst + off, b.buf[i], n, hipMemcpyHostToDevice, st)) != hipSuccess ||
            (e = hipEventRecord(b.ev[i], st)) != hipSuccess)
            return e;
        pending[i] = true;
    }
    for (int k = 0; k < 2; ++k)
        if (pending[k] && (e = hipEventSynchronize(b.ev[k])) != hipSuccess) return e;
    return hipSuccess;
}

hipError_t d2h(void *dst, const void *src, size_t bytes, hipStream_t st)
{
    if (bytes == 0) return hipSuccess;
    BounceLock lk;
    hipError_t e = bounce_acquire(&lk.b);
    if (e != hipSuccess) return e;
    Bounce &b = *lk.b;
    // chunk k's DMA into buffer k & 1 is issued before chunk k - 1 is copied
    // out on the CPU
    size_t prev_off = 0, prev_n = 0;
    int i = 0;
    for (size_t off = 0;; off += kBounceBytes, i ^= 1) {
        const size_t n = off < bytes ? std::min(kBounceBytes, bytes - off) : 0;
        if (n) {
            if ((e = hipMemcpyAsync(b.buf[i], (const char *)src + off, n, hipMemcpyDeviceToHost, st)) != hipSuccess ||
                (e = hipEventRecord(b.ev[i], st)) != hipSuccess)
                return e;
        }
        if (prev_n) {
            if ((e = hipEventSynchronize(b.ev[i ^ 1])) != hipSuccess) return e;
            std::memcpy((char *)dst + prev_off, b.buf[i ^ 1], prev_n);
        }
        if (!n) break;
        prev_off = off;
        prev_n = n;
    }
    return hipSuccess;
}

// 2-D copies (hipMemcpy2D semantics: `height` rows of `width` bytes).  No
// rectangular copy reaches the runtime either: the DMA moves the contiguous
// span of a chunk of rows (pitch included) and the CPU does the striding on
// the host side.
hipError_t d2h_2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width,
                  size_t height, hipStream_t st)
{
    if (width == 0 || height == 0) return hipSuccess;
    if (spitch == width && dpitch == width) return d2h(dst, src, width * height, st);
    if (spitch > kBounceBytes || width > spitch) {  // (a row span wider than a buffer: row by row)
        for (size_t r = 0; r < height; ++r) {
            const hipError_t e = d2h((char *)dst + r * dpitch, (const char *)src + r * spitch, width, st);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    BounceLock lk;
    hipError_t e = bounce_acquire(&lk.b);
    if (e != hipSuccess) return e;
    Bounce &b = *lk.b;
    const size_t rows = (kBounceBytes - width) / spitch + 1;  // per chunk: span <= a buffer
    auto unpack = [&](int k, size_t r0, size_t nr) {
        const char *p = b.buf[k];
        char *q = (char *)dst + r0 * dpitch;
        for (size_t r = 0; r < nr; ++r) std::memcpy(q + r * dpitch, p + r * spitch, width);
    };
    size_t prev_r0 = 0, prev_nr = 0;
    int i = 0;
    for (size_t r0 = 0;; r0 += rows, i ^= 1) {
        const size_t nr = r0 < height ? std::min(rows, height - r0) : 0;
        if (nr) {
            const size_t span = (nr - 1) * spitch + width;
            if ((e = hipMemcpyAsync(b.buf[i], (const char *)src + r0 * spitch, span,
                                    hipMemcpyDeviceToHost, st)) != hipSuccess ||
                (e = hipEventRecord(b.ev[i], st)) != hipSuccess)
                return e;
        }
        if (prev_nr) {
            if ((e = hipEventSynchronize(b.ev[i ^ 1])) != hipSuccess) return e;
            unpack(i ^ 1, prev_r0, prev_nr);
        }
        if (!nr) break;
        prev_r0 = r0;
        prev_nr = nr;
    }
    return hipSuccess;
}

hipError_t h2d_2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width,
                  size_t height, hipStream_t st)
{
    if (width == 0 || height == 0) return hipSuccess;
    if (dpitch != width || width > kBounceBytes) {  // (device rows not dense: row by row)
        for (size_t r = 0; r < height; ++r) {
            const hipError_t e = h2d((char *)dst + r * dpitch, (const char *)src + r * spitch, width, st);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    BounceLock lk;
    hipError_t e = bounce_acquire(&lk.b);
    if (e != hipSuccess) return e;
    Bounce &b = *lk.b;
    const size_t rows = kBounceBytes / width;
    bool pending[2] = {false, false};
    int i = 0;
    for (size_t r0 = 0; r0 < height; r0 += rows, i ^= 1) {
        const size_t nr = std::min(rows, height - r0);
        if (pending[i] && (e = hipEventSynchronize(b.ev[i])) != hipSuccess) return e;
        for (size_t r = 0; r < nr; ++r)
            std::memcpy(b.buf[i] + r * width, (const char *)src + (r0 + r) * spitch, width);
        if ((e = hipMemcpyAsync((char *)dst + r0 * width, b.buf[i], nr * width, hipMemcpyHostToDevice,
                                st)) != hipSuccess ||
            (e = hipEventRecord(b.ev[i], st)) != hipSuccess)
            return e;
        pending[i] = true;
    }
    for (int k = 0; k < 2; ++k)
        if (pending[k] && (e = hipEventSynchronize(b.ev[k])) != hipSuccess) return e;
    return hipSuccess;
}

}  // namespace burg
