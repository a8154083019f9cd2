// pipe.hip -- the pipe engine: K implicit time steps of the 2D inviscid Burgers
// FOM in ONE launch, exactly the sequential march (orc_march_step, bit for bit),
// pipelined over tiles and time steps.
//
// The dependence structure is the streaming engine's (stream.hip): the
// reference residual (C/hypernet2D.py:2512-2570) couples a cell only to itself
// and its west/south neighbours, so (step, row, column) is a 3-D wavefront.
// A tile is 64 rows (one per lane) x W columns; at diagonal s lane r works on
// local time t = s - r (step t / W, column t % W); the south inflow of lane r
// is lane r-1's north outflow of the previous diagonal (one DPP move) and the
// west inflow is the lane's own east outflow, except at tile edges.
//
// WHO moves the edge data, and through what:
//   * a workgroup = 4 compute waves = 4 horizontally adjacent tiles of one
//     strip, plus one comm wave (320 threads, one workgroup per CU);
//   * west->east edges between the workgroup's own tiles go through LDS rings;
//   * every edge that crosses workgroups is polled by the comm wave, which
//     deposits the granules into LDS inboxes, writes the global slot back to
//     "empty", and grants the compute waves permission to overwrite their
//     outbound global slots;
//   * so the compute waves never wait on a global load of edge data: they read
//     LDS, run the cell chain and fire-and-forget their stores (trajectory
//     ring and outbound granules).
//
// Where the previous step of a cell comes from depends on the tile width:
//   * narrow tiles (W = 8, 16): the lane's own output of diagonal s - W, kept
//     in LDS (st[W][64]): no global load at all in the loop;
//   * wide tiles (W = 32 .. 1024, the 4096^2 grid and the multi-GPU slabs of
//     2048 x 8192 / 16384 cells): the tile's trajectory ring in HBM, entry
//     s - W (written by the same wave W diagonals earlier).  A sixth wave per
//     workgroup, the loader, streams those entries into an LDS window of kWin
//     diagonals per compute wave (LDS-DMA, one 1 KB row per diagonal) and
//     publishes how far each window is filled; the compute waves read LDS
//     only.  A compute wave never issues a global load, so no s_waitcnt of
//     its own ever waits on its stores (vmcnt counts loads and stores
//     together, in issue order).  The loader reads an entry only after the
//     compute wave has published that the entry's store completed: at the
//     start of each block of U diagonals it waits vmcnt(3U) -- every store
//     older than U diagonals -- and publishes that point.
//
// South/north streams are indexed by diagonal: comm lane j of wave k's group
// of 16 handles the diagonals d = j (mod 16) of that tile -- the granule of
// (step d / W, column d % W).  The comm wave polls a stream only when the
// compute wave that needs it is at most kLA diagonals away (each compute wave
// publishes its progress in LDS), so the mailboxes are not re-read thousands
// of times before their data can exist.
//
// Global mailbox slots carry two sentinel colours: a slot is free for step q
// when it holds the sentinel of q's colour ((q / kPipeR) & 1); the consumer,
// after reading step q, writes the other colour -- the colour of step
// q + kPipeR.  A grant can then never be based on the emptiness that preceded
// the producer's own (possibly still in flight) store of step q - kPipeR.
//
// Multi-GPU: the bottom strip's south inflow and the top
// strip's north outflow may live in memory shared with the neighbour rank's
// process (halo_in / halo_out: pinned host memory or the consumer GPU's own
// memory), accessed at system scope (sc0 sc1); the protocol is unchanged.
//
// Residency: the pipeline needs every workgroup on the GPU at once.  Before
// its first wait each workgroup checks in on a census counter; if the whole
// grid is not resident within a bounded time the launch fails fast
// (err[3] = 64) instead of stalling.  Every later wait is bounded in wall time
// (s_memrealtime): a wave that gives up sets the error word and the LDS abort
// flag, and the launch drains.
#include <algorithm>
#include <climits>
#include <cstddef>
#include <type_traits>

#include "burg_internal.h"
#include "cell_math.h"

// pipe_narrow.hip includes this file with BURG_PIPE_NARROW_TU = 1: it
// compiles the narrow-tile kernels (W = 8, 16) in their own unit, this one the
// wide ones; both units are built with LLVM's max-ilp machine scheduler (the
// Makefile: narrow +1.2 % with 8-diagonal blocks, round 3; round 2's 4-diagonal
// blocks had preferred the default scheduler, profiles/r02/sched/)
#ifndef BURG_PIPE_NARROW_TU
#define BURG_PIPE_NARROW_TU 0
#endif

namespace burg {
const void *pipe_narrow_fn(int W, bool sweep);  // pipe_narrow.hip
const void *pipe_pair_fn(bool sweep);           // pipe_narrow.hip: pipe_kernel<16, sweep, true>
size_t pipe_pair_image(bool sweep);             // pipe_narrow.hip: its LDS image
namespace {

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// sentinel high words (signalling-NaN payloads: arithmetic never produces them)
constexpr unsigned kSentHi0 = 0x7FF4DEADu;  // global slot empty, colour 0
constexpr unsigned kSentHi1 = 0x7FF5DEADu;  // global slot empty, colour 1
constexpr unsigned kSentLo = 0xBEEF5A5Au;
constexpr unsigned kLdsEmptyHi = 0x7FF6DEADu;  // LDS slot empty
constexpr unsigned kOOB = 0xC0000000u;  // past every buffer's range: loads 0, stores dropped
constexpr int kR = kPipeR;
constexpr unsigned G = kPipeGranuleStride;
// BURG_DMA_READBACK: 1 = the loader reads each block's LDS-DMA bytes back
// before it publishes filled[] (round 5, defensive); 0 = publish right after
// the covering vmcnt (rounds 2-4, and the default again in round 6).  The
// covering vmcnt is what orders the DMA'd bytes for the issuing wave, and the
// filled[] flag, written after it and polled by the compute wave before its
// reads, plays the barrier's part for the other waves (MI355X_MICROARCH.md
// item 7); round 5's wrong window rows were the store-VGPR hazard (DESIGN.md
// section 6.2), not the DMA.  Without the read-back: 4096^2 +1.3 % (3
// interleaved rounds, profiles/r06/ab/aux/), the wide bitwise tests and the
// race screens with the loader / comm wave above the compute waves green.
#ifndef BURG_DMA_READBACK
#define BURG_DMA_READBACK 0
#endif
// BURG_LOADERS: loader waves per wide workgroup.  2 (round 5) = wave 5 fills
// compute waves 0-1's windows, wave 6 those of waves 2-3: twice the ring DMAs
// in flight per workgroup (one wave keeps at most 63 loads outstanding, and
// waits for a round to land before it issues the next); blocks waiting for
// their window 8.4 M -> 0.2 M per 16384 x 2048 launch, 179 -> 184.5 and
// 4096^2 184.7 -> 188.7 Gcell-updates/s (profiles/r05/ab/loaders).  1 = the
// single loader of rounds 2-4.
#ifndef BURG_LOADERS
#define BURG_LOADERS 2
#endif
// BURG_AB_SKIP (A/B ceiling probe, wrong results): diagonals per W of the
// wide tiles whose previous states the loader does not read back (0: off)
#ifndef BURG_AB_SKIP
#define BURG_AB_SKIP 0
#endif
// BURG_KEEP_BLOCK (round 6): the
// wide tiles keep the outputs of ONE block of U diagonals per W -- the block
// at diagonal kKeepS mod W -- in VGPRs of the compute wave, and read the next
// step's previous states of that block from there instead of the HBM ring
// (the loader skips their read-back); 0: every previous state from the ring
#ifndef BURG_KEEP_BLOCK
#define BURG_KEEP_BLOCK 0
#endif
constexpr int kKeepS = 64;  // (a steady / interior block for every W >= 128)
// BURG_KEEP_BLOCK=2: only the block's first half (8 diagonals, 32 VGPRs) is
// kept; the loader reads its other half back as usual
template <int W>
constexpr int uw_of();
template <int W>
constexpr int keep_n_of() { return BURG_KEEP_BLOCK == 2 ? uw_of<W>() / 2 : uw_of<W>(); }
template <int W>
constexpr bool keep_of() { return BURG_KEEP_BLOCK && (W == 128 || W == 256); }  // (W >= 512: the loader's
                                                                                 // column-table DMAs ride with the window's)
constexpr int kSL = 16;   // comm lanes per compute wave for the south / north streams
#ifndef BURG_KLA
#define BURG_KLA 16
#endif
// cache policy of the wide tiles' ring stores (16: sc1, write-through)
#ifndef BURG_RING_AUX
#define BURG_RING_AUX 16
#endif
// cache policy of the loader's ring reads (LDS-DMA): 18 = sc1 + nt, each
// entry is read once (4096^2 49.0 -> 46.2 ms per trajectory against sc1
// alone, profiles/r03/ab/ring_load_nt.txt)
#ifndef BURG_LOAD_AUX
#define BURG_LOAD_AUX 18
#endif
#ifndef BURG_NARROW_U
#define BURG_NARROW_U 8
#endif
// steady-edge diagonals, round 4: one lane-compare per diagonal instead of two
// (atE from the next diagonal's at0) and the narrow tiles' column-0 source +
// inlet sum once per block (A/B knob: 0 = the round-3 code)
#ifndef BURG_SE_OPT
#define BURG_SE_OPT 1
#endif
// the comm wave's poll window (diagonals ahead of a compute wave's progress):
// at least two blocks, so the next block's inflows arrive during this one
template <int W>
constexpr int la_of();
// Wide tiles run one workgroup per CU with a 16-diagonal window and blocks of
// 8.  Built with -DBURG_TWO_PER_CU=1, W = 64 and 128 run two workgroups per CU
// instead (two compute waves per SIMD: one wave's scalar, LDS and memory
// instructions issue beside the other's fp64 VALU -- 1.25x the compute rate
// per SIMD), which leaves 80 KB of LDS per workgroup: a 12-diagonal window,
// blocks of 4.  Measured at 4096^2 (W = 128, 2048 tiles) the longer
// hand-off chains then stall 20-27 % of the time and the whole runs slower
// (118-124 vs 135 Gcell-updates/s for W = 256), so it is off by default.
#ifndef BURG_TWO_PER_CU
#define BURG_TWO_PER_CU 0
#endif
// the wide tiles' window of previous states, diagonals per compute wave: a
// multiple of the block -- the loader fills up to KWIN - U diagonals ahead of
// the block being computed (W = 1024: 16, its column table takes the room; 24
// for W <= 512 measured no faster than 16)
#ifndef BURG_KWIN
#define BURG_KWIN 16
#endif
template <int W>
constexpr bool two_per_cu() { return BURG_TWO_PER_CU && (W == 64 || W == 128); }
// loader waves (BURG_LOADERS; at most 2 where two workgroups share a CU)
template <int W>
constexpr int nl_of() { return two_per_cu<W>() ? (BURG_LOADERS < 2 ? BURG_LOADERS : 2) : BURG_LOADERS; }
// BURG_STORE_WAVE (round 6): the
// one-cell W = 16 kernels' trajectory-ring stores are issued by a sixth wave
// that copies each compute wave's finished diagonals from its LDS state
// slots, so the compute waves neither issue them nor hold their VGPRs across
// diagonals: one 1024^2 trajectory -2.1 %, the one-cell 9-mu sweep -3.0 %
// (profiles/r06/ab/store_wave).  0: the compute waves store (rounds 1-5).
#ifndef BURG_STORE_WAVE
#define BURG_STORE_WAVE 1
#endif
template <int W>
constexpr bool store_wave_of() { return BURG_STORE_WAVE && W == 16; }
template <int W>
constexpr int threads_of()
{
    return W > 16 ? (5 + nl_of<W>()) * kWave : (store_wave_of<W>() ? 6 : 5) * kWave;  // + loader / store wave
}
// Blocks of 16 diagonals for W = 128 ... 1024 (round 3 for 128, 256; window
// 32 diagonals, LDS rings of 2 steps between the workgroup's waves -- the
// room for it; the LDS DMA reaches past 64 KB, tools/probes/
// dma_high_probe.hip): the block head is paid once per 16 diagonals --
// 4096^2 53.0 -> 49.0 ms per trajectory (profiles/r03/ab/wide_u16.txt).
// W = 512, 1024 (round 4): their full column tables (8 / 16 KB per wave)
// left no room for the 32-diagonal window, so they keep a rolling window of
// the last kCCW columns instead (ccw_of), refilled by the loader wave.
#ifndef BURG_WIDE_U16
#define BURG_WIDE_U16 1
#endif
#ifndef BURG_WIDE_U16_512
#define BURG_WIDE_U16_512 1
#endif
// BURG_W512_U8 (A/B build, round 5): W = 512 with blocks of 8 in the same
// 32-diagonal window (the loader then runs up to 3 blocks ahead instead of
// 1) and the rolling column table
#ifndef BURG_W512_U8
#define BURG_W512_U8 0
#endif
template <int W>
constexpr bool u16_of()
{
    return BURG_WIDE_U16 && !two_per_cu<W>() &&
           (W == 128 || W == 256 || (BURG_WIDE_U16_512 && ((W == 512 && !BURG_W512_U8) || W == 1024)));
}
// Rolling column table (W >= 512 with blocks of 16): slot t mod kCCW holds
// {hx, src} of local time t's column while lanes can need it.  A block at
// diagonal sb reads t in [sb - 63, sb + U); the loader writes the columns of
// the blocks it fills, t in [prog + U, prog + KWIN) (prog = the compute
// wave's block): 95 < kCCW apart, so no live slot is overwritten.
constexpr int kCCW = 128;
template <int W>
constexpr bool ccw_of() { return (u16_of<W>() || (BURG_W512_U8 && W == 512)) && W >= 512; }
template <int W>
constexpr int ccn_of() { return ccw_of<W>() ? kCCW : W; }  // column-table slots (before padding)
template <int W>
constexpr int win_of() { return two_per_cu<W>() ? 12 : (u16_of<W>() || (BURG_W512_U8 && W == 512)) ? 32 : W >= 1024 ? 16 : BURG_KWIN; }  // window (diagonals)
template <int W>
constexpr int uw_of() { return two_per_cu<W>() ? 4 : u16_of<W>() ? 16 : 8; }  // block (diagonals)
// (blocks of 16: 32 diagonals; BURG_U16_LA for A/B builds)
#ifndef BURG_U16_LA
#define BURG_U16_LA 32
#endif
template <int W>
constexpr int la_of() { return u16_of<W>() ? BURG_U16_LA : BURG_KLA; }
// LDS ring slots (steps) of the intra-workgroup west -> east edges
template <int W>
constexpr int rl_of() { return (u16_of<W>() || (W <= 16 && BURG_NARROW_U >= 16)) ? 2 : kPipeRL; }

// s_waitcnt vmcnt(N) with expcnt / lgkmcnt at their maximum (no wait): gfx9
// encoding vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14.  A
// builtin, not inline asm: asm would keep the compiler from proving the
// kernel AGPR-free, and the AGPR budget it then reserves caps the waves per
// SIMD.
template <int N>
__device__ __forceinline__ void wait_vmcnt()
{
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt(((N >> 4) << 14) | (0xF << 8) | (7 << 4) | (N & 15));
}

__device__ __forceinline__ d2 as_d2(v4u v)
{
    d2 r;
    r.x = __hiloint2double((int)v.y, (int)v.x);
    r.y = __hiloint2double((int)v.w, (int)v.z);
    return r;
}

__device__ __forceinline__ v4u as_v4u(double a, double b)
{
    v4u v;
    v.x = (unsigned)__double2loint(a);
    v.y = (unsigned)__double2hiint(a);
    v.z = (unsigned)__double2loint(b);
    v.w = (unsigned)__double2hiint(b);
    return v;
}

__device__ __forceinline__ v4u sent_g(int color)
{
    const unsigned hi = color ? kSentHi1 : kSentHi0;
    v4u v;
    v.x = kSentLo;
    v.y = hi;
    v.z = kSentLo;
    v.w = hi;
    return v;
}

__device__ __forceinline__ v4u lds_empty_g()
{
    v4u v;
    v.x = kSentLo;
    v.y = kLdsEmptyHi;
    v.z = kSentLo;
    v.w = kLdsEmptyHi;
    return v;
}

// a global granule holds data (neither sentinel colour in either half)
__device__ __forceinline__ bool g_is_data(v4u g)
{
    return ((g.y & ~0x00010000u) != kSentHi0) && ((g.w & ~0x00010000u) != kSentHi0);
}
__device__ __forceinline__ bool g_is_empty(v4u g, int color)
{
    const unsigned hi = color ? kSentHi1 : kSentHi0;
    return g.y == hi && g.w == hi;
}
__device__ __forceinline__ bool l_is_data(v4u g) { return g.y != kLdsEmptyHi && g.w != kLdsEmptyHi; }

// lane i <- lane i-1; lane 0 keeps `old0`
__device__ __forceinline__ double shr1_or(double old0, double x)
{
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old0), __double2loint(x), 0x138,
                                               0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old0), __double2hiint(x), 0x138,
                                               0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

// device mailboxes: sc1 (agent scope, write-through, L1 bypass);
// halo rings shared with another process / GPU: sc0 sc1 (system scope)
__device__ __forceinline__ v4u ld_dev(__amdgpu_buffer_rsrc_t rs, unsigned off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
}
__device__ __forceinline__ v4u ld_sys(__amdgpu_buffer_rsrc_t rs, unsigned off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 17);
}
__device__ __forceinline__ void st_dev(__amdgpu_buffer_rsrc_t rs, unsigned off, v4u v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);
}
__device__ __forceinline__ void st_sys(__amdgpu_buffer_rsrc_t rs, unsigned off, v4u v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 17);
}
// the same stores with a scalar offset part (soffset): a per-lane offset that
// stays constant over a block, a per-diagonal one in an SGPR
[[maybe_unused]] __device__ __forceinline__ void st_dev_so(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned soff, v4u v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff, soff, 16);
}
__device__ __forceinline__ void st_sys_so(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned soff, v4u v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff, soff, 17);
}
[[maybe_unused]] __device__ __forceinline__ void st_plain_so(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned soff, v4u v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff, soff, 0);
}
[[maybe_unused]] __device__ __forceinline__ void st_plain(__amdgpu_buffer_rsrc_t rs, unsigned off, v4u v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
}
[[maybe_unused]] __device__ __forceinline__ v4u ld_plain(__amdgpu_buffer_rsrc_t rs, unsigned off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, size_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ long long now_rt() { return (long long)__builtin_amdgcn_s_memrealtime(); }

// any lane: the ballot mask compared on the scalar unit (hipcc's __any goes
// through a VGPR select and a vector compare)
__device__ __forceinline__ bool any_lane(bool b) { return __builtin_amdgcn_ballot_w64(b) != 0; }

// (RetCursor, the retained-window walk: burg_internal.h)

// Launch diagnostics of one compute wave, recorded
// outside the hot path and with no loop-carried registers: when its first
// block could start (lane 0, once; the latest over the launch = the ramp,
// the earliest over the slab's halo strip = the wait for the rank below),
// the time each of its blocks waited for south inflow (lane 0, in the wait
// path), and at its end the number of such blocks -- split by where that
// inflow comes from (the halo ring / a strip of this GPU).
__device__ __forceinline__ void diag_first(const PipeArgs &a, bool halo)
{
    const unsigned long long t = (unsigned long long)now_rt();
    atomicMax(&a.stats->t_first_max, t);
    if (halo) atomicMin(&a.stats->t_halo_first, t);
}
__device__ __forceinline__ void diag_south_wait(const PipeArgs &a, bool halo, long long t0)
{
    atomicAdd(&a.stats->south_rt[halo ? 1 : 0], (unsigned long long)(now_rt() - t0));
}
__device__ __forceinline__ void diag_south_blocks(const PipeArgs &a, bool halo, unsigned n)
{
    if (n) atomicAdd(&a.stats->south_blocks[halo ? 1 : 0], (unsigned long long)n);
}


// LDS accesses that must not be cached in registers or merged (polled / handed
// off between waves).  Explicit address space 3: a volatile access through a
// generic pointer becomes a flat_load, which waits on vmcnt (and so on every
// older global store of the wave) -- the coupling this engine exists to avoid.
// The LDS image itself is addressed through address-space-3 pointers
// throughout (a select between two generic pointers costs a null check and a
// shared-aperture conversion per access).
#define LDS __attribute__((address_space(3)))
typedef LDS v4u lds_v4u;
typedef LDS unsigned lds_u32;
typedef LDS int lds_i32;
__device__ __forceinline__ v4u lds_ld(const LDS v4u *p) { return *(volatile const lds_v4u *)p; }
__device__ __forceinline__ void lds_st(LDS v4u *p, v4u v) { *(volatile lds_v4u *)p = v; }
__device__ __forceinline__ unsigned lds_ld32(const LDS void *p) { return *(volatile const lds_u32 *)p; }
__device__ __forceinline__ int lds_ldi(const LDS int *p) { return *(volatile const lds_i32 *)p; }
__device__ __forceinline__ void lds_sti(LDS int *p, int v) { *(volatile lds_i32 *)p = v; }
// Store VGPRs: a buffer store reads its offset and
// data VGPRs after it issues, so the kernels keep them live until the next
// iteration's stores.  launder: an opaque copy of a store's offset, so the
// store reads exactly the VGPR that is kept (no immediate-offset folding, no
// in-place offset increments); the data VGPRs are the kept values themselves.
__device__ __forceinline__ void launder(unsigned &off) { asm volatile("" : "+v"(off)); }
// (the comm wave: its data too -- a phi over two store branches let the
// compiler keep a copy and reuse the stored registers)
__device__ __forceinline__ void launder_all(unsigned &off, v4u &v) { asm volatile("" : "+v"(off), "+v"(v)); }

template <int W>
constexpr int ilog2() { return W <= 1 ? 0 : 1 + ilog2<W / 2>(); }

template <int W>
constexpr bool is_wide() { return W > 16; }

// south inbox ring (diagonals): a power of two above the comm wave's poll
// window plus a block; 32 for the narrow sweep kernel, whose LDS image is full
// (the room pads its per-trajectory source rows, read by block offsets)
template <int W, bool SWEEP>
constexpr int ni_of() { return (!is_wide<W>() && SWEEP) ? 32 : 64; }
// sweep source rows: W columns + the first kSrcPad again (steady blocks read
// base + u unwrapped, as the column table)
template <int W, bool SWEEP>
constexpr int src_pad_of() { return (!is_wide<W>() && SWEEP) ? BURG_NARROW_U : 0; }

// LDS image of one workgroup (SWEEP: a parameter sweep, burg_sweep -- the
// initial state and every trajectory's source / inlet terms stay on chip;
// PSW: the paired kernel with its store wave, DESIGN.md section 4.1g --
// two state slots per paired diagonal and half, and no st0: its sweeps start
// every trajectory from a uniform initial state, a constant)
template <int W, bool SWEEP, bool PSW = false>
struct PipeLds {
    static constexpr bool WIDE = is_wide<W>();
    static constexpr int kSW = SWEEP ? kPipeSweepMax : 1;
    static constexpr bool ST0 = SWEEP && !PSW;
    // wide: previous states by diagonal, filled by LDS-DMA (M0 base + 16 B
    // per lane) -- first in the image; the DMA reaches every byte of the
    // CU's LDS, not only the 64 KB below 2^16 (tools/probes/dma_high_probe.hip
    // writes and checks 0 .. 160 KB: profiles/r04/dma_high_probe.txt)
    // (narrow tiles: unused by the window; its 8 entries hold the zero south
    // inflow of a boundary strip, read by block offsets -- see zeros)
    v4u win[WIDE ? 4 : 1][WIDE ? win_of<W>() : 1][WIDE ? kWave : BURG_NARROW_U];
    // narrow: the lane's outputs of the last W diagonals (PSW: 2 W -- the
    // paired diagonal's A output in slot s mod 16, B's in 16 + s mod 16)
    v4u st[4][WIDE ? 1 : (PSW ? 2 * W : W)][WIDE ? 1 : kWave];
    v4u st0[4][ST0 ? W : 1][ST0 ? kWave : 1];  // sweep: initial state, st's layout
    double srcb[kSW][4][SWEEP ? W + src_pad_of<W, SWEEP>() : 1];  // sweep: src of trajectory j, by column
    double lbt[kSW][SWEEP ? kWave : 1];            // sweep: inlet term of trajectory j, by row
    // per wave: {hx, src} of the tile's columns, + the first kPad again, so a
    // steady block's lane reads base + u unwrapped (W = 8: no steady blocks)
    static constexpr int kPad = W == 8 ? 0 : (WIDE ? uw_of<W>() : BURG_NARROW_U);
    v4u cc[4][ccn_of<W>() + kPad];  // (W >= 512: the rolling window, ccw_of)
    v4u ewe[3][rl_of<W>()][kWave]; // wave k -> k+1 east outflow, by step slot and row
    v4u inw[rl_of<W>()][kWave];    // west inflow of wave 0 (comm wave deposits)
    v4u ins[4][ni_of<W, SWEEP>()];  // south inflow of each wave, by diagonal (comm wave deposits)
    v4u zero;               // inflow at the domain boundary
    v4u zeros[WIDE ? uw_of<W>() : 1];  // wide: south inflow of a boundary strip, read by block offsets
    // write target of lanes with nothing to hand off (W = 8 runs no steady
    // blocks: its image must fit three times in a CU)
    // (narrow 16-diagonal sweep blocks: 16 slots shared by 4 lanes each, the
    // room their longer column padding needs)
    // (narrow sweeps: 32 slots, two lanes each -- lanes 32 apart, in
    // different passes of a b128 write -- the room their padded source rows
    // need)
    static constexpr int kDump = W == 8 ? 1 : (!WIDE && SWEEP) ? (BURG_NARROW_U > 8 ? 16 : 32) : kWave;
    v4u dump[kDump];
    int perm[8];            // [0..3] north grants per wave (diagonal), [4] east grant of wave 3
                            // (step), [5] abort
    int prog[4];            // per compute wave: first diagonal of its current block
    int pe_row[kWave];      // east grant of wave 3, per row: steps whose slot is free
    int done[4];            // wide: per compute wave, diagonals whose stores completed
    int filled[4];          // wide: per compute wave, window filled below this diagonal
};

// The LDS image is DYNAMIC shared memory (launch_pipe passes its size): with a
// static image the compiler pads the kernel's VGPR allocation up to what the
// LDS-limited occupancy would leave (176 registers for a 90 KB image), and two
// 6-wave workgroups then no longer fit one CU.
extern __shared__ __attribute__((aligned(16))) unsigned char pipe_lds_image[];

// Waves per SIMD the register allocation must leave room for: the narrow
// W = 8 run kernel puts three 5-wave workgroups on a CU (4 waves on some
// SIMDs: <= 128 VGPRs -- round 5's store-VGPR fix had pushed it to 132, and
// eight slab processes sharing one GPU then no longer all fit)
template <int W, bool SWEEP>
constexpr int min_waves_of() { return (W == 8 && !SWEEP) ? 4 : 1; }

// PAIR (W = 16 run kernel only): the tile's two
// 8-column halves A (columns 0-7) and B (8-15) are marched by the same lanes,
// B one step behind A, so every lane carries two independent cell chains per
// diagonal -- each diagonal covers two columns, the launch half the diagonals.
template <int W, bool SWEEP, bool PAIR = false>
__global__ __launch_bounds__(threads_of<W>()) __attribute__((amdgpu_waves_per_eu(min_waves_of<W, SWEEP>()))) void pipe_kernel(PipeArgs a)
{
    constexpr int kThreads = threads_of<W>();
    // the paired kernel with a store wave: its
    // compute waves issue no ring stores
    constexpr bool PSW = PAIR && store_wave_of<W>();
    using Img = PipeLds<W, SWEEP, PSW>;
    static_assert(win_of<W>() % uw_of<W>() == 0, "the window holds whole blocks");
    static_assert(sizeof(Img) <= 160 * 1024, "LDS image exceeds the CU's 160 KiB");
    // the LDS-DMA window sits at the image's start and ends below the range
    // the probe verified (tools/probes/dma_high_probe.hip: 0 .. 160 KB)
    static_assert(offsetof(Img, win) == 0 && sizeof(Img::win) <= 160 * 1024,
                  "LDS-DMA window outside the probed range");
    static_assert(!(u16_of<W>() && two_per_cu<W>()), "blocks of 16 need the whole CU's LDS");
    constexpr bool WIDE = is_wide<W>();
    // three narrow W=8 workgroups per CU: room for 8 slab processes sharing one
    // GPU (the 750^2 C5 case, tests/test_gpu_parity.py) with all grids resident
    static_assert(W != 8 || SWEEP || 3 * sizeof(Img) <= 160 * 1024,
                  "narrow W=8 LDS image must fit three times in a CU");
    static_assert(W == 8 || W == 16 || (WIDE && W <= 1024 && (W & (W - 1)) == 0),
                  "pipe engine: W in {8, 16, 32, ..., 1024}");
    static_assert(!(WIDE && SWEEP), "parameter sweeps run on narrow tiles");
    constexpr int LW = ilog2<W>();
    // diagonals per block (progress published per block); narrow: at most W, so
    // a lane meets column 0 at most once per block
    constexpr int U = WIDE ? uw_of<W>() : (BURG_NARROW_U < W ? BURG_NARROW_U : W);
    constexpr int KWIN = win_of<W>();
    constexpr int kNI = ni_of<W, SWEEP>();
    constexpr int kRL = rl_of<W>();
    constexpr int kLA = la_of<W>();
    LDS Img &sm = *(LDS Img *)pipe_lds_image;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & (kWave - 1);
    const int wg = blockIdx.x;
    // a.wg_cm (host: pipe_args): column-major, workgroup i -> tile row i % nti,
    // so the dispatcher's XCD (i mod 8) is a tile-row class, not a column group
    const int ti = a.wg_cm ? wg % a.nti : wg / a.nwj;
    const int g = a.wg_cm ? wg / a.nti : wg - ti * a.nwj;
    const int tj0 = 4 * g;
    const int ntj = a.ntj;
    const int ny = a.cf.ny;
    // Side-by-side domains (a.nd > 1: burg_sweep's small-grid mode, DESIGN.md
    // section 4.1e): the strips are a.nd independent domains of a.nti_d
    // strips each, stacked (a domain's rows padded to whole strips; the
    // coefficient rows of cf are tiled the same way).  A domain's first strip
    // sees the boundary in the south, its last strip is partial and has no
    // north neighbour, and its columns read the domain's own table (mu2).
    const int dom = a.nd > 1 ? ti / a.nti_d : 0;
    const int tl = ti - dom * a.nti_d;  // strip within the domain
    const int ny_d = a.nd > 1 ? a.ny_d : ny;
    const d2 *const colc_d = a.colc + (size_t)dom * a.colc_dstride;
    const int nrow = min(kWave, ny_d - tl * kWave);
    const int top = nrow - 1;
    const int nval = min(4, ntj - tj0);  // valid tiles (waves) of this workgroup
    const int K = a.K;
    const int KW = K * W;
    const bool south_dev = tl > 0, south_host = tl == 0 && a.halo_in != nullptr;
    const bool north_dev = tl + 1 < a.nti_d, north_host = tl + 1 == a.nti_d && a.halo_out != nullptr;
    const int hcols = a.cf.nx;  // halo ring row length (granules): real columns only

    // ---- residency census: every workgroup must be on the GPU at once
    if (threadIdx.x == 0) {
        int ok = 1;
        if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
            ok = 0;
        } else {
            // (launch diagnostics: the first workgroup's entry)
            atomicMin(&a.stats->t_entry, (unsigned long long)now_rt());
            atomicAdd(a.census, 1u);
            const long long t0 = now_rt();
            for (;;) {
                const unsigned n = __hip_atomic_load(a.census, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                if (n >= gridDim.x) break;
                if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                    ok = 0;
                    break;
                }
                if (now_rt() - t0 > a.census_ticks) {
                    if (atomicOr(a.err, 1u) == 0) {
                        set_err3(a.err, (unsigned)wg, n, 64u);
                    }
                    ok = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(8);
            }
        }
        sm.perm[6] = ok;
    }
    __syncthreads();
    if (!sm.perm[6]) return;

    // ---- init (all waves), then one barrier; afterwards waves run freely
    for (int i = threadIdx.x; i < 3 * kRL * kWave; i += kThreads) (&sm.ewe[0][0][0])[i] = lds_empty_g();
    for (int i = threadIdx.x; i < kRL * kWave; i += kThreads) (&sm.inw[0][0])[i] = lds_empty_g();
    for (int i = threadIdx.x; i < 4 * kNI; i += kThreads) (&sm.ins[0][0])[i] = lds_empty_g();
    if (threadIdx.x < 6) sm.perm[threadIdx.x] = 0;
    if (threadIdx.x < kWave) sm.pe_row[threadIdx.x] = 0;
    if (threadIdx.x < 4) {
        sm.prog[threadIdx.x] = 0;
        sm.done[threadIdx.x] = 0;
        sm.filled[threadIdx.x] = 0;
    }
    if (threadIdx.x == 0) sm.zero = v4u{0u, 0u, 0u, 0u};
    if (threadIdx.x < (WIDE ? uw_of<W>() : BURG_NARROW_U))
        (WIDE ? &sm.zeros[0] : &sm.win[0][0][0])[threadIdx.x] = v4u{0u, 0u, 0u, 0u};
    // sweep: K / T trajectories of T steps (host guarantees <= kPipeSweepMax)
    const int nsw = SWEEP ? a.K / a.T : 1;
    if constexpr (SWEEP) {
        const size_t ncolp = (size_t)ntj * W;
        constexpr int WS = W + src_pad_of<W, SWEEP>();
        for (int i = threadIdx.x; i < nsw * 4 * WS; i += kThreads) {
            const int j = i / (4 * WS), kc = i - j * 4 * WS;
            const int kk = kc / WS, c = (kc - kk * WS) & (W - 1);
            (&sm.srcb[0][0][0])[i] = tj0 + kk < ntj ? a.colc_b[j * ncolp + (size_t)(tj0 + kk) * W + c].y
                                                    : 0.0;
        }
        for (int i = threadIdx.x; i < nsw * kWave; i += kThreads) {
            const int j = i / kWave, l = i - j * kWave;
            (&sm.lbt[0][0])[i] = a.lbc_b[(size_t)j * ny + ti * kWave + min(l, nrow - 1)];
        }
    }
    if (wave < nval) {
        const int tile = ti * ntj + tj0 + wave;
        // (the rolling window starts with the columns of t = 0 .. kCCW - 1)
        for (int c = lane; c < ccn_of<W>() + Img::kPad; c += kWave) {
            const d2 v = colc_d[(size_t)(tj0 + wave) * W + (c & (ccn_of<W>() - 1))];
            sm.cc[wave][c] = as_v4u(v.x, v.y);
        }
        if constexpr (!WIDE) {
            // state 0 of the lane's column c sits at diagonal c + lane - W (slot (c + lane) mod W)
            const __amdgpu_buffer_rsrc_t ring = rsrc(a.ring + (size_t)tile * a.Lt * kWave,
                                                     (size_t)a.Lt * kWave * 16);
            for (int c = 0; c < W; ++c) {
                const long long e = ring_pos(c + lane - W, a.origin, a.L, W, a.ret_k, a.ret_n, a.ret_base);
                const v4u x0 = ld_plain(ring, (unsigned)e * 1024u + lane * 16u);
                // (PAIR: half A in slots 0-7, half B in 8-15, slot (c + lane) mod 8;
                // PSW: A's column c read at paired diagonal c + lane from slot
                // (c + lane + 8) mod 16, B's column 8 + c at c + lane + 8 from
                // slot 16 + (c + lane) mod 16)
                const int slot = PSW ? ((c < 8) ? ((c + lane + 8) & 15) : 16 + ((c - 8 + lane) & 15))
                                     : PAIR ? ((c & 8) | ((c + lane) & 7)) : ((c + lane) & (W - 1));
                sm.st[wave][slot][lane] = x0;
                if constexpr (Img::ST0) sm.st0[wave][slot][lane] = x0;
            }
        }
    }
    __syncthreads();

    if (wave == 4) {
        // ================= comm wave =================
#ifndef BURG_COMM_PRIO
#define BURG_COMM_PRIO 0
#endif
        __builtin_amdgcn_s_setprio(BURG_COMM_PRIO);
        // south / north streams: lane = kS * 16 + jS handles the diagonals
        // jS (mod 16) of wave kS's tile
        const int kS = lane >> 4, jS = lane & (kSL - 1);
        const bool kval = kS < nval;
        const int tS = ti * ntj + tj0 + kS;  // this lane's tile (S/N groups)
        const bool actS = kval && (south_dev || south_host);
        const bool actN = kval && (north_dev || north_host);
        const bool rowok = lane < nrow;
        const bool actW = tj0 > 0 && rowok;                     // west inflow of wave 0
        const bool actE = nval == 4 && tj0 + 4 < ntj && rowok;  // east outflow of wave 3
        const __amdgpu_buffer_rsrc_t wbox = rsrc(a.wbox, a.wbox_bytes);
        const __amdgpu_buffer_rsrc_t sbox = rsrc(a.sbox, a.sbox_bytes);
        const __amdgpu_buffer_rsrc_t hin = rsrc(a.halo_in, a.halo_in ? a.halo_bytes : 0);
        const __amdgpu_buffer_rsrc_t hout = rsrc(a.halo_out, a.halo_out ? a.halo_bytes : 0);
        // halo rings hold real columns only: a padding column (C >= nx) of a
        // boundary strip is served a zero inflow / granted at once
        const int C0 = (tj0 + kS) * W;  // first global column of the lane's tile
        const unsigned sSb = (unsigned)tS * kR * W * G;          // south box of the lane's tile
        const unsigned sNb = (unsigned)(tS + ntj) * kR * W * G;  // south box of the north tile
        const unsigned sW = ((unsigned)(ti * ntj + tj0) * kR * kWave + lane) * G;
        const unsigned sE = ((unsigned)(ti * ntj + tj0 + 4) * kR * kWave + lane) * G;
        const unsigned sWEstep = (unsigned)kWave * G;
        const int kq = kS & 3;
        int qs = jS, qn = jS, qw = 0, qe = 0;  // qs, qn: diagonals; qw, qe: steps
        long long t_prog = now_rt();
        unsigned long long iters = 0;
        // the previous iteration's sentinel stores (data, offsets), kept live
        // until this one's (store VGPRs: see launder)
        v4u kc_s = v4u{0u, 0u, 0u, 0u}, kc_w = kc_s;
        unsigned kc_os = 0u, kc_ow = 0u;
        for (;;) {
            asm volatile("" ::"v"(kc_s), "v"(kc_w), "v"(kc_os), "v"(kc_ow));
            const bool rS = actS && qs < KW, rN = actN && qn < KW;
            const bool rW = actW && qw < K, rE = actE && qe < K;
            if (!__any(rS || rN || rW || rE)) break;
            ++iters;
            // due: the consuming / producing compute wave is within kLA diagonals
            const int pS = lds_ldi(&sm.prog[kq]);
            const int p0 = lds_ldi(&sm.prog[0]);
            const int p3 = lds_ldi(&sm.prog[3]);
            // (PAIR: a paired diagonal covers two stream indices; a lane meets
            // column 0 of step q at paired diagonal 8 q + lane, column 15 at
            // 8 q + 15 + lane)
            const bool wS = rS && (PAIR ? qs <= 2 * (pS + kLA) : qs <= pS + kLA);
            const bool wN = rN && (PAIR ? qn + 2 * top <= 2 * (pS + 2 * kLA) : qn + top <= pS + 2 * kLA);
            const bool wW = rW && (PAIR ? 8 * qw + lane <= p0 + kLA : qw * W + lane <= p0 + kLA);
            const bool wE = rE && (PAIR ? 8 * qe + 15 + lane <= p3 + 2 * kLA
                                        : qe * W + (W - 1) + lane <= p3 + 2 * kLA);
            const int aS = a.qbase + (qs >> LW), aN = a.qbase + (qn >> LW);
            const int aW = a.qbase + qw, aE = a.qbase + qe;
            const int cS = qs & (W - 1), cN = qn & (W - 1);
            const bool virtS = south_host && C0 + cS >= hcols;
            const bool virtN = north_host && C0 + cN >= hcols;
            const unsigned oS = wS && !virtS
                                    ? (south_dev ? sSb + ((unsigned)(aS & (kR - 1)) * W + cS) * G
                                                 : ((unsigned)(aS & (kR - 1)) * hcols + C0 + cS) * 16u)
                                    : kOOB;
            const unsigned oN = wN && !virtN
                                    ? (north_dev ? sNb + ((unsigned)(aN & (kR - 1)) * W + cN) * G
                                                 : ((unsigned)(aN & (kR - 1)) * hcols + C0 + cN) * 16u)
                                    : kOOB;
            const unsigned oW = wW ? sW + (unsigned)(aW & (kR - 1)) * sWEstep : kOOB;
            const unsigned oE = wE ? sE + (unsigned)(aE & (kR - 1)) * sWEstep : kOOB;
            const v4u gS = south_host ? ld_sys(hin, oS) : ld_dev(sbox, oS);  // OOB: zeros
            const v4u gN = north_host ? ld_sys(hout, oN) : ld_dev(sbox, oN);
            const v4u gW = ld_dev(wbox, oW);
            const v4u gE = ld_dev(wbox, oE);
            bool prog = false;
            if (wS && g_is_data(gS)) {
                LDS v4u *slot = &sm.ins[kq][qs & (kNI - 1)];
                if (!l_is_data(lds_ld(slot))) {
                    lds_st(slot, gS);
                    v4u e = sent_g(((aS / kR) & 1) ^ 1);
                    unsigned os = oS;
                    launder_all(os, e);
                    if (south_host) st_sys(hin, os, e);  // (virtual: oS is OOB, dropped)
                    else st_dev(sbox, os, e);
                    kc_s = e;
                    kc_os = os;
                    qs += kSL;
                    prog = true;
                }
            }
            if (wW && g_is_data(gW)) {
                LDS v4u *slot = &sm.inw[qw & (kRL - 1)][lane];
                if (!l_is_data(lds_ld(slot))) {
                    lds_st(slot, gW);
                    kc_w = sent_g(((aW / kR) & 1) ^ 1);
                    kc_ow = oW;
                    launder_all(kc_ow, kc_w);
                    st_dev(wbox, kc_ow, kc_w);
                    ++qw;
                    prog = true;
                }
            }
            if (wN && (virtN || g_is_empty(gN, (aN / kR) & 1))) {
                qn += kSL;
                prog = true;
            }
            if (wE && g_is_empty(gE, (aE / kR) & 1)) {
                ++qe;
                prog = true;
            }
            // grants: north of wave k = the first diagonal not yet verified
            // free over its 16 stream lanes; east of wave 3 = per row (a
            // minimum over rows would tie row 0's progress to row 63's)
            int vN = actN ? qn : INT_MAX;
            for (int m = 1; m < kSL; m <<= 1) vN = min(vN, __shfl_xor(vN, m));
            if (jS == 0 && kval) lds_sti(&sm.perm[kq], vN);
            if (actE) lds_sti(&sm.pe_row[lane], qe);
            const long long tn = now_rt();
            if (__any(prog) || !__any(wS || wN || wW || wE)) {
                t_prog = tn;  // progress, or nothing due (the compute waves time out themselves)
            } else if (tn - t_prog > a.spin_ticks) {
                if (lane == 0) {
                    lds_sti(&sm.perm[5], 1);
                    if (atomicOr(a.err, 1u) == 0) {
                        set_err3(a.err, (unsigned)(ti * ntj + tj0),
                                 (unsigned)min(min(wS ? qs : INT_MAX, wN ? qn : INT_MAX),
                                               min(wW ? qw : INT_MAX, wE ? qe : INT_MAX)),
                                 16u | (__any(wS) ? 1u : 0u) | (__any(wW) ? 2u : 0u) |
                                     (__any(wN) ? 4u : 0u) | (__any(wE) ? 8u : 0u));
                    }
                }
                break;
            }
            if (!__any(prog)) __builtin_amdgcn_s_sleep(2);
#ifdef BURG_COMM_SLEEP
            else __builtin_amdgcn_s_sleep(BURG_COMM_SLEEP);
#endif
            if (lds_ldi(&sm.perm[5])) break;
        }
        if (lane == 0) atomicAdd(&a.stats->why[5], iters);
        return;
    }
    if (WIDE && wave >= 5) {
        const int lw = wave - 5;
        // ================= loader wave (wide tiles) =================
        // window slot d mod KWIN of compute wave k <- ring entry (origin +
        // d - W) of its tile, once (1) the slot's previous diagonal is done
        // (d < prog + KWIN), (2) that entry's store has completed
        // (d - W < done) -- entries d < W are the initial state, written
        // before the launch.  One block of U entries per compute wave and
        // round; the DMAs land in issue order, so each wave's block is
        // published as soon as it (not the whole round) has landed.  (At a
        // priority above the compute waves' it would slow the compute wave it
        // shares a SIMD with, and with it the whole pipeline.)
        // (BURG_LOADER_PRIO: race-screen builds only)
#ifndef BURG_LOADER_PRIO
#define BURG_LOADER_PRIO 0
#endif
        __builtin_amdgcn_s_setprio(BURG_LOADER_PRIO);
        // the compute waves run whole blocks of U diagonals
        const int total = (KW + kWave - 1 + U - 1) / U * U;
        const long long L = a.L;
        int nf[4] = {0, 0, 0, 0};
        // retained windows: per wave, the walk of the entries it reads
        // (diagonal nf - W), block by block
        const bool ret = a.ret_k > 0;
        RetCursor rc[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) rc[k].init(a, W, -W);
        long long t_prog = now_rt();
        for (;;) {
            bool left = false;
            int got[4] = {0, 0, 0, 0};  // blocks issued this round, per wave
            int nld[4] = {0, 0, 0, 0};  // their loads
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (k >= nval) continue;
                if ((k * nl_of<W>()) >> 2 != lw) continue;  // (this loader's compute waves)
                const int pk = lds_ldi(&sm.prog[k]), dk = lds_ldi(&sm.done[k]);
                const int lim = min(min(total, pk + KWIN), dk + W);  // multiples of U
                // (kept half block: only its last U - KN rows are read back)
                const bool khalf = keep_of<W>() && keep_n_of<W>() < U && nf[k] >= W &&
                                   (nf[k] & (W - 1)) == kKeepS;
                if constexpr (keep_of<W>() && keep_n_of<W>() == U) {
                    // the kept block's previous states are in the compute
                    // wave's registers (after the first W diagonals): no read
                    if (nf[k] < lim && nf[k] >= W && (nf[k] & (W - 1)) == kKeepS) {
                        if (ret) (void)rc[k].next(a, W, U);  // (the walk moves on)
                        nf[k] += U;
                        if (lane == 0) lds_sti(&sm.filled[k], nf[k]);  // (earlier blocks: published)
                        left |= nf[k] < total;
                        continue;
                    }
                }
#if BURG_AB_SKIP > 0
                // A/B ceiling probe only (WRONG results):
                // the blocks of diagonals 64 .. 64 + BURG_AB_SKIP of every W
                // (after the first W) are not read back from the ring -- the
                // rate a read-back cut of that share could reach at most
                if (nf[k] < lim && nf[k] >= W && (unsigned)((nf[k] & (W - 1)) - 64) < (unsigned)BURG_AB_SKIP) {
                    if (ret) (void)rc[k].next(a, W, U);
                    nf[k] += U;
                    if (lane == 0) lds_sti(&sm.filled[k], nf[k]);  // (earlier blocks: published)
                    left |= nf[k] < total;
                    continue;
                }
#endif
                if (nf[k] < lim) {
                    const __amdgpu_buffer_rsrc_t ring =
                        rsrc(a.ring + (size_t)(ti * ntj + tj0 + k) * a.Lt * kWave, (size_t)a.Lt * kWave * 16);
                    long long e;
                    if (ret) {
                        e = rc[k].next(a, W, U);  // (a window's entries lie past L: no wrap below)
                    } else {
                        e = (a.origin + nf[k] - W) % L;
                        e = e < 0 ? e + L : e;
                    }
                    int slot = nf[k] % KWIN;
                    if (khalf) {
                        // (a block's U entries are consecutive: plain ring
                        // with a wrap, retained windows without one)
                        constexpr int KN = keep_n_of<W>() < U ? keep_n_of<W>() : 0;
                        e = ret ? e + KN : (e + KN >= L ? e + KN - L : e + KN);  // (windows lie past L)
                        slot += KN;
                    }
                    if constexpr (ccw_of<W>()) {
                        // the block's U columns into the rolling table (slot
                        // t mod kCCW, and its padding copy for the first U
                        // slots; else the same slot again): 2 DMAs of U lanes,
                        // issued before the window rows, landed by the same
                        // waits (kLoadsPerBlock per block)
                        const __amdgpu_buffer_rsrc_t colc = rsrc(colc_d + (size_t)(tj0 + k) * W, (size_t)W * 16);
                        const int sl = nf[k] & (kCCW - 1);
                        const unsigned co = (unsigned)((nf[k] + lane) & (W - 1)) * 16u;
                        if (lane < U) {
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(colc, (LDS void *)&sm.cc[k][sl], 16, co, 0, 0, 0);
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(colc, (LDS void *)&sm.cc[k][sl == 0 ? kCCW : sl], 16,
                                                                     co, 0, 0, 0);
                        }
                    }
                    if (khalf) {
                        constexpr int KN = keep_n_of<W>() < U ? keep_n_of<W>() : 0;
#pragma unroll
                        for (int u = KN; u < U; ++u) {
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(ring, (LDS void *)&sm.win[k][slot][0], 16,
                                                                     (unsigned)e * 1024u + lane * 16u, 0, 0, BURG_LOAD_AUX);
                            e = e + 1 == L ? 0 : e + 1;
                            slot = slot + 1 == KWIN ? 0 : slot + 1;
                        }
                        nld[k] = U - KN;
                    } else {
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(ring, (LDS void *)&sm.win[k][slot][0], 16,
                                                                     (unsigned)e * 1024u + lane * 16u, 0, 0, BURG_LOAD_AUX);
                            e = e + 1 == L ? 0 : e + 1;
                            slot = slot + 1 == KWIN ? 0 : slot + 1;
                        }
                        nld[k] = U + (ccw_of<W>() ? 2 : 0);
                    }
                    nf[k] += U;
                    got[k] = 1;
                }
                left |= nf[k] < total;
            }
            const int nb = got[0] + got[1] + got[2] + got[3];
            if (nb) {
                // wave k's rows have landed once at most NB x (blocks issued
                // after it) loads are outstanding
                constexpr int NB = U + (ccw_of<W>() ? 2 : 0);  // loads per block
                int after = nb;
                // (kept half blocks: the loads issued after wave k's, counted
                // exactly -- multiples of 8 up to 3 x 16)
                int la = nld[0] + nld[1] + nld[2] + nld[3];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (!got[k]) continue;
                    --after;
                    la -= nld[k];
                    if constexpr (keep_of<W>() && keep_n_of<W>() < U) {
                        static_assert(NB == 16 && U == 16, "kept half blocks: blocks of 16 rows");
                        switch (la >> 3) {
                        case 0: wait_vmcnt<0>(); break;
                        case 1: wait_vmcnt<8>(); break;
                        case 2: wait_vmcnt<16>(); break;
                        case 3: wait_vmcnt<24>(); break;
                        case 4: wait_vmcnt<32>(); break;
                        case 5: wait_vmcnt<40>(); break;
                        default: wait_vmcnt<48>(); break;
                        }
                    } else {
                        switch (after) {
                        case 0: wait_vmcnt<0>(); break;
                        case 1: wait_vmcnt<NB>(); break;
                        case 2: wait_vmcnt<2 * NB>(); break;
                        default: wait_vmcnt<3 * NB>(); break;
                        }
                    }
                    // Read the block's DMA'd bytes back before publishing them:
                    // an LDS-DMA write is ordered only for the ISSUING wave's
                    // own LDS reads behind its covering vmcnt (MI355X_MICROARCH.md
                    // item 7); the reads return only after the writes they are
                    // ordered behind, and the flag store waits for the reads.
                    // (Defensive: round 5's wrong window rows turned out to be
                    // the ring stores' VGPR hazard)
                    if constexpr (BURG_DMA_READBACK) {
                        v4u acc = v4u{0u, 0u, 0u, 0u};
                        const int s0 = (nf[k] - U) % KWIN;
#pragma unroll
                        for (int j = 0; j < U; ++j) acc ^= lds_ld(&sm.win[k][s0 + j][lane]);
                        if constexpr (ccw_of<W>()) {
                            const int sl = (nf[k] - U) & (kCCW - 1);
                            if (lane < U) {
                                acc ^= lds_ld(&sm.cc[k][sl + lane]);
                                acc ^= lds_ld(&sm.cc[k][(sl == 0 ? kCCW : sl) + lane]);
                            }
                        }
                        asm volatile("" ::"v"(acc));  // (the s_waitcnt lgkmcnt for the reads lands here)
                    }
                    if (lane == 0) lds_sti(&sm.filled[k], nf[k]);
                }
                t_prog = now_rt();
            }
            const bool issued = nb != 0;
            if (!left || lds_ldi(&sm.perm[5])) break;
            if (!issued) {
                if (now_rt() - t_prog > a.spin_ticks) {
                    if (lane == 0 && !lds_ldi(&sm.perm[5])) {
                        lds_sti(&sm.perm[5], 1);
                        if (atomicOr(a.err, 1u) == 0) {
                            // (the first compute wave this loader fills, and
                            // the loader's index in err[3] >> 8: ADVICE r05)
                            const int k0 = lw * 4 / nl_of<W>();
                            set_err3(a.err, (unsigned)(ti * ntj + tj0 + k0), (unsigned)nf[k0],
                                     128u | ((unsigned)lw << 8));
                        }
                    }
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        return;
    }
    if constexpr (!WIDE && store_wave_of<W>()) {
        if (wave == 5) {
            // ================= store wave (BURG_STORE_WAVE) =================
            // copies diagonal d of compute wave k from its LDS state slot
            // d mod W to the tile's ring entry -- the walk of the compute
            // wave's own stores (pw from origin with a wrap at L, or the
            // retained-window cursor per block) -- once the wave has moved
            // past d's block (prog), and publishes done[k] (diagonals
            // copied), which the compute wave's readiness test waits for
            // before it overwrites a slot (W diagonals later)
            // (BURG_STOREWAVE_PRIO: race-screen builds only)
#ifndef BURG_STOREWAVE_PRIO
#define BURG_STOREWAVE_PRIO 0
#endif
            __builtin_amdgcn_s_setprio(BURG_STOREWAVE_PRIO);
            if constexpr (PAIR) {
                // paired kernel (PSW): block [sb, sb + 8) of compute wave k left
                // its A outputs in slots (sb & 8) + u and its B outputs in
                // 16 + (sb & 8) + u.  Sweeps (a.play): each half of paired
                // diagonal s goes to ONE contiguous entry, origin + 2 s (+ 1
                // for B) -- ring_pos_paired, burg_internal.h; a full block
                // without a wrap is 16 stores at a lane offset plus a scalar
                // entry offset.  Otherwise the standard W = 16 layout, per
                // lane: the walk the paired compute waves stored along before
                // (A at eA: +1 per paired diagonal, +9 past column 7; B at
                // eA - 8).  Cells outside the launch are not stored (A:
                // 0 <= tau < 8 K, B: 8 <= tau < 8 K + 8; tau = sb + u - lane).
                // Store VGPRs: waves k = 0, 2 copy
                // through array x, k = 1, 3 through y, and the wave drains its
                // stores (vmcnt(0)) before it reloads either -- at k = 2 and at
                // the end of a pass -- with both arrays kept live until then.
                const int K8 = 8 * K;
                const int totalb = (K8 + 8 + kWave - 1 + U - 1) / U * U;
                const unsigned Lu = (unsigned)a.L;
                const bool play = a.play != 0;
                const unsigned lane16 = lane * 16u;
                int cp[4] = {0, 0, 0, 0};
                long long e0l = (long long)a.origin + 16LL * ((-lane) >> 3) + ((-lane) & 7) + lane;
                e0l %= a.L;
                if (e0l < 0) e0l += a.L;
                unsigned eA4[4];  // standard walk, per lane
                unsigned ep4[4];  // paired layout: entry origin + 2 cp (mod L), uniform
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    eA4[k] = (unsigned)e0l;
                    ep4[k] = (unsigned)a.origin;
                }
                static_assert(U == 8, "paired store wave: blocks of 8");
                auto keep = [](const v4u (&v)[2 * U], const unsigned (&o)[2 * U]) {
                    asm volatile("" ::"v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]),
                                 "v"(v[7]));
                    asm volatile("" ::"v"(v[8]), "v"(v[9]), "v"(v[10]), "v"(v[11]), "v"(v[12]), "v"(v[13]),
                                 "v"(v[14]), "v"(v[15]));
                    asm volatile("" ::"v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]), "v"(o[4]), "v"(o[5]), "v"(o[6]),
                                 "v"(o[7]), "v"(o[8]), "v"(o[9]), "v"(o[10]), "v"(o[11]), "v"(o[12]), "v"(o[13]),
                                 "v"(o[14]), "v"(o[15]));
                };
                long long t_prog = now_rt();
                for (;;) {
                    bool left = false, any = false;
                    v4u x[2 * U], y[2 * U];
                    unsigned ox[2 * U], oy[2 * U];  // (per-lane offsets: the standard walk's slow path)
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (k == 2) {
                            // (k = 0's and 1's stores complete before x, y are reloaded)
                            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                            keep(x, ox);
                            keep(y, oy);
                        }
                        v4u(&v)[2 * U] = (k & 1) ? y : x;
                        unsigned(&o)[2 * U] = (k & 1) ? oy : ox;
                        if (k >= nval) continue;
                        if (cp[k] < totalb && cp[k] + U <= lds_ldi(&sm.prog[k])) {
                            const __amdgpu_buffer_rsrc_t ring =
                                rsrc(a.ring + (size_t)(ti * ntj + tj0 + k) * a.Lt * kWave, (size_t)a.Lt * kWave * 16);
                            const int sb = cp[k], base = sb & 8;
#pragma unroll
                            for (int u = 0; u < U; ++u) {
                                v[u] = lds_ld(&sm.st[k][base + u][lane]);
                                v[U + u] = lds_ld(&sm.st[k][16 + base + u][lane]);
                            }
                            const unsigned ep = ep4[k];
                            if (play && sb >= 72 && sb + U <= K8 && ep + 2u * U <= Lu) {
                                // full block, no wrap: entries ep + 2 u (A), + 1 (B)
#pragma unroll
                                for (int u = 0; u < U; ++u) {
                                    st_plain_so(ring, lane16, (ep + 2u * u) * 1024u, v[u]);
                                    st_plain_so(ring, lane16, (ep + 2u * u + 1u) * 1024u, v[U + u]);
                                }
                            } else if (play) {
                                // ramp, tail or wrap: the cells inside the launch
                                // (exec-masked; the lane offset stays unwritten)
                                unsigned eq = ep;
#pragma unroll
                                for (int u = 0; u < U; ++u) {
                                    const int tau = sb + u - lane;
                                    const unsigned eq1 = eq + 1u == Lu ? 0u : eq + 1u;
                                    if ((unsigned)tau < (unsigned)K8) st_plain_so(ring, lane16, eq * 1024u, v[u]);
                                    if ((unsigned)(tau - 8) < (unsigned)K8) st_plain_so(ring, lane16, eq1 * 1024u, v[U + u]);
                                    eq = eq1 + 1u == Lu ? 0u : eq1 + 1u;
                                }
                            } else if (sb >= 72 && sb + U <= K8 &&
                                       !any_lane((eA4[k] < 8u) | (eA4[k] + 15u >= Lu))) {
                                // standard layout, full block, no wrap (the
                                // compute waves' former steady block): A at
                                // the lane's entry + u (+ 8 once its column
                                // wraps), B 8 entries below; u * 1 KB as the
                                // scalar offset
                                const unsigned e = eA4[k];
                                const int c0 = (sb - lane) & 7;
                                const int uw8 = c0 == 0 ? 8 : ((8 - c0) & 7);
                                const unsigned rA1 = e * 1024u + lane16, rA2 = rA1 + 8192u, rB1 = rA1 - 8192u;
#pragma unroll
                                for (int u = 0; u < U; ++u) {
                                    o[u] = u < uw8 ? rA1 : rA2;
                                    o[U + u] = u < uw8 ? rB1 : rA1;
                                    st_plain_so(ring, o[u], (unsigned)u * 1024u, v[u]);
                                    st_plain_so(ring, o[U + u], (unsigned)u * 1024u, v[U + u]);
                                }
                                // (per-lane offsets: drained before they are reused)
                                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                                eA4[k] = e + 16u >= Lu ? e + 16u - Lu : e + 16u;
                            } else {
                                unsigned e = eA4[k];
#pragma unroll
                                for (int u = 0; u < U; ++u) {
                                    const int tau = sb + u - lane;
                                    const unsigned eB = e >= 8u ? e - 8u : e + Lu - 8u;
                                    o[u] = (unsigned)tau < (unsigned)K8 ? e * 1024u + lane16 : kOOB;
                                    o[U + u] = (unsigned)(tau - 8) < (unsigned)K8 ? eB * 1024u + lane16 : kOOB;
                                    st_plain(ring, o[u], v[u]);
                                    st_plain(ring, o[U + u], v[U + u]);
                                    e += (tau & 7) == 7 ? 9u : 1u;
                                    if (e >= Lu) e -= Lu;
                                }
                                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                                eA4[k] = e;
                            }
                            ep4[k] = ep + 2u * U >= Lu ? ep + 2u * U - Lu : ep + 2u * U;
                            cp[k] += U;
                            // (the slots' reads have returned -- the stores used
                            // them -- so the compute wave may overwrite them)
                            if (lane == 0) lds_sti(&sm.done[k], cp[k]);
                            any = true;
                        }
                        left |= cp[k] < totalb;
                    }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    keep(x, ox);
                    keep(y, oy);
                    if (!left || lds_ldi(&sm.perm[5])) break;
                    const long long tn = now_rt();
                    if (any) {
                        t_prog = tn;
                    } else {
                        if (tn - t_prog > a.spin_ticks) break;  // (the compute waves time out themselves)
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                return;
            }
            const int totalb = (KW + kWave - 1 + U - 1) / U * U;
            const unsigned Lu = (unsigned)a.L;
            int cp[4] = {0, 0, 0, 0};
            unsigned pw4[4];
            RetCursor rc4[4];
            const bool ret = a.ret_k > 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                pw4[k] = (unsigned)a.origin;
                rc4[k].init(a, W, 0);
            }
            // Store VGPRs: waves k = 0, 2 copy through
            // array x, k = 1, 3 through y, and the wave drains its stores
            // (vmcnt(0)) before it reloads either -- at k = 2 and at the end
            // of a pass -- with both arrays kept live until then.  A full
            // block (every lane inside the launch, no wrap) stores at a lane
            // offset plus a scalar entry offset: no per-lane address math.
            static_assert(U == 8, "store wave: blocks of 8");
            const unsigned lane16 = lane * 16u;
            auto keep = [](const v4u (&v)[U], const unsigned (&o)[U]) {
                asm volatile("" ::"v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]),
                             "v"(v[7]));
                asm volatile("" ::"v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]), "v"(o[4]), "v"(o[5]), "v"(o[6]),
                             "v"(o[7]));
            };
            long long t_prog = now_rt();
            for (;;) {
                bool left = false, any = false;
                v4u x[U], y[U];
                unsigned ox[U], oy[U];  // (per-lane offsets: ramp and tail blocks)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (k == 2) {
                        // (k = 0's and 1's stores complete before x, y are reloaded)
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        keep(x, ox);
                        keep(y, oy);
                    }
                    v4u(&v)[U] = (k & 1) ? y : x;
                    unsigned(&o)[U] = (k & 1) ? oy : ox;
                    if (k >= nval) continue;
                    if (cp[k] < totalb && cp[k] + U <= lds_ldi(&sm.prog[k])) {
                        const __amdgpu_buffer_rsrc_t ring =
                            rsrc(a.ring + (size_t)(ti * ntj + tj0 + k) * a.Lt * kWave, (size_t)a.Lt * kWave * 16);
                        unsigned e = ret ? rc4[k].next(a, W, U) : pw4[k];
#pragma unroll
                        for (int u = 0; u < U; ++u) v[u] = lds_ld(&sm.st[k][(cp[k] + u) & (W - 1)][lane]);
                        // (a retained-window block's U entries are consecutive)
                        if (cp[k] >= kWave && cp[k] + U <= KW && (ret || e + U <= Lu)) {
#pragma unroll
                            for (int u = 0; u < U; ++u) st_plain_so(ring, lane16, (e + u) * 1024u, v[u]);
                            e += U;
                            if (!ret && e == Lu) e = 0u;
                        } else {
#pragma unroll
                            for (int u = 0; u < U; ++u) {
                                const int t = cp[k] + u - lane;
                                o[u] = (unsigned)t < (unsigned)KW ? e * 1024u + lane16 : kOOB;
                                st_plain(ring, o[u], v[u]);
                                e = (!ret && e + 1 == Lu) ? 0u : e + 1;
                            }
                            // (per-lane offsets: drained before they are reused)
                            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        }
                        if (!ret) pw4[k] = e;
                        cp[k] += U;
                        // (the slots' reads have returned -- the stores used
                        // them -- so the compute wave may overwrite them)
                        if (lane == 0) lds_sti(&sm.done[k], cp[k]);
                        any = true;
                    }
                    left |= cp[k] < totalb;
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                keep(x, ox);
                keep(y, oy);
                if (!left || lds_ldi(&sm.perm[5])) break;
                const long long tn = now_rt();
                if (any) {
                    t_prog = tn;
                } else {
                    if (tn - t_prog > a.spin_ticks) break;  // (the compute waves time out themselves)
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            return;
        }
    }
    if (wave >= nval) return;

    // ================= compute wave =================
    // (BURG_COMPUTE_PRIO: race-screen builds only)
#ifndef BURG_COMPUTE_PRIO
#define BURG_COMPUTE_PRIO 1
#endif
    __builtin_amdgcn_s_setprio(BURG_COMPUTE_PRIO);
    const int k = wave;
    const int tj = tj0 + k;
    const int tile = ti * ntj + tj;
    const bool rowok = lane < nrow;
    const unsigned long long rowmask = __builtin_amdgcn_ballot_w64(rowok);
    const bool has_west = tj > 0;
    const bool has_south = south_dev || south_host;
    const bool east_lds = k < 3 && k + 1 < nval;
    const bool east_glob = k == 3 && tj + 1 < ntj;
    const bool has_north = north_dev || north_host;
    const bool col0_tile = tj == 0;
    const int r = ti * kWave + min(lane, top);
    const double ay = a.cf.alpha * a.cf.inv_dy[r];
    const double hy = 0.5 * ay;
    // inlet term of the lane's trajectory (sweep: lb of trajectory jl, lb_next
    // of jl + 1; qn = first step of trajectory jl + 1, whose W columns read
    // the initial state -- every trajectory starts from w0)
    double lb = SWEEP ? sm.lbt[0][SWEEP ? lane : 0] : a.cf.lbc[r];
    double lb_next = SWEEP ? sm.lbt[min(1, nsw - 1)][SWEEP ? lane : 0] : lb;
    int qn = SWEEP ? a.T : INT_MAX, jl = 0;
    // LDS rows of the src table for trajectories jl and jl + 1 (clamped)
    typedef __attribute__((address_space(3))) const double lds_f64;
    lds_f64 *src_cur = (lds_f64 *)&sm.srcb[0][k][0];
    lds_f64 *src_nxt = (lds_f64 *)&sm.srcb[min(1, nsw - 1)][k][0];
    const __amdgpu_buffer_rsrc_t ring = rsrc(a.ring + (size_t)tile * a.Lt * kWave,
                                             (size_t)a.Lt * kWave * 16);
    const __amdgpu_buffer_rsrc_t wbox = rsrc(a.wbox, a.wbox_bytes);
    // north outflow target: the north tile's south box, or the halo ring
    const __amdgpu_buffer_rsrc_t nrs = north_host ? rsrc(a.halo_out, a.halo_bytes)
                                                  : rsrc(a.sbox, a.sbox_bytes);
    const unsigned lane16 = lane * 16u;
    // outbound bases (slot offsets added per step)
    const unsigned eb = ((unsigned)(tile + 1) * kR * kWave + lane) * G;  // east tile's west box
    const unsigned nb = north_dev ? (unsigned)(tile + ntj) * kR * W * G
                                  : (unsigned)tj * W * 16u;                // + c
    const unsigned nstep = north_dev ? (unsigned)W * G : (unsigned)hcols * 16u;
    const int ncol_real = north_host ? hcols - tj * W : W;  // columns with a halo slot
    const unsigned ncol = north_dev ? G : 16u;
    LDS v4u(*src_w)[kWave] = k == 0 ? sm.inw : sm.ewe[k - 1];
    LDS v4u *const my_st = &sm.st[k][0][0];
    LDS v4u *const my_st0 = &sm.st0[k][0][0];
    const unsigned Lu = (unsigned)a.L;  // < 2^21 entries (one descriptor)
    unsigned pw = (unsigned)a.origin;
    // retained windows (a.ret_k > 0): the ring entry of each block's first
    // diagonal comes from the walk (set at the block start)
    const bool ret = a.ret_k > 0;
    RetCursor rcur;
    rcur.init(a, W, 0);
    const v4u lempty = lds_empty_g();

    if constexpr (PAIR) {
        // ============ paired halves ============
        // Lane r at paired diagonal s: local time tau = s - r; half A works
        // on column tau mod 8 of step tau / 8, half B on column 8 + tau mod 8
        // of the step before.  A's west inflow: the tile's west edge at its
        // column 0, else its own east outflow of the previous diagonal; B's:
        // A's east outflow of the previous diagonal at column 8 (A's column 7
        // of the same step), else its own.  South: lane r - 1's north outflow
        // of the previous diagonal (lane 0: the south inbox, stream index
        // 16 step + column).  Previous states: LDS slot s mod 8 (A) and 8 +
        // s mod 8 (B), written 8 paired diagonals earlier (PSW: written to
        // slots s mod 16 and 16 + s mod 16, read 8 diagonals later from
        // the other half -- the store wave copies a block out while the
        // next one runs).  The ring keeps the standard W = 16 layout
        // (extraction unchanged): the A cell of (step q, column c) at
        // diagonal 16 q + c + r, per lane.
        static_assert(W == 16 && U == 8, "paired halves: W = 16, blocks of 8");
        LDS int *const sink = (LDS int *)&sm.dump[lane & (Img::kDump - 1)];
        LDS v4u *const dumpv = &sm.dump[lane & (Img::kDump - 1)];
        const int K8 = 8 * K;
        const int total2 = K8 + 8 + kWave - 1;  // lane 63's B cell ends at local time 8K + 7
        long long e0l = (long long)a.origin + 16LL * ((-lane) >> 3) + ((-lane) & 7) + lane;
        e0l %= a.L;
        if (e0l < 0) e0l += a.L;
        unsigned eA = (unsigned)e0l;  // ring entry of the lane's A cell (+1 per diagonal, +9 past column 7)
        double eAx = 0.0, eAy = 0.0, eBx = 0.0, eBy = 0.0;  // east outflows, previous diagonal
        double nAx = 0.0, nAy = 0.0, nBx = 0.0, nBy = 0.0;  // north outflows, previous diagonal
        // sweeps: each half's trajectory (B trails A by one step, so it
        // switches to the next trajectory 8 diagonals later): inlet terms,
        // source rows, first step of the next trajectory (its W columns read
        // the initial state: st0, or PSW the uniform initial state w0c)
        // (B is never at the domain's column 0: no inlet term of its own)
        double lbA = lb, lbA_next = lb_next;
        int qnA = qn, qnB = qn, jlA = 0, jlB = 0;
        lds_f64 *srcA_cur = src_cur, *srcA_nxt = src_nxt, *srcB_cur = src_cur, *srcB_nxt = src_nxt;
        unsigned long long pspins = 0, pslow = 0, pieee = 0, pnonfin = 0, pwait = 0;
        unsigned pwhy[5] = {0, 0, 0, 0, 0};
        bool paborted = false;
        // the previous paired diagonal's store data and offsets, kept live
        // until this one's stores (store VGPRs: see launder)
        v4u kq_a = v4u{0u, 0u, 0u, 0u}, kq_b = kq_a, kq_e = kq_a, kq_na = kq_a, kq_nb = kq_a;
        unsigned kq_ra = 0u, kq_rb = 0u, kq_eo = 0u, kq_oa = 0u, kq_ob = 0u;
        auto keep_prev = [&]() {
            if constexpr (PSW)
                asm volatile("" ::"v"(kq_e), "v"(kq_na), "v"(kq_nb), "v"(kq_eo), "v"(kq_oa), "v"(kq_ob));
            else
                asm volatile("" ::"v"(kq_a), "v"(kq_b), "v"(kq_e), "v"(kq_na), "v"(kq_nb), "v"(kq_ra), "v"(kq_rb),
                             "v"(kq_eo), "v"(kq_oa), "v"(kq_ob));
        };
        const v4u w0c = v4u{a.w0c[0], a.w0c[1], a.w0c[2], a.w0c[3]};  // (PSW sweeps)
        // missing inflows / grants of block [sb, sb + 8): name_it = false: any
        // (one ballot); true: the kinds (bits as err[3] >> 8)
        auto missing2 = [&](int sb, bool name_it) -> unsigned {
            const int t0 = sb - lane, c0 = t0 & 7;
            const int uw = (8 - c0) & 7, tw = t0 + uw;  // the lane's A column 0 in the block
            const bool nw = has_west & ((unsigned)tw < (unsigned)K8) & rowok;
            const v4u gw = lds_ld(&src_w[(tw >> 3) & (kRL - 1)][lane]);
            const bool miss_w = nw & !l_is_data(gw);
            const int d = 2 * sb - 8 + lane;  // lanes 0-15: the block's 16 south stream indices
            const unsigned hs = lds_ld32((const LDS char *)&sm.ins[k][d & (kNI - 1)] + 4);
            const bool miss_s = has_south & (lane < 16) & (d >= 0) & (d < KW) & (hs == kLdsEmptyHi);
            const int ue = (7 - c0) & 7, te = t0 + ue, qe = (te >> 3) - 1;  // B column 15 (step qe)
            const bool oe = ((unsigned)qe < (unsigned)K) & rowok;
            const unsigned he = lds_ld32((const LDS char *)&sm.ewe[east_lds ? k : 0][qe & (kRL - 1)][lane] + 4);
            const int pe = lds_ldi(&sm.pe_row[lane]);
            const bool miss_el = oe & east_lds & (he != kLdsEmptyHi);
            const bool miss_eg = oe & east_glob & (qe >= pe);
            const int pn = lds_ldi(&sm.perm[k]);
            const int tt = min(sb + 7 - top, K8 + 7);  // the top lane's last local time in the block
            const int th = min(16 * (tt >> 3) + (tt & 7) - (tt >= K8 ? 8 : 0), KW - 1);
            const bool miss_n = has_north & (tt >= 0) & (th >= pn);
            // PSW: the block overwrites the slots of block sb - 16: copied out?
            const bool miss_sw = PSW && lds_ldi(&sm.done[k]) < sb - 8;
            if (!name_it)
                return (__builtin_amdgcn_ballot_w64(miss_w | miss_s | miss_el | miss_eg | miss_n) != 0) | miss_sw;
            unsigned why = 0;
            if (miss_sw) why |= 64u;
            if (any_lane(miss_w)) why |= 1u;
            if (any_lane(miss_s)) why |= 2u;
            if (any_lane(miss_el)) why |= 4u;
            if (any_lane(miss_eg)) why |= 8u;
            if (any_lane(miss_n)) why |= 16u;
            return why;
        };
        struct In2 {
            v4u xa, xb, ca, cb, gw, gsa, gsb;
            double srca, srcb;  // sweep: the cells' source terms (their trajectory's row)
        };
        auto fetch2 = [&](int s) -> In2 {
            In2 in;
            const int tau = s - lane;
            const int cA = tau & 7, qA = tau >> 3;
            // previous states: slot s mod 8 (PSW: the other half's, (s mod 16) ^ 8)
            const int rA = PSW ? ((s & 15) ^ 8) : (s & 7), rB = (PSW ? 16 : 8) + rA;
            if constexpr (SWEEP) {
                const bool ntA = qA >= qnA, ntB = qA - 1 >= qnB;
                if constexpr (PSW) {
                    in.xa = ntA ? w0c : my_st[rA * kWave + lane];
                    in.xb = ntB ? w0c : my_st[rB * kWave + lane];
                } else {
                    in.xa = (ntA ? my_st0 : my_st)[rA * kWave + lane];
                    in.xb = (ntB ? my_st0 : my_st)[rB * kWave + lane];
                }
                in.srca = (ntA ? srcA_nxt : srcA_cur)[cA];
                in.srcb = (ntB ? srcB_nxt : srcB_cur)[8 + cA];
            } else {
                in.xa = my_st[rA * kWave + lane];
                in.xb = my_st[rB * kWave + lane];
                in.srca = in.srcb = 0.0;
            }
            in.ca = sm.cc[k][cA];
            in.cb = sm.cc[k][8 + cA];
            const bool need_w = has_west & (cA == 0) & ((unsigned)tau < (unsigned)K8) & rowok;
            in.gw = lds_ld(need_w ? &src_w[qA & (kRL - 1)][lane] : &sm.zero);
            const int dA0 = 16 * (s >> 3) + (s & 7);  // lane 0's stream indices: A, and B = A - 8
            in.gsa = lds_ld((has_south & (s < K8)) ? &sm.ins[k][dA0 & (kNI - 1)] : &sm.zero);
            in.gsb = lds_ld((has_south & (s >= 8) & (s - 8 < K8)) ? &sm.ins[k][(dA0 - 8) & (kNI - 1)] : &sm.zero);
            return in;
        };
        auto mkpre = [&](const v4u xv, const v4u cv, double srcc, bool inlet, double lbu) -> MarchCell::Pre {
            const d2 x = as_d2(xv), co = as_d2(cv);
            MarchCell::Pre p;
            const double pu = x.x, pv = x.y;
            const double hx = co.x, ax = hx + hx;  // exact: hx = 0.5 * (alpha * inv_dx)
            const double sl = inlet ? srcc + lbu : srcc;
            p.hx = hx;
            const double hu = 0.5 * pu;
            p.xfp = ax * (hu * pu);
            p.xhp = ax * (hu * pv);
            p.yhp = ay * (hu * pv);
            p.ygp = ay * ((0.5 * pv) * pv);
            p.bu = ((pu - p.xfp) - p.yhp) + sl;
            p.bv = (pv - p.ygp) - p.xhp;
            return p;
        };
        auto diag2 = [&](const int s, const In2 &in) {
            const int tau = s - lane;
            const int cA = tau & 7, qA = tau >> 3, qB = qA - 1;
            const bool vA = (unsigned)tau < (unsigned)K8;
            const bool vB = (unsigned)(tau - 8) < (unsigned)K8;
            const bool at0 = cA == 0, atE = cA == 7;
            const bool ntA = SWEEP && qA >= qnA, ntB = SWEEP && qB >= qnB;
            const double lbuA = ntA ? lbA_next : lbA;
            const MarchCell::Pre pa = mkpre(in.xa, in.ca, SWEEP ? in.srca : as_d2(in.ca).y, col0_tile & at0, lbuA);
            const MarchCell::Pre pb = mkpre(in.xb, in.cb, SWEEP ? in.srcb : as_d2(in.cb).y, false, 0.0);
            const MarchCell::Row rw{ay, hy, lbuA};
            const d2 g = as_d2(in.gw);
            const double wa0 = at0 ? g.x : eAx, wa1 = at0 ? g.y : eAy;
            const double wb0 = at0 ? eAx : eBx, wb1 = at0 ? eAy : eBy;
            const d2 sa = as_d2(in.gsa), sb2 = as_d2(in.gsb);
            const double na0 = shr1_or(sa.x, nAx), na1 = shr1_or(sa.y, nAy);
            const double nb0 = shr1_or(sb2.x, nBx), nb1 = shr1_or(sb2.y, nBy);
            double oeA0, oeA1, onA0, onA1, oA0, oA1, oeB0, oeB1, onB0, onB1, oB0, oB1;
            bool okA, okB;
            MarchCell::chain<true>(pa, rw, wa0, wa1, na0, na1, oeA0, oeA1, onA0, onA1, oA0, oA1, okA);
            MarchCell::chain<true>(pb, rw, wb0, wb1, nb0, nb1, oeB0, oeB1, onB0, onB1, oB0, oB1, okB);
            const unsigned long long badA =
                __builtin_amdgcn_ballot_w64(!okA) & __builtin_amdgcn_ballot_w64(vA) & rowmask;
            const unsigned long long badB =
                __builtin_amdgcn_ballot_w64(!okB) & __builtin_amdgcn_ballot_w64(vB) & rowmask;
            if (__builtin_expect(badA != 0, 0)) {
                MarchCell::chain<false>(pa, rw, wa0, wa1, na0, na1, oeA0, oeA1, onA0, onA1, oA0, oA1, okA);
                ++pieee;
                if (__any(vA && rowok && !(__builtin_isfinite(oA0) && __builtin_isfinite(oA1)))) ++pnonfin;
            }
            if (__builtin_expect(badB != 0, 0)) {
                MarchCell::chain<false>(pb, rw, wb0, wb1, nb0, nb1, oeB0, oeB1, onB0, onB1, oB0, oB1, okB);
                ++pieee;
                if (__any(vB && rowok && !(__builtin_isfinite(oB0) && __builtin_isfinite(oB1)))) ++pnonfin;
            }
            eAx = oeA0;
            eAy = oeA1;
            eBx = oeB0;
            eBy = oeB1;
            nAx = onA0;
            nAy = onA1;
            nBx = onB0;
            nBy = onB1;
            // ---- outputs (a half that has not started keeps its step-0 state)
            const v4u outA = as_v4u(oA0, oA1), outB = as_v4u(oB0, oB1);
            const int wA = PSW ? (s & 15) : (s & 7), wB = (PSW ? 16 : 8) + wA;
            if (tau >= 0) my_st[wA * kWave + lane] = outA;
            if (tau >= 8) my_st[wB * kWave + lane] = outB;
            keep_prev();
            unsigned ra = kOOB, rb = kOOB;
            v4u ka = outA, kb = outB;
            if constexpr (!PSW) {  // (PSW: the store wave stores them)
                const unsigned eB = eA >= 8u ? eA - 8u : eA + Lu - 8u;
                ra = vA ? eA * 1024u + lane16 : kOOB;
                rb = vB ? eB * 1024u + lane16 : kOOB;
                launder(ra);
                launder(rb);
                st_plain(ring, ra, ka);
                st_plain(ring, rb, kb);
                eA += atE ? 9u : 1u;
                if (eA >= Lu) eA -= Lu;
            }
            // east edge: B's column 15 (step qB)
            const bool out_e = atE & vB & rowok;
            v4u eo = as_v4u(oeB0, oeB1);
            if (east_lds) lds_st(out_e ? &sm.ewe[k][qB & (kRL - 1)][lane] : dumpv, eo);
            unsigned eoff = kOOB;
            if (east_glob) {
                eoff = out_e ? eb + (unsigned)((a.qbase + qB) & (kR - 1)) * (kWave * G) : kOOB;
                launder(eoff);
                st_dev(wbox, eoff, eo);
            }
            unsigned offA = kOOB, offB = kOOB;
            // north edge: the top lane's A (step qA, column cA) and B (qB, 8 + cA)
            // (the kept north data assigned on every path: a value kept only
            // on some paths is copied into a loop register of its own, and
            // the store then reads the copy's source -- unkept)
            kq_na = as_v4u(onA0, onA1);
            kq_nb = as_v4u(onB0, onB1);
            if (has_north) {
                const bool tl = lane == top;
                offA = (tl & vA & (cA < ncol_real))
                           ? nb + (unsigned)((a.qbase + qA) & (kR - 1)) * nstep + (unsigned)cA * ncol
                           : kOOB;
                offB = (tl & vB & (8 + cA < ncol_real))
                           ? nb + (unsigned)((a.qbase + qB) & (kR - 1)) * nstep + (unsigned)(8 + cA) * ncol
                           : kOOB;
                launder(offA);
                launder(offB);
                st_sys(nrs, offA, kq_na);
                st_sys(nrs, offB, kq_nb);
            }
            kq_a = ka;
            kq_b = kb;
            kq_e = eo;
            kq_ra = ra;
            kq_rb = rb;
            kq_eo = eoff;
            kq_oa = offA;
            kq_ob = offB;
            // the consumed west granule back to empty
            if (has_west) {
                const bool need_w = at0 & vA & rowok;
                lds_st(need_w ? &src_w[qA & (kRL - 1)][lane] : dumpv, lempty);
            }
            if constexpr (SWEEP) {
                // a half that finished the first step of its next trajectory switches
                if (ntA && atE) {
                    ++jlA;
                    qnA += a.T;
                    lbA = lbA_next;
                    srcA_cur = srcA_nxt;
                    const int jn = min(jlA + 1, nsw - 1);
                    lbA_next = sm.lbt[jn][SWEEP ? lane : 0];
                    srcA_nxt = (lds_f64 *)&sm.srcb[jn][k][0];
                }
                if (ntB && atE) {
                    ++jlB;
                    qnB += a.T;
                    srcB_cur = srcB_nxt;
                    srcB_nxt = (lds_f64 *)&sm.srcb[min(jlB + 1, nsw - 1)][k][0];
                }
            }
        };
        // Steady block: a full strip, every lane's A and B inside the
        // launch for all 8 diagonals, no ring wrap, no trajectory switch.
        // Every lane then meets A's column 0 exactly once (diagonal uw of the
        // block; A's column 7 = B's column 15 one before it), so the west
        // granule is read once, the hand-off targets are fixed per block, the
        // state slots and south inbox entries sit at constant offsets, and
        // nothing is masked.
        auto steady2 = [&](const int sb) {
            const int t0 = sb - lane, c0 = t0 & 7, q0 = t0 >> 3;
            const int uw = (8 - c0) & 7;           // A at column 0
            const int uw8 = c0 == 0 ? 8 : uw;      // A's step advances from here (8: not in this block)
            const int ue = (uw + 7) & 7;           // A at column 7, B at column 15
            const int qw = q0 + (c0 == 0 ? 0 : 1);  // A's step at its column 0
            const int qe = ((t0 + ue) >> 3) - 1;    // B's step at its column 15
            const v4u gw = lds_ld(has_west ? &src_w[qw & (kRL - 1)][lane] : &sm.zero);
            LDS v4u *const eaddr = east_lds ? &sm.ewe[k][qe & (kRL - 1)][lane] : dumpv;
            const unsigned eoff = east_glob ? eb + (unsigned)((a.qbase + qe) & (kR - 1)) * (kWave * G) : kOOB;
            // ring: A's entry at diagonal u is eA + u (+ 8 from uw8 on); B's is 8 below
            // (rA*: byte offsets -- not oA*, the cells' outputs below)
            const unsigned rA1 = eA * 1024u + lane16, rA2 = rA1 + 8192u;
            // north (top lane): A at (step, column) = (q0, c0 + u) before uw8, (q0 + 1, c0 + u - 8)
            // after; B one step earlier at column 8 + that
            const bool tl = has_north & (lane == top);
            const unsigned sq0 = (unsigned)((a.qbase + q0) & (kR - 1)) * nstep;
            const unsigned sq1 = (unsigned)((a.qbase + q0 + 1) & (kR - 1)) * nstep;
            const unsigned sqm = (unsigned)((a.qbase + q0 - 1) & (kR - 1)) * nstep;
            const unsigned nA1 = tl ? nb + sq0 + (unsigned)c0 * ncol : kOOB;
            const unsigned nA2 = tl ? nb + sq1 + (unsigned)c0 * ncol - 8u * ncol : kOOB;
            const unsigned nB1 = tl ? nb + sqm + (unsigned)(8 + c0) * ncol : kOOB;
            const unsigned nB2 = tl ? nb + sq0 + (unsigned)c0 * ncol : kOOB;
            const int m16 = 2 * sb;  // lane 0's stream index of A at u = 0 (16 (sb / 8))
            const LDS v4u *const insA = has_south ? &sm.ins[k][m16 & (kNI - 1)] : &sm.win[0][0][0];
            const LDS v4u *const insB = has_south ? &sm.ins[k][(m16 - 8) & (kNI - 1)] : &sm.win[0][0][0];
            const double lbuA = SWEEP ? lbA : lb;  // (sweep: the lane's current trajectory's inlet term)
            // state slots: read u, write u (PSW: write (sb mod 16) + u, read the other half)
            const int swA = PSW ? (sb & 8) : 0, srA = PSW ? (swA ^ 8) : 0, oB = PSW ? 16 : 8;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int ci = (c0 + u) & 7;
                const bool at0 = u == uw, atE = u == ue;
                const v4u xa = my_st[(srA + u) * kWave + lane], xb = my_st[(oB + srA + u) * kWave + lane];
                const v4u ca = sm.cc[k][ci], cb = sm.cc[k][8 + ci];
                // (volatile: the comm wave deposits these -- a plain load could be
                // hoisted above the readiness wait)
                const v4u gsa = lds_ld(insA + u), gsb = lds_ld(insB + u);
                double srca = 0.0, srcb = 0.0;
                if constexpr (SWEEP) {
                    srca = srcA_cur[ci];
                    srcb = srcB_cur[8 + ci];
                }
                const MarchCell::Pre pa = mkpre(xa, ca, SWEEP ? srca : as_d2(ca).y, col0_tile & at0, lbuA);
                const MarchCell::Pre pb = mkpre(xb, cb, SWEEP ? srcb : as_d2(cb).y, false, 0.0);
                const MarchCell::Row rw{ay, hy, lbuA};
                const d2 g = as_d2(gw);
                const double wa0 = at0 ? g.x : eAx, wa1 = at0 ? g.y : eAy;
                const double wb0 = at0 ? eAx : eBx, wb1 = at0 ? eAy : eBy;
                const d2 sa = as_d2(gsa), sb2 = as_d2(gsb);
                const double na0 = shr1_or(sa.x, nAx), na1 = shr1_or(sa.y, nAy);
                const double nb0 = shr1_or(sb2.x, nBx), nb1 = shr1_or(sb2.y, nBy);
                double oeA0, oeA1, onA0, onA1, oA0, oA1, oeB0, oeB1, onB0, onB1, oB0, oB1;
                bool okA, okB;
                MarchCell::chain<true>(pa, rw, wa0, wa1, na0, na1, oeA0, oeA1, onA0, onA1, oA0, oA1, okA);
                MarchCell::chain<true>(pb, rw, wb0, wb1, nb0, nb1, oeB0, oeB1, onB0, onB1, oB0, oB1, okB);
                if (__builtin_expect(__builtin_amdgcn_ballot_w64(!(okA & okB)) != 0, 0)) {
                    // (both halves redone with IEEE sqrt / division: same bits where the fast path held)
                    MarchCell::chain<false>(pa, rw, wa0, wa1, na0, na1, oeA0, oeA1, onA0, onA1, oA0, oA1, okA);
                    MarchCell::chain<false>(pb, rw, wb0, wb1, nb0, nb1, oeB0, oeB1, onB0, onB1, oB0, oB1, okB);
                    pieee += 2;
                    if (__any(!(__builtin_isfinite(oA0) && __builtin_isfinite(oA1) && __builtin_isfinite(oB0) &&
                                __builtin_isfinite(oB1))))
                        ++pnonfin;
                }
                eAx = oeA0;
                eAy = oeA1;
                eBx = oeB0;
                eBy = oeB1;
                nAx = onA0;
                nAy = onA1;
                nBx = onB0;
                nBy = onB1;
                const v4u outA = as_v4u(oA0, oA1), outB = as_v4u(oB0, oB1);
                my_st[(swA + u) * kWave + lane] = outA;
                my_st[(oB + swA + u) * kWave + lane] = outB;
                keep_prev();
                unsigned rA = kOOB, rB = kOOB;
                v4u ka = outA, kb = outB;
                if constexpr (!PSW) {  // (PSW: the store wave stores them)
                    rA = (u < uw8 ? rA1 : rA2) + (unsigned)u * 1024u;
                    rB = rA - 8192u;
                    launder(rA);
                    launder(rB);
                    st_plain(ring, rA, ka);
                    st_plain(ring, rB, kb);
                }
                v4u eo = as_v4u(oeB0, oeB1);
                lds_st(atE ? eaddr : dumpv, eo);
                unsigned eo_off = atE ? eoff : kOOB;
                if (east_glob) {
                    launder(eo_off);
                    st_dev(wbox, eo_off, eo);
                }
                unsigned oa = (u < uw8 ? nA1 : nA2) + (unsigned)u * ncol;
                unsigned ob = (u < uw8 ? nB1 : nB2) + (unsigned)u * ncol;
                v4u na = as_v4u(onA0, onA1), nbv = as_v4u(onB0, onB1);
                launder(oa);
                launder(ob);
                st_sys(nrs, oa, na);
                st_sys(nrs, ob, nbv);
                kq_a = ka;
                kq_b = kb;
                kq_e = eo;
                kq_na = na;
                kq_nb = nbv;
                kq_ra = rA;
                kq_rb = rB;
                kq_eo = eo_off;
                kq_oa = oa;
                kq_ob = ob;
            }
            if (has_west) lds_st(&src_w[qw & (kRL - 1)][lane], lempty);
            if constexpr (!PSW) {
                eA += 16u;
                if (eA >= Lu) eA -= Lu;
            }
        };
        __builtin_amdgcn_s_waitcnt(0);  // (the prologue's global loads land here)
        for (int sb = 0; sb < total2; sb += U) {
            lds_sti(lane == 0 ? &sm.prog[k] : sink, sb);
            if (__builtin_expect(missing2(sb, false) != 0, 0)) {
                long long t0 = 0;
                unsigned long long c0 = 0;
                bool waited = false, wsouth = false;
                for (;;) {
                    const unsigned why = missing2(sb, true);
                    if (!why) break;
                    if (!waited) {
                        waited = true;
                        t0 = now_rt();
                        c0 = __builtin_amdgcn_s_memtime();
                        ++pslow;
                        pwhy[0] += (why & 12u) != 0;
                        pwhy[1] += (why & 16u) != 0;
                        pwhy[2] += (why & 1u) != 0;
                        pwhy[3] += (why & 2u) != 0;
                        pwhy[4] += (why & 64u) != 0;  // the store wave (PSW)
                        wsouth = (why & 2u) != 0;
                    } else if (lds_ldi(&sm.perm[5]) || now_rt() - t0 > a.spin_ticks) {
                        if (lane == 0 && !lds_ldi(&sm.perm[5])) {
                            lds_sti(&sm.perm[5], 1);
                            if (atomicOr(a.err, 1u) == 0) {
                                set_err3(a.err, (unsigned)tile, (unsigned)sb, 32u | (why << 8));
                            }
                        }
                        paborted = true;
                        break;
                    }
                    ++pspins;
                    __builtin_amdgcn_s_sleep(1);
                }
                if (waited) {
                    pwait += __builtin_amdgcn_s_memtime() - c0;
                    if (wsouth && lane == 0) diag_south_wait(a, south_host, t0);
                }
                if (paborted) break;
            }
            if (sb == 0 && lane == 0) diag_first(a, south_host);
            bool steady = (a.pair == 1) & (nrow == kWave) & (sb >= 72) & (sb + U <= K8) & (!has_north | (ncol_real >= W));
            if constexpr (!PSW) steady = steady & !any_lane((eA < 8u) | (eA + 15u >= Lu));
            if constexpr (SWEEP)
                steady = steady & !any_lane((((sb + U - 1 - lane) >> 3) >= qnA) | ((((sb + U - 1 - lane) >> 3) - 1) >= qnB));
            if (steady) {
                steady2(sb);
            } else if constexpr (SWEEP) {
                // (inputs read after the previous diagonal: a trajectory switch
                // there decides which state and source row this one reads)
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const In2 cur = fetch2(sb + u);
                    diag2(sb + u, cur);
                }
            } else {
                In2 cur = fetch2(sb);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    In2 nxt;
                    if (u + 1 < U) nxt = fetch2(sb + u + 1);
                    diag2(sb + u, cur);
                    if (u + 1 < U) cur = nxt;
                }
            }
            // the block's south inbox slots back to empty: lane i frees index 2 sb - 8 + i
            if (has_south) {
                const int d = 2 * sb - 8 + lane;
                lds_st(((lane < 16) & (d >= 0) & (d < KW)) ? &sm.ins[k][d & (kNI - 1)] : dumpv, lempty);
            }
        }
        // (PSW: the store wave copies up to the last block)
        if constexpr (PSW) lds_sti(lane == 0 ? &sm.prog[k] : sink, total2 + U);
        if (lane == 0) {
            if (pspins) atomicAdd(&a.stats->stall_spins, pspins);
            if (pslow) atomicAdd(&a.stats->slow_diagonals, pslow);
            if (pieee) atomicAdd(&a.stats->ieee_diagonals, pieee);
            if (pnonfin) atomicAdd(&a.stats->nonfinite_diagonals, pnonfin);
            if (pwait) atomicAdd(&a.stats->slow_ticks, pwait);
            for (int i = 0; i < 5; ++i)
                if (pwhy[i]) atomicAdd(&a.stats->why[i], (unsigned long long)pwhy[i]);
            diag_south_blocks(a, south_host, pwhy[3]);
            atomicAdd(&a.stats->tile_steps, (unsigned long long)K);
        }
        return;
    }

    double e0 = 0.0, e1 = 0.0, no0 = 0.0, no1 = 0.0;
    // the previous diagonal's store data and offsets, kept live until this
    // diagonal's stores (store VGPRs: see launder)
    v4u kp_out = v4u{0u, 0u, 0u, 0u}, kp_e = kp_out, kp_n = kp_out;
    unsigned kp_ro = 0u, kp_eo = 0u, kp_no = 0u;
    unsigned long long spins = 0, slow_n = 0, ieee_n = 0, nonfin_n = 0, wait_ticks = 0;
    unsigned wait_why[5] = {0, 0, 0, 0, 0};  // blocks that waited, by first missing kind
    bool aborted = false;


    // LDS inputs of diagonal s (read at the end of diagonal s - 1, or after
    // the block's readiness check for the first diagonal of a block)
    struct In {
        v4u xs, cs, gw, gs;
        bool nt;     // sweep: first step of the lane's next trajectory (state reset)
        double src;  // sweep: the column's source term of the step's trajectory
    };
    // EDGE: some lane of the block may sit at column 0 or W-1 (west inflow,
    // east outflow); interior blocks of wide tiles (W >= 128: 64 lanes cover
    // at most 64 consecutive columns) skip that work altogether
    // STEADY: an interior block of a full strip with every lane inside the
    // launch's time range, no ring wrap and no north-column wrap in the block
    // -- no validity masks, ring and north store offsets in SGPRs
    typedef std::integral_constant<int, 0> Edge;
    typedef std::integral_constant<int, 1> Interior;
    typedef std::integral_constant<int, 2> Steady;
    // SteadyEdge: a wide-tile edge block (W > 64) with the steady conditions:
    // each lane meets column 0 and column W-1 at most once in the block, at
    // block-constant diagonals (uw, ue) and steps -- its west granule is read
    // once, its hand-off addresses are fixed, the inputs come by block base
    typedef std::integral_constant<int, 3> SteadyEdge;
    typedef std::integral_constant<int, 4> SteadyEdgeG;  // (the east wave's build)
    int se_uw = U, se_ue = U;  // SteadyEdge: the lane's column-0 / column-(W-1) diagonal in the block
    v4u se_gw = v4u{0u, 0u, 0u, 0u};
    LDS v4u *se_eaddr = nullptr;
    unsigned se_eoff = kOOB;
    // steady blocks: the top lane's north slot offset at the block's first
    // diagonal, and (noffs2) at column 0 of the next step, reached at
    // diagonal uwrap of the block (>= U: no wrap in the block)
    unsigned noffs = 0, noffs2 = 0;
    int uwrap = U;
    // narrow steady-edge blocks: the north slot offsets as per-lane values
    // (kOOB on every lane but a north-writing top lane: no scalar state, no
    // branch), and the inlet term added at column 0 (0 off the inlet tile)
    unsigned nv1 = kOOB, nv2 = kOOB;
    double lb_se = 0.0;
    // narrow steady-edge blocks (BURG_SE_OPT): the column-0 source plus the
    // inlet term, added once per block (the diagonal selects it at column 0)
    double src0_se = 0.0;
    // a column's {hx, src}; sweeps take src from their per-trajectory tables,
    // so they load hx alone (a dead src half would be a register the compiler
    // reuses while the load is in flight: an LDS wait per diagonal)
    auto cc_ld = [&](const LDS v4u *p) -> v4u {
        if constexpr (SWEEP) {
            typedef unsigned v2u __attribute__((ext_vector_type(2)));
            const v2u x = *(const LDS v2u *)p;
            return v4u{x.x, x.y, 0u, 0u};
        } else {
            return *p;
        }
    };

    auto fetch = [&](auto edge_tag, int s) -> In {
        constexpr bool EDGE = decltype(edge_tag)::value == 0;
        constexpr bool STEADY = decltype(edge_tag)::value >= 2;
        const int t = s - lane;
        const int c = t & (W - 1);
        const int q = t >> LW;
        const bool valid = (unsigned)t < (unsigned)KW;
        const bool need_w = has_west & (c == 0) & valid & rowok;
        In in;
        if constexpr (SWEEP) {
            in.nt = q >= qn;
            in.xs = (in.nt ? my_st0 : my_st)[(s & (W - 1)) * kWave + lane];
            in.src = (in.nt ? src_nxt : src_cur)[c];
        } else if constexpr (!WIDE) {
            in.nt = false;
            in.xs = my_st[(s & (W - 1)) * kWave + lane];
            in.src = 0.0;
        } else {
            in.nt = false;
            in.src = 0.0;
            in.xs = lds_ld(&sm.win[k][s % KWIN][lane]);
        }
        in.cs = cc_ld(&sm.cc[k][t & (ccn_of<W>() - 1)]);  // (= c unless ccw_of)
        if constexpr (EDGE) in.gw = lds_ld(need_w ? &src_w[q & (kRL - 1)][lane] : &sm.zero);
        else in.gw = v4u{0u, 0u, 0u, 0u};
        in.gs = lds_ld((has_south & (STEADY || s < KW)) ? &sm.ins[k][s & (kNI - 1)] : &sm.zero);
        return in;
    };

    // Wide interior / steady blocks: no lane wraps a column inside the block,
    // and the block starts at a multiple of U in the window (16) and south
    // inbox (64) rings, so diagonal sb + u reads base + u -- the offsets fold
    // into the LDS instructions' immediate fields.
    struct Bases {
        LDS v4u *wb, *cb, *ib;
        lds_f64 *sr;  // sweep: the lane's source row at its first column of the block
        int c0;  // the lane's column at the block's first diagonal
    };
    auto bases_of = [&](int sb) -> Bases {
        Bases b;
        // narrow tiles: the lane's previous states in st (slot s mod W; a block
        // starts at a multiple of U, so sb + u does not wrap)
        if constexpr (WIDE) b.wb = &sm.win[k][sb % KWIN][lane];
        else b.wb = (LDS v4u *)&my_st[(sb & (W - 1)) * kWave + lane];
        b.cb = &sm.cc[k][(sb - lane) & (ccn_of<W>() - 1)];
        b.ib = has_south ? &sm.ins[k][sb & (kNI - 1)] : WIDE ? &sm.zeros[0] : &sm.win[0][0][0];
        b.c0 = (sb - lane) & (W - 1);
        b.sr = src_cur + b.c0;  // (padded row: + u does not wrap)
        return b;
    };
    auto fetch_b = [&](const Bases &b, int u) -> In {
        In in;
        in.nt = false;
        in.src = 0.0;
        if constexpr (SWEEP) in.src = b.sr[u];  // (no trajectory switch in the block)
        in.xs = lds_ld(b.wb + u * kWave);
        in.cs = cc_ld(b.cb + u);
        in.gw = v4u{0u, 0u, 0u, 0u};
        in.gs = lds_ld(b.ib + u);
        return in;
    };
    // the same without the previous state (the kept block: keep_of)
    auto fetch_b_nx = [&](const Bases &b, int u) -> In {
        In in;
        in.nt = false;
        in.src = 0.0;
        in.xs = v4u{0u, 0u, 0u, 0u};
        in.cs = cc_ld(b.cb + u);
        in.gw = v4u{0u, 0u, 0u, 0u};
        in.gs = lds_ld(b.ib + u);
        return in;
    };

    // Readiness of a whole block of diagonals [sb, sb + U): every inflow it
    // consumes is deposited, every outbound slot it fills is granted and (wide
    // tiles) every previous state is in the window.  Checked once per block,
    // so the diagonals themselves run without waits.  Returns the missing
    // kinds (0: ready; bits as err[3] >> 8), wave-uniform.
    auto block_missing = [&](int sb) -> unsigned {
        unsigned why = 0;
        const int t0 = sb - lane;  // the lane's local time at the block's first diagonal
        const int c0 = t0 & (W - 1);
        if (has_west) {  // the lane's column-0 diagonal in the block (U <= W: at most one)
            const int uw = (W - c0) & (W - 1);
            const int tw = t0 + uw;
            const bool nw = (uw < U) & ((unsigned)tw < (unsigned)KW) & rowok;
            const v4u g = lds_ld(&src_w[(tw >> LW) & (kRL - 1)][lane]);
            if (any_lane(nw & !l_is_data(g))) why |= 1u;
        }
        if (has_south) {  // lane i checks the inflow of diagonal sb + i
            const int d = sb + lane;
            const unsigned hi = lds_ld32((const LDS char *)&sm.ins[k][d & (kNI - 1)] + 4);
            if (any_lane((lane < U) & (d < KW) & (hi == kLdsEmptyHi))) why |= 2u;
        }
        const int ue = (W - 1 - c0) & (W - 1);  // the lane's column W-1 diagonal in the block
        const int te = t0 + ue;
        const bool oe = (ue < U) & ((unsigned)te < (unsigned)KW) & rowok;
        if (east_lds) {
            const unsigned hi = lds_ld32((const LDS char *)&sm.ewe[k][(te >> LW) & (kRL - 1)][lane] + 4);
            if (any_lane(oe & (hi != kLdsEmptyHi))) why |= 4u;
        }
        if (east_glob) {
            const int pe = lds_ldi(&sm.pe_row[lane]);
            if (any_lane(oe & ((te >> LW) >= pe))) why |= 8u;
        }
        if (has_north) {  // the top lane's last local time in the block
            const int pn = lds_ldi(&sm.perm[k]);
            const int th = min(sb - top + U - 1, KW - 1);
            if (any_lane((th >= 0) & (th >= pn))) why |= 16u;
        }
        if constexpr (WIDE) {
            if (any_lane(lds_ldi(&sm.filled[k]) < sb + U)) why |= 32u;
        }
        // store wave: the block's slots (diagonals sb - W .. sb - W + U) copied
        if constexpr (!WIDE && store_wave_of<W>()) {
            if (lds_ldi(&sm.done[k]) < sb - W + U) why |= 64u;
        }
        return why;
    };

    // The same test, fused for the common case: every kind's per-lane
    // condition folded into one predicate, read without branches (an LDS load
    // of a kind the wave has no edge for reads a harmless slot) and decided
    // by ONE ballot -- block_missing's per-kind branches and ballots (each an
    // i1 -> VGPR -> compare -> SCC round trip in the compiler's hands) cost
    // tens of instructions per block.  block_missing then only runs when a
    // block has to wait (it names the missing kinds).
    auto block_ready = [&](int sb) -> bool {
        const int t0 = sb - lane;
        const int c0 = t0 & (W - 1);
        const int uw = (W - c0) & (W - 1);
        const int tw = t0 + uw;
        const v4u g = lds_ld(&src_w[(tw >> LW) & (kRL - 1)][lane]);
        const bool miss_w = has_west & (uw < U) & ((unsigned)tw < (unsigned)KW) & rowok & !l_is_data(g);
        const int d = sb + lane;
        const unsigned hs = lds_ld32((const LDS char *)&sm.ins[k][d & (kNI - 1)] + 4);
        const bool miss_s = has_south & (lane < U) & (d < KW) & (hs == kLdsEmptyHi);
        const int ue = (W - 1 - c0) & (W - 1);
        const int te = t0 + ue;
        const bool oe = (ue < U) & ((unsigned)te < (unsigned)KW) & rowok;
        const unsigned he = lds_ld32((const LDS char *)&sm.ewe[east_lds ? k : 0][(te >> LW) & (kRL - 1)][lane] + 4);
        const int pe = lds_ldi(&sm.pe_row[lane]);
        const bool miss_e = oe & ((east_lds & (he != kLdsEmptyHi)) | (east_glob & ((te >> LW) >= pe)));
        const int pn = lds_ldi(&sm.perm[k]);
        const int th = min(sb - top + U - 1, KW - 1);
        const bool miss_n = has_north & (th >= 0) & (th >= pn);
        bool miss = miss_w | miss_s | miss_e | miss_n;
        if constexpr (WIDE) miss = miss | (lds_ldi(&sm.filled[k]) < sb + U);
        if constexpr (!WIDE && store_wave_of<W>()) miss = miss | (lds_ldi(&sm.done[k]) < sb - W + U);
        return __builtin_amdgcn_ballot_w64(miss) == 0;
    };

    // one diagonal, diagonal u of its block (no waits: the block was checked)
    auto diagonal = [&](auto edge_tag, const int s, const int u, In &in) -> v4u {
        constexpr bool EDGE = decltype(edge_tag)::value == 0;
        constexpr bool SE = decltype(edge_tag)::value >= 3;
        // (narrow steady-edge blocks come in two builds: 4 for the
        // workgroup's east wave, whose east outflow goes to the global
        // mailbox, 3 for the others, whose outflow goes to the LDS ring --
        // each issues only its own; wide tiles run 3 only, with both)
        constexpr bool SE_G = decltype(edge_tag)::value == 4;
        constexpr bool STEADY = decltype(edge_tag)::value >= 2;
        const int t = s - lane;
        const int c = t & (W - 1);
        const int q = t >> LW;
        const bool valid = STEADY || (unsigned)t < (unsigned)KW;
        const bool at0 = SE ? u == se_uw : EDGE & (c == 0);
        // (a lane reaches column W-1 one diagonal before column 0: with U < W
        // the compare of diagonal u + 1's at0 serves as this one's atE)
        const bool atE = SE ? ((BURG_SE_OPT && U < W) ? u + 1 == se_uw : u == se_ue)
                            : EDGE & (c == W - 1);
        const bool need_w = has_west & at0 & valid & rowok;
        const bool need_s = has_south & (STEADY || s < KW);  // wave-uniform (lane 0 consumes)
        const bool out_e = atE & valid & rowok;
        const bool out_n = (lane == top) & valid & has_north;
        // ---- inflow-independent part of the cell (MarchCell::pre, same op order)
        const double lbu = SWEEP && in.nt ? lb_next : lb;
        MarchCell::Pre p;
        {
            const d2 x = as_d2(in.xs);
            const d2 co = as_d2(in.cs);
            const double pu = x.x, pv = x.y;
            const double hx = co.x, ax = hx + hx;  // exact: hx = 0.5 * (alpha * inv_dx)
            const double srcc = SWEEP ? in.src : co.y;
            // (narrow steady edge: srcc + 0.0 is srcc exactly -- the source
            // term is positive -- so both forms give the same bits)
            const double sl = (!WIDE && STEADY) ? (BURG_SE_OPT ? (at0 ? src0_se : srcc)
                                                              : srcc + (at0 ? lb_se : 0.0))
                                                : (col0_tile && at0) ? srcc + lbu : srcc;
            p.hx = hx;
            const double hu = 0.5 * pu;
            p.xfp = ax * (hu * pu);
            p.xhp = ax * (hu * pv);
            p.yhp = ay * (hu * pv);
            p.ygp = ay * ((0.5 * pv) * pv);
            p.bu = ((pu - p.xfp) - p.yhp) + sl;
            p.bv = (pv - p.ygp) - p.xhp;
        }
        const MarchCell::Row rw{ay, hy, lbu};
        // ---- the cell's chain
        // (steady blocks: a select, not an exec-masked move -- the compiler
        // guards the masked form with a branch, taken on most diagonals)
        if constexpr (STEADY) {
            const d2 gv = as_d2(SE ? se_gw : in.gw);
            e0 = at0 ? gv.x : e0;
            e1 = at0 ? gv.y : e1;
        } else if (at0) {
            const d2 gv = as_d2(in.gw);
            e0 = gv.x;
            e1 = gv.y;
        }
        const d2 sv = as_d2(in.gs);
        const double n0 = shr1_or(sv.x, no0);
        const double n1 = shr1_or(sv.y, no1);
        double oe0, oe1, on0, on1, o0, o1;
        bool ok;
        MarchCell::chain<true>(p, rw, e0, e1, n0, n1, oe0, oe1, on0, on1, o0, o1, ok);
        // (ballots of the single compares, combined on the scalar unit: a
        // ballot of the combined lane predicate costs a select and a compare)
        // (steady blocks cover full strips: every lane is a row)
        const unsigned long long bad =
            STEADY ? __builtin_amdgcn_ballot_w64(!ok)
                   : __builtin_amdgcn_ballot_w64(!ok) & __builtin_amdgcn_ballot_w64(valid) & rowmask;
        if (__builtin_expect(bad != 0, 0)) {
            MarchCell::chain<false>(p, rw, e0, e1, n0, n1, oe0, oe1, on0, on1, o0, o1, ok);
            ++ieee_n;
            // the only place a non-finite state can appear (the fast path's
            // operands and results are finite by its range check)
            if (__any(valid && rowok && !(__builtin_isfinite(o0) && __builtin_isfinite(o1))))
                ++nonfin_n;
        }
        e0 = oe0;
        e1 = oe1;
        no0 = on0;
        no1 = on1;
        // ---- outputs (lanes that have not started keep their step-0 state)
        const v4u out = as_v4u(o0, o1);
        if constexpr (!WIDE) {
            if (STEADY || t >= 0) my_st[(s & (W - 1)) * kWave + lane] = out;
        }
        // Store VGPRs are not reused before the NEXT diagonal's stores: a
        // buffer store reads its data / offset VGPRs after it issues, and
        // under load on the CU's memory pipeline that read has come after a
        // following VALU overwrote them (round 5: ring entries with u = 0.5
        // -- the next cell's 0.5 * pu -- in lanes 12-15 of every 16, once the
        // comm wave ran at a higher priority)
        asm volatile("" ::"v"(kp_out), "v"(kp_e), "v"(kp_n), "v"(kp_ro), "v"(kp_eo), "v"(kp_no));
        // wide tiles: the loader wave reads this entry back (sc1 DMA) W
        // diagonals later, so it is stored write-through to L2 (sc1): the
        // store's vmcnt then completes at L2, which the done[] protocol needs
        unsigned ro;        // the ring store's voffset
        unsigned eoff = kOOB, noff = kOOB;  // the east / north stores' voffsets
        v4u outk = out;
        if constexpr (!WIDE && store_wave_of<W>()) {
            ro = 0u;  // (the store wave copies the LDS state slots to the ring)
        } else if constexpr (STEADY) {
            ro = lane16;
            launder(ro);
            if constexpr (WIDE) __builtin_amdgcn_raw_buffer_store_b128(outk, ring, ro, pw * 1024u, BURG_RING_AUX);
            else st_plain_so(ring, ro, pw * 1024u, outk);
            ++pw;  // (no wrap inside a steady block)
        } else {
            ro = valid ? pw * 1024u + lane16 : kOOB;
            launder(ro);
            if constexpr (WIDE) __builtin_amdgcn_raw_buffer_store_b128(outk, ring, ro, 0, BURG_RING_AUX);
            else st_plain(ring, ro, outk);
            pw = pw + 1 == Lu ? 0u : pw + 1;
        }
        v4u eo = as_v4u(oe0, oe1);
        const int aq = a.qbase + q;
        // (LDS writes go to a selected address -- a dump slot for lanes
        // that have nothing to write -- instead of an exec-masked branch)
        if constexpr (SE) {
            if constexpr (!SE_G) lds_st(atE ? se_eaddr : &sm.dump[lane & (Img::kDump - 1)], eo);
        } else if constexpr (WIDE) {
            if (EDGE && east_lds) lds_st(out_e ? &sm.ewe[k][q & (kRL - 1)][lane] : &sm.dump[lane & (Img::kDump - 1)], eo);
        } else {
            if (east_lds && out_e) lds_st(&sm.ewe[k][q & (kRL - 1)][lane], eo);
        }
        // wide tiles issue every store on every diagonal (out-of-range offsets
        // are dropped): exactly 3 per edge and 2 per interior diagonal, which
        // the vmcnt of done[] counts
        if constexpr (SE) {
            // (wide: every diagonal issues the same number of stores, for done[];
            // narrow: unconditional too -- se_eoff is out of range unless this is
            // the workgroup's east wave -- a dropped store costs less than the
            // two taken branches around a conditional one)
            if (WIDE || SE_G) {
                eoff = atE ? se_eoff : kOOB;
                launder(eoff);
                st_dev(wbox, eoff, eo);
            }
        }
        else if (EDGE && (WIDE || east_glob)) {
            eoff = east_glob && out_e ? eb + (unsigned)(aq & (kR - 1)) * (kWave * G) : kOOB;
            launder(eoff);
            st_dev(wbox, eoff, eo);
        }
        // (narrow steady blocks store unconditionally: nv1 / nv2 are out of
        // range on every lane but a north-writing top lane)
        if (WIDE || STEADY || has_north) {
            // one store flavour for both targets: sc0 sc1 (system scope) reaches
            // the host / peer halo ring and is write-through like sc1 for the
            // device mailboxes (consumers poll with sc1 / sc0 sc1 loads)
            v4u no = as_v4u(on0, on1);
            if constexpr (STEADY) {
                // the top lane's slot: SGPR offset, advanced one column per diagonal
                if constexpr (WIDE) {
                    noff = (has_north & (lane == top)) ? 0u : kOOB;
                    launder(noff);
                    st_sys_so(nrs, noff, noffs, no);
                    noffs += ncol;
                } else {
                    noff = (u < uwrap ? nv1 : nv2) + (unsigned)u * ncol;
                    launder(noff);
                    st_sys(nrs, noff, no);
                }
            } else {
                noff = (out_n & (c < ncol_real)) ? nb + (unsigned)(aq & (kR - 1)) * nstep + (unsigned)c * ncol
                                                 : kOOB;
                launder(noff);
                st_sys(nrs, noff, no);
            }
            kp_n = no;
        }
        kp_out = outk;
        kp_e = eo;
        kp_ro = ro;
        kp_eo = eoff;
        kp_no = noff;
        // consumed inbound slots back to empty (steady-edge blocks: once per
        // block, run_block)
        if constexpr (WIDE || STEADY) {
            if (EDGE && has_west) lds_st(need_w ? &src_w[q & (kRL - 1)][lane] : &sm.dump[lane & (Img::kDump - 1)], lempty);
            // (the south slots are freed once per block, run_block)
        } else {
            if (need_w) lds_st(&src_w[q & (kRL - 1)][lane], lempty);
            if (need_s && lane == 0) lds_st(&sm.ins[k][s & (kNI - 1)], lempty);
        }
        if constexpr (SWEEP && !STEADY) {
            // the lane finished the first step of its next trajectory: switch
            if (in.nt && atE) {
                ++jl;
                qn += a.T;
                lb = lb_next;
                src_cur = src_nxt;
                const int jn = min(jl + 1, nsw - 1);
                lb_next = sm.lbt[jn][SWEEP ? lane : 0];
                src_nxt = (lds_f64 *)&sm.srcb[jn][k][0];
            }
        }
        (void)u;
        return out;
    };

    // One block: the LDS inputs are read two diagonals ahead (their latency
    // hides behind a whole diagonal of arithmetic); everything a block reads
    // was checked ready by block_missing.  Sweeps read one ahead, after the
    // diagonal: a lane's trajectory switch (in diagonal s) decides which
    // state and source table diagonal s + 1 reads.
    // the kept block's outputs (keep_of: VGPRs, one block per W)
    constexpr int KN = keep_of<W>() ? keep_n_of<W>() : 1;  // kept diagonals of the block
    v4u kr[KN];
#pragma unroll
    for (int u = 0; u < KN; ++u) kr[u] = v4u{0u, 0u, 0u, 0u};
    auto run_block = [&](auto tag, const int sb, auto keep_tag) {
        // KEEP: the kept block -- previous states from kr once the first W
        // diagonals are past (before that the loader read them), outputs to kr
        constexpr bool KEEP = decltype(keep_tag)::value;
        const bool reg_ok = KEEP && sb >= W;
        if constexpr (SWEEP && decltype(tag)::value < 3) {
            In a0 = fetch(tag, sb);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                diagonal(tag, sb + u, u, a0);
                if (u + 1 < U) a0 = fetch(tag, sb + u + 1);
            }
        } else if constexpr ((!WIDE && decltype(tag)::value < 3) || decltype(tag)::value == 0) {
            In a0 = fetch(tag, sb), a1 = fetch(tag, sb + 1);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                In nx;
                if (u + 2 < U) nx = fetch(tag, sb + u + 2);
                diagonal(tag, sb + u, u, a0);
                a0 = a1;
                if (u + 2 < U) a1 = nx;
            }
        } else {
            int se_qw = 0;
            bool se_in = false;
            if constexpr (decltype(tag)::value >= 3) {
                if constexpr (!WIDE) {
                    lb_se = col0_tile ? lb : 0.0;  // (no switch inside)
                    // the same sum the diagonal at column 0 would form:
                    // src + lb_se (+ 0.0 off the inlet tile: src > 0, exact)
                    src0_se = (SWEEP ? src_cur[0] : as_d2(sm.cc[k][0]).y) + lb_se;
                }
                // the lane's column-0 and column-(W-1) cells in this block
                const int c0 = (sb - lane) & (W - 1);
                se_uw = (W - c0) & (W - 1);
                se_ue = (W - 1 - c0) & (W - 1);
                se_qw = (sb + se_uw - lane) >> LW;
                const int qe = (sb + se_ue - lane) >> LW;
                se_in = has_west & (se_uw < U);
                const bool oute = se_ue < U;
                se_gw = lds_ld(se_in ? &src_w[se_qw & (kRL - 1)][lane] : &sm.zero);
                se_eaddr = (east_lds & oute) ? &sm.ewe[k][qe & (kRL - 1)][lane] : &sm.dump[lane & (Img::kDump - 1)];
                se_eoff = (east_glob & oute) ? eb + (unsigned)((a.qbase + qe) & (kR - 1)) * (kWave * G) : kOOB;
            }
            const Bases b = bases_of(sb);
            if constexpr (KEEP) {
                // the first W diagonals: the kept block's previous states came
                // through the loader's window (once per launch)
                if (!reg_ok) {
#pragma unroll
                    for (int u = 0; u < KN; ++u) kr[u] = lds_ld(b.wb + u * kWave);
                }
            }
            // (KEEP: the previous state is kr[u], not loaded into In)
            auto fb = [&](int u) -> In {
                if constexpr (KEEP) {
                    if (u < KN) {
                        In in = fetch_b_nx(b, u);
                        in.xs = kr[u < KN ? u : 0];
                        return in;
                    }
                }
                return fetch_b(b, u);
            };
            In a0 = fb(0), a1 = fb(1);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                In nx;
                if (u + 2 < U) nx = fb(u + 2);
                const v4u o = diagonal(tag, sb + u, u, a0);
                if constexpr (KEEP) {
                    if (u < KN) kr[u < KN ? u : 0] = o;
                }
                a0 = a1;
                if (u + 2 < U) a1 = nx;
            }
            // SteadyEdge: the west granule consumed in this block back to empty
            if (decltype(tag)::value >= 3 && has_west)
                lds_st(se_in ? &src_w[se_qw & (kRL - 1)][lane] : &sm.dump[lane & (Img::kDump - 1)], lempty);
        }
        if constexpr (WIDE || decltype(tag)::value >= 3) {
            // the block's south inbox slots back to empty, one write: lane i
            // frees diagonal sb + i's slot
            if (has_south)
                lds_st(((lane < U) & (sb + lane < KW)) ? &sm.ins[k][(sb + lane) & (kNI - 1)] : &sm.dump[lane & (Img::kDump - 1)],
                       lempty);
        }
    };

    const int total = KW + kWave - 1;
    LDS int *const sink_i = (LDS int *)&sm.dump[lane & (Img::kDump - 1)];
    // Land the prologue's global loads (row coefficients) here: a first use
    // inside the loop would put an s_waitcnt vmcnt(0) -- a wait on every store
    // in flight -- into every diagonal.
    __builtin_amdgcn_s_waitcnt(0);
#ifdef BURG_PIPE_PROF
    unsigned long long pf_vm = 0;
    const unsigned long long pf0 = __builtin_amdgcn_s_memtime();
#endif
    for (int sb = 0; sb < total; sb += U) {
#ifdef BURG_PIPE_PROF
        const unsigned long long pfa = __builtin_amdgcn_s_memtime();
#endif
        if constexpr (WIDE) {
            // every store older than this block's predecessor has completed
            // (2 or 3 stores per diagonal, no loads: waiting down to the smaller
            // count, 2 U, covers both kinds of predecessor): the loader may read
            // ring entries written before diagonal sb - U
            wait_vmcnt<2 * U>();
#ifdef BURG_PIPE_PROF
            pf_vm += __builtin_amdgcn_s_memtime() - pfa;
#endif
            lds_sti(lane == 0 ? &sm.done[k] : sink_i, sb - U);
        }
        // (every lane stores -- lane 0 the progress, the others into their
        // dump slot -- instead of an exec-masked branch around one store)
        lds_sti(lane == 0 ? &sm.prog[k] : sink_i, sb);
        if (__builtin_expect(!block_ready(sb), 0)) {
            // (block_missing runs inside the wait loop, out of the hot path)
            long long t0 = 0;
            unsigned long long c0 = 0;
            bool waited = false, wsouth = false;
            for (;;) {
                const unsigned why = block_missing(sb);
                if (!why) break;
                if (!waited) {
                    waited = true;
                    t0 = now_rt();
                    c0 = __builtin_amdgcn_s_memtime();
                    ++slow_n;
                    wait_why[0] += (why & 12u) != 0;  // east (LDS ring or global grant)
                    wait_why[1] += (why & 16u) != 0;  // north grant
                    wait_why[2] += (why & 1u) != 0;   // west inflow
                    wait_why[3] += (why & 2u) != 0;   // south inflow
                    wait_why[4] += (why & 96u) != 0;  // previous states (loader window) / the store wave
                    wsouth = (why & 2u) != 0;
                } else if (lds_ldi(&sm.perm[5]) || now_rt() - t0 > a.spin_ticks) {
                    if (lane == 0 && !lds_ldi(&sm.perm[5])) {
                        lds_sti(&sm.perm[5], 1);
                        if (atomicOr(a.err, 1u) == 0) {
                            set_err3(a.err, (unsigned)tile, (unsigned)sb, 32u | (why << 8));
                        }
                    }
                    aborted = true;
                    break;
                }
                ++spins;
                __builtin_amdgcn_s_sleep(1);
            }
            if (waited) {
                wait_ticks += __builtin_amdgcn_s_memtime() - c0;
                if (wsouth && lane == 0) diag_south_wait(a, south_host, t0);
            }
            if (aborted) break;
        }
        if (sb == 0 && lane == 0) diag_first(a, south_host);
        // (retained windows: the block's ring entries are consecutive and
        // never wrap; plain ring: wrap checked below)
        if (ret) pw = rcur.next(a, W, U);
        const bool pw_nowrap = ret | (pw + U <= Lu);
        const int sm_ = sb & (W - 1);
        const int tt0 = sb - top, ct0 = tt0 & (W - 1);  // the top lane at the block start
        // (narrow tiles: the top lane's column may wrap to the next step
        // inside the block -- noffs2 -- except on a halo ring, whose row is
        // the whole slab width (and a partial last tile has fewer real
        // columns); wide tiles keep the no-wrap condition: the select would
        // cost more instructions than the 1 in W / U blocks it makes steady)
        // narrow tiles (U <= W: a lane meets column 0 at most once per block)
        // run steady-edge blocks too; sweeps only where no lane is in the
        // first step of its next trajectory (that step reads the initial state)
        // (bitwise, not short-circuit: scalar ops and one branch, not a chain)
        bool steady = (nrow == kWave) & (sb >= kWave) & (sb + U <= KW) & pw_nowrap &
                      ((!WIDE & north_dev) | (ct0 + U <= min(W, ncol_real)));
        if constexpr (SWEEP)
            steady = steady & !any_lane(((sb + U - 1 - lane) >> LW) >= qn);
        if (steady)
        {
            noffs = nb + (unsigned)((a.qbase + (tt0 >> LW)) & (kR - 1)) * nstep + (unsigned)ct0 * ncol;
            noffs2 = nb + (unsigned)((a.qbase + (tt0 >> LW) + 1) & (kR - 1)) * nstep;
            uwrap = W - ct0;
            if constexpr (!WIDE) {
                // (nv2 + u ncol for u >= uwrap is noffs2 + (u - uwrap) ncol,
                // modulo 2^32)
                const bool tl = has_north & (lane == top);
                nv1 = tl ? noffs : kOOB;
                nv2 = tl ? noffs2 - (unsigned)uwrap * ncol : kOOB;
            }
        }
        if (!WIDE || W <= kWave || sm_ < kWave || sm_ == W - U) {
            // (narrow-or-equal tiles, W <= 64: one block's lanes span several
            // steps, so the steady offsets do not hold -- plain edge blocks)
            if ((W == 16 || W > kWave) && steady) {
                // (narrow tiles only: the wide kernel measured 0.6 % slower
                // with the two builds, profiles/r03/ab/steady_edge_east.txt)
                if (!WIDE && east_glob) run_block(SteadyEdgeG(), sb, std::false_type());
                else run_block(SteadyEdge(), sb, std::false_type());
            } else {
                run_block(Edge(), sb, std::false_type());
            }
        } else if (steady) {
            if constexpr (keep_of<W>()) {
                if (sm_ == kKeepS) run_block(Steady(), sb, std::true_type());
                else run_block(Steady(), sb, std::false_type());
            } else {
                run_block(Steady(), sb, std::false_type());
            }
        } else {
            if constexpr (keep_of<W>()) {
                if (sm_ == kKeepS) run_block(Interior(), sb, std::true_type());
                else run_block(Interior(), sb, std::false_type());
            } else {
                run_block(Interior(), sb, std::false_type());
            }
        }
        // a steady block advances the ring pointer without wrapping (it may
        // end exactly at the ring's end: the next store goes to entry 0)
        if (steady && pw == Lu) pw = 0u;
    }
    // store wave: the last block is finished too
    if constexpr (!WIDE && store_wave_of<W>()) lds_sti(lane == 0 ? &sm.prog[k] : sink_i, total + U);
    if (lane == 0) {
        if (spins) atomicAdd(&a.stats->stall_spins, spins);
        if (slow_n) atomicAdd(&a.stats->slow_diagonals, slow_n);
        if (ieee_n) atomicAdd(&a.stats->ieee_diagonals, ieee_n);
        if (nonfin_n) atomicAdd(&a.stats->nonfinite_diagonals, nonfin_n);
        if (wait_ticks) atomicAdd(&a.stats->slow_ticks, wait_ticks);
        for (int i = 0; i < 5; ++i)
            if (wait_why[i]) atomicAdd(&a.stats->why[i], (unsigned long long)wait_why[i]);
        diag_south_blocks(a, south_host, wait_why[3]);
#ifdef BURG_PIPE_PROF
        atomicAdd(&a.stats->prof[0], __builtin_amdgcn_s_memtime() - pf0);
        atomicAdd(&a.stats->prof[1], pf_vm);
        atomicAdd(&a.stats->prof[2], wait_ticks);
        atomicAdd(&a.stats->prof[4 + k], wait_ticks);
#endif
        atomicAdd(&a.stats->tile_steps, (unsigned long long)K);
    }
}

#if BURG_PIPE_NARROW_TU
}  // namespace

const void *pipe_pair_fn(bool sweep)
{
    return sweep ? (const void *)pipe_kernel<16, true, true> : (const void *)pipe_kernel<16, false, true>;
}

size_t pipe_pair_image(bool sweep)
{
    constexpr bool psw = store_wave_of<16>();
    return sweep ? sizeof(PipeLds<16, true, psw>) : sizeof(PipeLds<16, false, psw>);
}

const void *pipe_narrow_fn(int W, bool sweep)
{
    if (sweep) return W == 8 ? (const void *)pipe_kernel<8, true> : W == 16 ? (const void *)pipe_kernel<16, true> : nullptr;
    return W == 8 ? (const void *)pipe_kernel<8, false> : W == 16 ? (const void *)pipe_kernel<16, false> : nullptr;
}

}  // namespace burg
#else
__global__ void pipe_fill_kernel(v4u *p, size_t n, int color)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = sent_g(color);
}

// Halo ring self-test (one lane): store `put` at granule put_at (if >= 0) and
// poll granule get_at (if >= 0) for `want` for at most `ticks` of the 100 MHz
// realtime clock, both at system scope as the pipe kernel's halo accesses;
// out = the last value read.
__global__ void halo_probe_kernel(v4u *ring, unsigned bytes, int put_at, v4u put, int get_at,
                                  v4u want, long long ticks, v4u *out)
{
    if (threadIdx.x != 0) return;
    const __amdgpu_buffer_rsrc_t rs = rsrc(ring, bytes);
    if (put_at >= 0) st_sys(rs, (unsigned)put_at * 16u, put);
    v4u g = want;
    if (get_at >= 0) {
        const long long t0 = now_rt();
        for (;;) {
            g = ld_sys(rs, (unsigned)get_at * 16u);
            if ((g.x == want.x && g.y == want.y && g.z == want.z && g.w == want.w) ||
                now_rt() - t0 > ticks)
                break;
            __builtin_amdgcn_s_sleep(8);
        }
    }
    *out = g;
}

template <bool SWEEP>
const void *kernel_of(int W)
{
    if (W <= 16) return pipe_narrow_fn(W, SWEEP);  // (the other translation unit)
    if constexpr (!SWEEP) {
        switch (W) {
        case 32: return (const void *)pipe_kernel<32, false>;
        case 64: return (const void *)pipe_kernel<64, false>;
        case 128: return (const void *)pipe_kernel<128, false>;
        case 256: return (const void *)pipe_kernel<256, false>;
        case 512: return (const void *)pipe_kernel<512, false>;
        case 1024: return (const void *)pipe_kernel<1024, false>;
        default: break;
        }
    }
    return nullptr;
}

const void *pipe_fn(int W, bool sweep) { return sweep ? kernel_of<true>(W) : kernel_of<false>(W); }

template <bool SWEEP>
size_t image_of(int W)
{
    switch (W) {
    case 8: return sizeof(PipeLds<8, SWEEP>);
    case 16: return sizeof(PipeLds<16, SWEEP>);
    case 32: return sizeof(PipeLds<32, SWEEP>);
    case 64: return sizeof(PipeLds<64, SWEEP>);
    case 128: return sizeof(PipeLds<128, SWEEP>);
    case 256: return sizeof(PipeLds<256, SWEEP>);
    case 512: return sizeof(PipeLds<512, SWEEP>);
    case 1024: return sizeof(PipeLds<1024, SWEEP>);
    default: return 0;
    }
}

// LDS bytes per workgroup: the image, padded for the wide-tile engine so that
// exactly `per_cu` workgroups share a CU (narrow tiles keep their image size;
// pair: the paired kernel's image)
size_t pipe_dyn_lds(int W, bool sweep, int per_cu, bool pair = false)
{
    if (pair) return pipe_pair_image(sweep);
    const size_t img = sweep ? image_of<true>(W) : image_of<false>(W);
    if (W <= 16) return img;
    const size_t lds_cu = 160 * 1024;
    const size_t want = lds_cu / (size_t)(per_cu + 1) + 1024;
    if (want > lds_cu / (size_t)per_cu) return img;
    return img >= want ? img : want;
}

bool set_lds_limit(const void *fn, size_t bytes)
{
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) == hipSuccess;
}

// workgroups per CU of the wide-tile engine: one, or two for W = 64, 128 in a
// -DBURG_TWO_PER_CU=1 build (their LDS image fits twice); BURG_PIPE_WG_PER_CU
// overrides (tuning knob)
int pipe_per_cu_opt(int W)
{
    static int v = -1;
    if (v < 0) {
        v = 0;
        if (const char *e = std::getenv("BURG_PIPE_WG_PER_CU")) {
            const int x = std::atoi(e);
            if (x >= 1 && x <= 2) v = x;
        }
    }
    return v ? v : (BURG_TWO_PER_CU && (W == 64 || W == 128)) ? 2 : 1;
}

}  // namespace

bool pipe_width_supported(int W) { return pipe_fn(W, false) != nullptr; }

// diagonals per block of the trajectory kernel (its ring walk advances per
// block; burg_ring_audit replays it)
static int pipe_threads(int W)
{
    switch (W) {
    case 8: return threads_of<8>();
    case 16: return threads_of<16>();
    case 32: return threads_of<32>();
    case 64: return threads_of<64>();
    case 128: return threads_of<128>();
    case 256: return threads_of<256>();
    case 512: return threads_of<512>();
    case 1024: return threads_of<1024>();
    }
    return 0;
}

int pipe_block_of(int W)
{
    switch (W) {
    case 8: return BURG_NARROW_U < 8 ? BURG_NARROW_U : 8;
    case 16: return BURG_NARROW_U < 16 ? BURG_NARROW_U : 16;
    case 32: return uw_of<32>();
    case 64: return uw_of<64>();
    case 128: return uw_of<128>();
    case 256: return uw_of<256>();
    case 512: return uw_of<512>();
    case 1024: return uw_of<1024>();
    default: return 0;
    }
}
bool pipe_sweep_width_supported(int W) { return pipe_fn(W, true) != nullptr; }

// the paired sweep kernel runs with a store wave and starts every trajectory
// from a uniform initial state (PipeArgs::w0c): pipe_args pairs a sweep only
// when the uploaded state is uniform
bool pipe_pair_sweep_uniform_only() { return store_wave_of<16>(); }

// resident workgroups of the pipe kernel (sweep = the burg_sweep variant,
// whose larger LDS image must also fit one workgroup per CU)
int pipe_max_resident_blocks(int W, bool sweep)
{
    int dev = 0, n = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -3;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return -3;
    const void *fn = pipe_fn(W, sweep);
    if (!fn) return -1;
    const size_t dyn = pipe_dyn_lds(W, sweep, pipe_per_cu_opt(W));
    if (dyn > 160 * 1024 || !set_lds_limit(fn, dyn)) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, pipe_threads(W), dyn) !=
        hipSuccess)
        return -3;
    if (W == 16) {  // the paired-halves build of the same plan must fit as well
        int np = 0;
        const size_t dp = pipe_dyn_lds(16, sweep, 1, true);
        if (dp > 160 * 1024 || !set_lds_limit(pipe_pair_fn(sweep), dp) ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&np, pipe_pair_fn(sweep), pipe_threads(16), dp) != hipSuccess)
            return -3;
        n = std::min(n, np);
    }
    return n * ncu;
}

int launch_pipe(const PipeArgs &a, int W, hipStream_t st)
{
    const int blocks = a.nti * a.nwj;
    const bool sweep = a.colc_b != nullptr;
    if (sweep && (a.T < 1 || a.K % a.T != 0 || a.K / a.T > kPipeSweepMax)) return -1;
    if (a.pair && (W != 16 || a.ret_k != 0)) return -1;
    const void *fn = a.pair ? pipe_pair_fn(sweep) : pipe_fn(W, sweep);
    if (!fn) return -1;
    const size_t dyn = pipe_dyn_lds(W, sweep, pipe_per_cu_opt(W), a.pair != 0);
    if (dyn > 160 * 1024 || !set_lds_limit(fn, dyn)) return -1;
    // the census counter starts at zero in every launch
    if (hipMemsetAsync(a.census, 0, sizeof(unsigned), st) != hipSuccess) return -3;
    PipeArgs args = a;
    void *kargs[] = {&args};
    const int threads = pipe_threads(W);
    if (hipLaunchKernel(fn, dim3(blocks), dim3(threads), kargs, dyn, st) != hipSuccess) return -3;
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int halo_probe(void *ring, size_t bytes, int put_at, const unsigned put[4], int get_at,
               const unsigned want[4], double seconds, unsigned got[4], hipStream_t st)
{
    if (bytes < 16 || bytes > 0xFFFFFFF0u) return -1;
    v4u *d_out = nullptr;
    if (hipMalloc(&d_out, sizeof(v4u)) != hipSuccess) return -3;
    const v4u p = {put[0], put[1], put[2], put[3]};
    const v4u w = {want[0], want[1], want[2], want[3]};
    hipLaunchKernelGGL(halo_probe_kernel, dim3(1), dim3(kWave), 0, st, (v4u *)ring, (unsigned)bytes,
                       put_at, p, get_at, w, (long long)(seconds * 1e8), d_out);
    v4u h{};
    const bool ok = hipGetLastError() == hipSuccess &&
                    hipMemcpyAsync(&h, d_out, sizeof(v4u), hipMemcpyDeviceToHost, st) == hipSuccess &&
                    hipStreamSynchronize(st) == hipSuccess;
    (void)hipFree(d_out);
    if (!ok) return -3;
    got[0] = h.x;
    got[1] = h.y;
    got[2] = h.z;
    got[3] = h.w;
    return 0;
}

int launch_pipe_fill(void *p, size_t n16, int color, hipStream_t st)
{
    if (n16 == 0) return 0;
    hipLaunchKernelGGL(pipe_fill_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, st,
                       (v4u *)p, n16, color);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace burg
#endif  // BURG_PIPE_NARROW_TU
