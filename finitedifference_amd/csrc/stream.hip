// stream.hip -- the streaming engine: K implicit time steps of the 2D inviscid
// Burgers FOM in ONE launch, exactly the sequential march (orc_march_step,
// bit for bit), pipelined over tiles and time steps.
//
// Why this works: the reference residual (C/hypernet2D.py:2512-2570) couples
// a cell only to itself and its west/south neighbours, so the implicit step
// is a forward substitution in (row, column) order (cell_math.h), and step
// n+1 of a cell needs only step n of the same cell.  The dependence graph over
// (step, row, column) is therefore a 3-D wavefront with no iteration at all.
//
// Mapping: a tile = 64 rows (one per lane) x W columns, owned by ONE wavefront
// for the whole launch.  At diagonal s lane r works on local time t = s - r,
// i.e. step t / W + 1, column t % W: lane r+1 trails lane r by one diagonal, so
// the south inflow of every lane is its neighbour's north outflow of the
// previous diagonal (one DPP move), and the west inflow is the lane's own east
// outflow of the previous diagonal.  The skew runs continuously across time
// steps, so after a 63-diagonal ramp every lane does useful work every
// diagonal.
//
// State lives in a per-tile ring indexed by diagonal: entry s holds, for every
// lane r, the state that lane produced at diagonal s.  The previous step of the
// same cell was produced exactly W diagonals earlier by the same lane, so the
// read for diagonal s is entry s - W: both the read and the write of a
// diagonal are one contiguous 1 KB row (64 lanes x {u, v}), fully coalesced.
//
// Between tiles: outflows cross tile edges through mailboxes of 16-byte
// granules (west edge: 64 rows, south edge: W columns, R step slots each).
// A granule is data-as-flag: the producer writes it write-through (sc1), the
// consumer polls it with sc1 loads until neither half is the sentinel, uses
// it, and writes the sentinel back; the producer checks the slot holds the
// sentinel before reusing it R steps later.  No fences, no counters
// (MI355X_MICROARCH.md, hand-off forms R2).  Every wait is bounded: a wave that
// gives up sets the error word and the launch still drains.
#include <cstdlib>

#include "burg_internal.h"
#include "cell_math.h"

namespace burg {
namespace {

typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr unsigned long long kSentBits = 0x7FF4DEADBEEF5A5AULL;  // a signalling NaN:
                                                                  // never produced by arithmetic
constexpr int kSpinLimit = 1 << 21;  // ~seconds: only a broken pipeline gets there

constexpr unsigned kSentHi = (unsigned)(kSentBits >> 32);
constexpr unsigned kOOB = 0xC0000000u;  // past every mailbox descriptor's range, also
                                        // after adding a slot offset (< 2^30)

// A granule is {x, y} as two little-endian doubles: the high words (where the
// sentinel test looks) are dwords 1 and 3.
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

__device__ __forceinline__ bool has_sent(v4u g) { return g.y == kSentHi || g.w == kSentHi; }
__device__ __forceinline__ bool all_sent(v4u g) { return g.y == kSentHi && g.w == kSentHi; }

// lane i <- lane i-1; lane 0 keeps `old0` (its own value of `old0`)
__device__ __forceinline__ double shr1_or(double old0, double x)
{
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old0), __double2loint(x), 0x138,
                                               0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old0), __double2hiint(x), 0x138,
                                               0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ v4u ld_sc1(__amdgpu_buffer_rsrc_t rs, unsigned off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
}

__device__ __forceinline__ v4u ld_plain(__amdgpu_buffer_rsrc_t rs, unsigned off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
}

__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t rs, unsigned off, v4u v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);
}

__device__ __forceinline__ void st_plain(__amdgpu_buffer_rsrc_t rs, unsigned off, v4u v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
}

template <int W>
constexpr int ilog2() { return W <= 1 ? 0 : 1 + ilog2<W / 2>(); }

// Store VGPRs (as pipe.hip): an opaque copy of a
// store's offset, so the store reads exactly the VGPR the kernel keeps live
// until the next diagonal's stores (tools/store_reuse_check.py checks it)
__device__ __forceinline__ unsigned launder(unsigned off)
{
    asm volatile("" : "+v"(off));
    return off;
}

// One wavefront per tile; 4 tiles per workgroup (one per SIMD).
template <int W, int D, int DM>
__global__ __launch_bounds__(256) void stream_kernel(StreamArgs a)
{
    static_assert((W & (W - 1)) == 0 && W > D, "W: power of two > D");
    static_assert(D % DM == 0, "mailbox slots must tile the unroll");
    constexpr int LW = ilog2<W>();
    // Narrow tiles (W <= 32) keep each lane's last W states in LDS: the
    // previous step of the cell of diagonal s is the lane's own output of
    // diagonal s - W, i.e. LDS slot s mod W.  Wider tiles read it back from
    // the tile's ring in HBM (ring entry s - W, prefetched D diagonals ahead).
    constexpr bool LDSST = W <= 32;
    constexpr bool LDSCC = W <= 1024;  // column table in LDS (else prefetched from HBM)
    __shared__ v4u lds_st[LDSST ? 4 * W * kWave : 1];  // [wave][s mod W][lane]
    __shared__ v4u lds_cc[LDSCC ? 4 * W : 1];          // [wave][column] {hx, src}
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & (kWave - 1);
    const int tile = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wave);
    if (tile >= a.ntiles) return;
    const int ti = tile / a.ntj, tj = tile - ti * a.ntj;
    const int ny = a.cf.ny;
    const int nrow = min(kWave, ny - ti * kWave);
    const int top = nrow - 1;
    const bool iso = a.flags & 1;
    const bool has_west = tj > 0 && !iso, has_east = tj + 1 < a.ntj && !iso;
    const bool has_south = ti > 0 && !iso, has_north = ti + 1 < a.nti && !iso;
    const bool rowok = lane < nrow;
    const int Rm = a.R - 1;
    const int KW = a.K * W;

    // row coefficients (MarchCell::row); padding lanes reuse the top row
    const int r = ti * kWave + min(lane, top);
    const double ay = a.cf.alpha * a.cf.inv_dy[r];
    const double hy = 0.5 * ay;
    const double lb = a.cf.lbc[r];
    const bool col0_tile = tj == 0;

    // the tile's ring (L entries of 64 x 16 B) in HBM
    const __amdgpu_buffer_rsrc_t ring = __builtin_amdgcn_make_buffer_rsrc(
        a.ring + (size_t)tile * a.Lt * kWave, 0, (int)(a.Lt * kWave * 16), 0x00020000);
    const unsigned lane16 = lane * 16u;
    const __amdgpu_buffer_rsrc_t wbox =
        __builtin_amdgcn_make_buffer_rsrc(a.wbox, 0, (int)a.wbox_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t sbox =
        __builtin_amdgcn_make_buffer_rsrc(a.sbox, 0, (int)a.sbox_bytes, 0x00020000);
    // mailbox byte offsets (G = kGranuleStride): west box of tile t, slot q,
    // row l: ((t*R + q)*64 + l)*G; south box of tile t, slot q, column c:
    // ((t*R + q)*W + c)*G
    constexpr unsigned G = kGranuleStride;
    const unsigned wb_mine = (unsigned)tile * a.R * kWave * G + lane * G;
    const unsigned wb_step = (unsigned)a.R * kWave * G;  // -> the east tile's box
    const unsigned sb_mine = (unsigned)tile * a.R * W * G;
    const unsigned sb_step = (unsigned)a.ntj * a.R * W * G;  // -> the north tile's box
    const v4u sent = as_v4u(__longlong_as_double((long long)kSentBits),
                            __longlong_as_double((long long)kSentBits));
    const long long L = a.L;

    // column table and (LDSST) state 0 into LDS: state 0 of the lane's column
    // c sits at diagonal c + lane - W, i.e. LDS slot (c + lane) mod W
    v4u *my_st = lds_st + (LDSST ? wave * W * kWave : 0);
    v4u *my_cc = lds_cc + (LDSCC ? wave * W : 0);
    const __amdgpu_buffer_rsrc_t colc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.colc + (size_t)tj * W), 0, W * 16, 0x00020000);
    if constexpr (LDSCC) {
        for (int c = lane; c < W; c += kWave) {
            const d2 v = a.colc[(size_t)tj * W + c];
            my_cc[c] = as_v4u(v.x, v.y);
        }
    }
    if constexpr (LDSST) {
        for (int c = 0; c < W; ++c) {
            long long e = (a.origin + c + lane - W) % L;
            e = e < 0 ? e + L : e;
            my_st[((c + lane) & (W - 1)) * kWave + lane] = ld_plain(ring, (unsigned)e * 1024u + lane16);
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0);

    // Prefetch rings.  Edge granules, DM diagonals ahead (slot j = s mod DM):
    //   gw: the lane's west/east granule -- at column 0 the west inflow of this
    //       step (consume), at column W-1 the east tile's slot (must be empty)
    //   gs: lane 0: the south inflow granule; lane `top`: the north tile's slot
    //   ow, os: the byte offsets of gw, gs (kOOB where the lane has no access:
    //       buffer loads there return 0 and stores are dropped)
    // DM is short on purpose: a pipelined consumer runs just behind its
    // producer, and a granule fetched too early is still the sentinel.
    // State and columns of wide tiles, D diagonals ahead (slot i = s mod D):
    //   pf (!LDSST): the lane's previous-step state (ring entry s - W)
    //   cc (!LDSCC): {hx, src} of the lane's column
    v4u gw[DM], gs[DM], pf[LDSST ? 1 : D], cc[LDSCC ? 1 : D];
    unsigned ow[DM], os[DM];
    long long pw = a.origin;                       // ring entry of diagonal s
    long long pr = ((a.origin - W) % L + L) % L;  // ring entry of the next prefetch's s - W
    const int lane_j = lane;  // keep lane in a VGPR
    // bases with the tile's neighbourhood folded in (kOOB: no such neighbour).
    // Padding lanes (rows past the grid in a partial strip) stay out of the
    // edge protocol: their consumer would not wait (only real rows take the
    // slow path), so it could empty a slot before the producer filled it.
    const unsigned wcb = has_west && rowok ? wb_mine : kOOB;            // west inflow
    const unsigned wpb = has_east && rowok ? wb_mine + wb_step : kOOB;  // east outflow
    // lane 0 consumes the south edge, lane `top` produces the north edge
    const unsigned slb = lane == 0 ? (has_south ? sb_mine : kOOB)
                                   : (lane == top && has_north ? sb_mine + sb_step : kOOB);
    auto prefetch_ring = [&](int sp, int i) {
        const int cp = (sp - lane_j) & (W - 1);
        if constexpr (!LDSST) {
            pf[i % (LDSST ? 1 : D)] = ld_plain(ring, (unsigned)pr * 1024u + lane16);
            pr = pr + 1 == L ? 0 : pr + 1;
        }
        if constexpr (!LDSCC) cc[i % (LDSCC ? 1 : D)] = ld_plain(colc, (unsigned)cp * 16u);
    };
    auto prefetch_mail = [&](int sp, int j) {
        const int tp = sp - lane_j;
        const int cp = tp & (W - 1);
        const unsigned qp = (unsigned)(tp >> LW) & (unsigned)Rm;
        const bool vp = (unsigned)tp < (unsigned)KW;
        const unsigned o = cp == 0 ? wcb : (cp == W - 1 ? wpb : kOOB);
        ow[j] = vp ? o + qp * (kWave * G) : kOOB;
        gw[j] = ld_sc1(wbox, ow[j]);
        os[j] = vp ? slb + ((qp << LW) | (unsigned)cp) * G : kOOB;
        gs[j] = ld_sc1(sbox, os[j]);
    };
#pragma unroll
    for (int i = 0; i < D; ++i) prefetch_ring(i, i);
#pragma unroll
    for (int j = 0; j < DM; ++j) prefetch_mail(j, j);
    // Land the first slots here: otherwise the compiler's wait counts at the
    // loop head are those of this short prologue path (few operations after
    // each load) and every round would wait on its newest write-through stores.
    __builtin_amdgcn_s_waitcnt(0);

    double e0 = 0.0, e1 = 0.0, no0 = 0.0, no1 = 0.0;
    // the previous diagonal's store data and offsets, kept live until this
    // diagonal's stores (store VGPRs)
    v4u k_out = v4u{0u, 0u, 0u, 0u}, k_e = k_out, k_n = k_out;
    unsigned k_r = 0u, k_w0 = 0u, k_we = 0u, k_s0 = 0u, k_sn = 0u;
    unsigned spins = 0, slow_n = 0, nonfin_n = 0, why_n[6] = {0, 0, 0, 0, 0, 0};
    unsigned long long slow_t = 0;
    bool bad_range = false;

    // one diagonal s, prefetch slots k = s mod D, m = s mod DM
    auto diagonal = [&](const int s, const int k) {
        const int m = k % DM;
        const int t = s - lane_j;
        const int c = t & (W - 1);
        const bool valid = (unsigned)t < (unsigned)KW;
        const bool at0 = c == 0, atE = c == W - 1;
        const bool s_in = lane == 0, n_out = lane == top && lane != 0;
        v4u *st_slot = my_st + (LDSST ? (s & (W - 1)) * kWave + lane : 0);
        // ---- the cell (MarchCell::pre + chain, same op order)
        const d2 x = as_d2(LDSST ? *st_slot : pf[k % (LDSST ? 1 : D)]);
        const d2 co = as_d2(LDSCC ? my_cc[c] : cc[k % (LDSCC ? 1 : D)]);
        const double pu = x.x, pv = x.y;
        const double hx = co.x, ax = hx + hx;  // exact: hx = 0.5 * (alpha * inv_dx)
        const double sl = (col0_tile && at0) ? co.y + lb : co.y;
        MarchCell::Pre p;
        p.hx = hx;
        const double hu = 0.5 * pu;
        p.xfp = ax * (hu * pu);
        p.xhp = ax * (hu * pv);
        p.yhp = ay * (hu * pv);
        p.ygp = ay * ((0.5 * pv) * pv);
        p.bu = ((pu - p.xfp) - p.yhp) + sl;
        p.bv = (pv - p.ygp) - p.xhp;
        const MarchCell::Row rw{ay, hy, lb};
        // producers: the east / north slot must be empty (sentinel in both halves)
        bool pbad = false;
        if (has_east) pbad |= valid && rowok && atE && !all_sent(gw[m]);
        if (has_north) pbad |= valid && n_out && !all_sent(gs[m]);
        // west inflow at column 0: the granule, or +0.0 at the domain
        // boundary (the load was out of range); south inflow of lane 0 likewise.
        // A granule not yet written holds the sentinel NaN, which fails the
        // chain's range check: the slow path below then waits for it.
        if (at0) {
            const d2 g = as_d2(gw[m]);
            e0 = g.x;
            e1 = g.y;
        }
        double n0 = shr1_or(as_d2(gs[m]).x, no0);
        double n1 = shr1_or(as_d2(gs[m]).y, no1);
        double oe0, oe1, on0, on1, o0, o1;
        bool ok;
        MarchCell::chain<true>(p, rw, e0, e1, n0, n1, oe0, oe1, on0, on1, o0, o1, ok);
        if (__builtin_expect(__any((!ok && valid && rowok) || pbad), 0)) {
            // slow path: poll the granules until inputs are written and
            // output slots are free, then redo the cell with IEEE sqrt/div
            const unsigned long long t_in = __builtin_amdgcn_s_memtime();
            if (has_east && __any(valid && rowok && atE && !all_sent(gw[m]))) ++why_n[0];
            if (has_north && __any(valid && n_out && !all_sent(gs[m]))) ++why_n[1];
            if (has_west && __any(valid && rowok && at0 && has_sent(gw[m]))) ++why_n[2];
            if (has_south && __any(valid && s_in && has_sent(gs[m]))) ++why_n[3];
            if (__any(!ok && valid && rowok && !(at0 && has_sent(gw[m])) &&
                      !(s_in && has_sent(gs[m]))))
                ++why_n[4];
            bool first = true;
            for (;;) {
                gw[m] = ld_sc1(wbox, ow[m]);
                gs[m] = ld_sc1(sbox, os[m]);
                bool b = false;
                if (has_west) b |= valid && rowok && at0 && has_sent(gw[m]);
                if (has_south) b |= valid && s_in && has_sent(gs[m]);
                if (has_east) b |= valid && rowok && atE && !all_sent(gw[m]);
                if (has_north) b |= valid && n_out && !all_sent(gs[m]);
                if (!__any(b)) break;
                if (first) ++why_n[5];
                first = false;
                if (++spins >= kSpinLimit) {
                    // report which wait gave up: tile, diagonal, and which edge
                    unsigned why = 0;
                    if (has_west && __any(valid && rowok && at0 && has_sent(gw[m]))) why |= 1;
                    if (has_south && __any(valid && s_in && has_sent(gs[m]))) why |= 2;
                    if (has_east && __any(valid && rowok && atE && !all_sent(gw[m]))) why |= 4;
                    if (has_north && __any(valid && n_out && !all_sent(gs[m]))) why |= 8;
                    if (lane == 0 && atomicOr(a.err, 1u) == 0) {
                        set_err3(a.err, (unsigned)tile, (unsigned)s, why);
                    }
                    break;
                }
                __builtin_amdgcn_s_sleep(4);
            }
            // back off once more: a consumer that keeps running exactly
            // behind its producer finds every prefetched granule stale; a
            // little extra lag lets the prefetches land after the writes
            for (int q = (a.flags >> 8) & 0xff; q > 0; q -= 8) __builtin_amdgcn_s_sleep(8);
            if (at0) {
                const d2 g = as_d2(gw[m]);
                e0 = g.x;
                e1 = g.y;
            }
            n0 = shr1_or(as_d2(gs[m]).x, no0);
            n1 = shr1_or(as_d2(gs[m]).y, no1);
            MarchCell::chain<false>(p, rw, e0, e1, n0, n1, oe0, oe1, on0, on1, o0, o1, ok);
            bad_range = true;
            // the only place a non-finite state can appear (fast-path range check)
            if (__any(valid && rowok && !(__builtin_isfinite(o0) && __builtin_isfinite(o1))))
                ++nonfin_n;
            ++slow_n;
            slow_t += __builtin_amdgcn_s_memtime() - t_in;
        }
        e0 = oe0;
        e1 = oe1;
        no0 = on0;
        no1 = on1;
        // ---- outputs (lanes that have not started keep their step-0 state)
        const v4u out = as_v4u(o0, o1);
        if constexpr (LDSST) {
            if (t >= 0) *st_slot = out;
        }
        asm volatile("" ::"v"(k_out), "v"(k_e), "v"(k_n), "v"(k_r), "v"(k_w0), "v"(k_we), "v"(k_s0),
                     "v"(k_sn));
        const v4u eo = as_v4u(oe0, oe1), no = as_v4u(on0, on1);
        const unsigned o_r = launder(valid ? (unsigned)pw * 1024u + lane16 : kOOB);
        const unsigned o_w0 = launder(at0 ? ow[m] : kOOB), o_we = launder(atE ? ow[m] : kOOB);
        const unsigned o_s0 = launder(s_in ? os[m] : kOOB), o_sn = launder(s_in ? kOOB : os[m]);
        st_plain(ring, o_r, out);
        st_sc1(wbox, o_w0, sent);  // consumed: empty it
        st_sc1(wbox, o_we, eo);    // east outflow
        st_sc1(sbox, o_s0, sent);
        st_sc1(sbox, o_sn, no);    // north outflow
        k_out = out;
        k_e = eo;
        k_n = no;
        k_r = o_r;
        k_w0 = o_w0;
        k_we = o_we;
        k_s0 = o_s0;
        k_sn = o_sn;
        pw = pw + 1 == L ? 0 : pw + 1;
        prefetch_ring(s + D, k);
        prefetch_mail(s + DM, m);
    };

    const int total = KW + kWave - 1;
    for (int sb = 0; sb < total; sb += D) {
#pragma unroll
        for (int k = 0; k < D; ++k) diagonal(sb + k, k);
    }
    if (lane == 0) {
        if (spins) atomicAdd(&a.stats->stall_spins, (unsigned long long)spins);
        if (slow_n) {
            atomicAdd(&a.stats->slow_diagonals, (unsigned long long)slow_n);
            atomicAdd(&a.stats->slow_ticks, slow_t);
            for (int q = 0; q < 6; ++q)
                if (why_n[q]) atomicAdd(&a.stats->why[q], (unsigned long long)why_n[q]);
        }
        atomicAdd(&a.stats->tile_steps, (unsigned long long)a.K);
        if (nonfin_n) atomicAdd(&a.stats->nonfinite_diagonals, (unsigned long long)nonfin_n);
    }
    if (__any(bad_range) && lane == 0) atomicAdd(&a.stats->ieee_diagonals, 1ull);
}

// {hx, src} per column, padded to ntj*W with the last column's values.
__global__ void colc_kernel(Coeffs cf, d2 *colc, int ncols_pad)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncols_pad) return;
    const int cc = min(c, cf.nx - 1);
    const double ax = cf.alpha * cf.inv_dx[cc];
    colc[c] = d2{0.5 * ax, cf.src[cc]};
}

// sweep table: {hx, src_j} per trajectory j and (padded) column, hx as colc_kernel
__global__ void colc_batch_kernel(Coeffs cf, const double *src_b, d2 *colc_b, int ncols_pad,
                                  int nb)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = blockIdx.y;
    if (c >= ncols_pad || j >= nb) return;
    const int cc = min(c, cf.nx - 1);
    const double ax = cf.alpha * cf.inv_dx[cc];
    colc_b[(size_t)j * ncols_pad + c] = d2{0.5 * ax, src_b[(size_t)j * cf.nx + cc]};
}

__global__ void fill_sent_kernel(d2 *p, size_t n)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double s = __longlong_as_double((long long)kSentBits);
    p[i] = d2{s, s};
}

// entry of state k (k >= 0) of local cell (lane, cl) of a tile
// ring entry of state k (0: the launch's initial state), column cl, lane
__device__ __forceinline__ long long ring_entry(const StreamArgs &a, int W, int k, int cl, int lane)
{
    if (a.play && k >= 1) return ring_pos_paired(k - 1, cl, lane, a.origin, a.L);
    return ring_pos((long long)(k - 1) * W + cl + lane, a.origin, a.L, W, a.ret_k, a.ret_n,
                    a.ret_base);
}

// C-order state w (u plane | v plane) -> ring entries of state 0.
// Padding cells (rows >= ny, columns >= nx) get u = v = 1.  Consecutive
// threads fill consecutive lanes of ONE ring entry (a skewed diagonal s =
// cl + lane of the tile: 1 KB stores per wave) and read the state along that
// diagonal (8 B per row; reads scattered rather than stores, as in
// ring_extract_kernel): 4096^2 218 us per load, against 289 us with
// consecutive lanes of one column (stores and reads scattered) and 249 us
// with consecutive columns of one row (profiles/r04/ringload).
// Bounds guard of the flat-pointer ring kernels: an
// entry outside the tile's Lt entries, or an output index past the caller's
// buffer, is not accessed; it sets err[5] (kErrBounds), which the host checks
// after the copy (check_bounds, capi.hip).  One compare per thread.
constexpr int kErrBounds = 5;
__device__ __forceinline__ bool ring_ok(const StreamArgs &a, long long e)
{
    if (e >= 0 && e < a.Lt) return true;
    atomicOr(a.err + kErrBounds, 1u);
    return false;
}
__device__ __forceinline__ bool out_ok(const StreamArgs &a, size_t i, size_t n)
{
    if (i < n) return true;
    atomicOr(a.err + kErrBounds, 2u);
    return false;
}

__global__ void ring_load_kernel(StreamArgs a, int W, const double *w)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t per_tile = (size_t)kWave * (W + kWave - 1);
    if (i >= (size_t)a.ntiles * per_tile) return;
    const int tile = (int)(i / per_tile);
    const int rem = (int)(i - (size_t)tile * per_tile);
    const int lane = rem % kWave, cl = rem / kWave - lane;  // diagonal rem / kWave = cl + lane
    if (cl < 0 || cl >= W) return;
    const int ti = tile / a.ntj, tj = tile % a.ntj;
    const int row = ti * kWave + lane, col = tj * W + cl;
    const size_t n = (size_t)a.cf.nx * a.cf.ny;
    d2 v{1.0, 1.0};
    if (row < a.cf.ny && col < a.cf.nx) {
        const size_t j = (size_t)row * a.cf.nx + col;
        v = d2{w[j], w[n + j]};
    }
    const long long e = ring_entry(a, W, 0, cl, lane);
    if (ring_ok(a, e)) a.ring[((size_t)tile * a.Lt + e) * kWave + lane] = v;
}

// Snapshot extraction: out[e * ldo + j] = element e of state (k0 + j*kstep),
// e over the 2*nx*ny C-order state (u plane | v plane), j < count.
__global__ void ring_extract_kernel(StreamArgs a, int W, int k0, int kstep, int count,
                                    double *out, int ldo, size_t out_elems)
{
    const size_t n = (size_t)a.cf.nx * a.cf.ny;
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n * count) return;
    const size_t cell = idx / count;
    const int j = (int)(idx - cell * count);
    const int row = (int)(cell / a.cf.nx), col = (int)(cell - (size_t)row * a.cf.nx);
    const int ti = row / kWave, lane = row - ti * kWave;
    const int tj = col / W, cl = col - tj * W;
    const int tile = ti * a.ntj + tj;
    const long long e = ring_entry(a, W, k0 + j * kstep, cl, lane);
    if (!ring_ok(a, e) || !out_ok(a, (n + cell) * ldo + j, out_elems)) return;
    const d2 v = a.ring[((size_t)tile * a.Lt + e) * kWave + lane];
    out[cell * ldo + j] = v.x;
    out[(n + cell) * ldo + j] = v.y;
}

// Row block of the C-order snapshot matrix: out[(e - e0) * ncols + j] =
// element e (u plane, then v plane) of state k0 + j*kstep, e in [e0, e0 + ne).
// Consecutive threads walk j: the reads gather 16-B cells from the ring, the
// writes are the contiguous rows of the .npy file.
__global__ void ring_extract_rows_kernel(StreamArgs a, int W, size_t e0, size_t ne, int k0,
                                         int kstep, int ncols, double *out, size_t out_elems)
{
    const size_t n = (size_t)a.cf.nx * a.cf.ny;
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= ne * (size_t)ncols) return;
    const size_t er = idx / ncols;
    const int j = (int)(idx - er * ncols);
    const size_t e = e0 + er;
    const bool vplane = e >= n;
    const size_t cell = vplane ? e - n : e;
    const int row = (int)(cell / a.cf.nx), col = (int)(cell - (size_t)row * a.cf.nx);
    const int ti = row / kWave, lane = row - ti * kWave;
    const int tj = col / W, cl = col - tj * W;
    const int tile = ti * a.ntj + tj;
    const long long en = ring_entry(a, W, k0 + j * kstep, cl, lane);
    if (!ring_ok(a, en) || !out_ok(a, idx, out_elems)) return;
    const d2 v = a.ring[((size_t)tile * a.Lt + en) * kWave + lane];
    out[idx] = vplane ? v.y : v.x;
}

template <int W, int D, int DM = 4>
int launch_w(const StreamArgs &a, int blocks, hipStream_t st)
{
    hipLaunchKernelGGL((stream_kernel<W, D, DM>), dim3(blocks), dim3(256), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace

// ---------------------------------------------------------------------------
StreamPlan plan_stream(int nx, int ny, int tiles_target, int w_force)
{
    StreamPlan p{};
    p.nti = (ny + kWave - 1) / kWave;
    int W = 8;
    if (w_force > 0) {
        W = w_force;
    } else {
        // smallest power-of-two width (>= 8) whose tile count fits the target
        while (W < 4096 && (long long)p.nti * ((nx + W - 1) / W) > tiles_target) W *= 2;
    }
    p.W = W;
    p.ntj = (nx + W - 1) / W;
    p.ntiles = p.nti * p.ntj;
    p.R = 4;
    while (p.R < 64 / W + 4) p.R *= 2;
    if (const char *e = std::getenv("BURG_STREAM_R")) {  // diagnostics
        const int v = std::atoi(e);
        if (v >= 4 && (v & (v - 1)) == 0) p.R = v;
    }
    return p;
}

bool stream_width_supported(int W)
{
    return W == 8 || W == 16 || W == 32 || W == 64 || W == 128 || W == 256 || W == 512 ||
           W == 1024 || W == 2048 || W == 4096;
}

int launch_stream(const StreamArgs &a, int W, hipStream_t st)
{
    const int blocks = (a.ntiles + 3) / 4;
    switch (W) {
    case 8: return launch_w<8, 4>(a, blocks, st);
    case 16: return (a.flags & 2) ? launch_w<16, 8, 2>(a, blocks, st)
                                  : launch_w<16, 8, 4>(a, blocks, st);
    case 32: return launch_w<32, 8>(a, blocks, st);
    case 64: return launch_w<64, 8>(a, blocks, st);
    case 128: return launch_w<128, 8>(a, blocks, st);
    case 256: return launch_w<256, 8>(a, blocks, st);
    case 512: return launch_w<512, 8>(a, blocks, st);
    case 1024: return launch_w<1024, 8>(a, blocks, st);
    case 2048: return launch_w<2048, 8>(a, blocks, st);
    case 4096: return launch_w<4096, 8>(a, blocks, st);
    default: return -1;
    }
}

int stream_max_resident_blocks(int W, int *per_cu, int *cus)
{
    int dev = 0, n = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -3;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return -3;
    const void *fn = nullptr;
    switch (W) {
    case 8: fn = (const void *)stream_kernel<8, 4, 4>; break;
    case 16: fn = (const void *)stream_kernel<16, 8, 4>; break;
    case 32: fn = (const void *)stream_kernel<32, 8, 4>; break;
    case 64: fn = (const void *)stream_kernel<64, 8, 4>; break;
    case 128: fn = (const void *)stream_kernel<128, 8, 4>; break;
    case 256: fn = (const void *)stream_kernel<256, 8, 4>; break;
    case 512: fn = (const void *)stream_kernel<512, 8, 4>; break;
    case 1024: fn = (const void *)stream_kernel<1024, 8, 4>; break;
    case 2048: fn = (const void *)stream_kernel<2048, 8, 4>; break;
    case 4096: fn = (const void *)stream_kernel<4096, 8, 4>; break;
    default: return -1;
    }
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 256, 0) != hipSuccess) return -3;
    // the API can over-report by one block per CU (MI355X_MICROARCH.md, residency)
    n = n > 1 ? n - 1 : n;
    if (per_cu) *per_cu = n;
    if (cus) *cus = ncu;
    return n * ncu;
}

int launch_colc(const Coeffs &cf, int ncols_pad, void *colc, hipStream_t st)
{
    hipLaunchKernelGGL(colc_kernel, dim3((ncols_pad + 255) / 256), dim3(256), 0, st, cf,
                       (d2 *)colc, ncols_pad);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_colc_batch(const Coeffs &cf, int nb, const double *src_b, int ncols_pad, void *colc_b,
                      hipStream_t st)
{
    hipLaunchKernelGGL(colc_batch_kernel, dim3((ncols_pad + 255) / 256, nb), dim3(256), 0, st, cf,
                       src_b, (d2 *)colc_b, ncols_pad, nb);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_fill_sentinel(void *p, size_t n16, hipStream_t st)
{
    if (n16 == 0) return 0;
    hipLaunchKernelGGL(fill_sent_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, st,
                       (d2 *)p, n16);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_ring_load(const StreamArgs &a, int W, const double *w, hipStream_t st)
{
    const size_t total = (size_t)a.ntiles * kWave * (W + kWave - 1);
    hipLaunchKernelGGL(ring_load_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                       a, W, w);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_ring_extract_rows(const StreamArgs &a, int W, size_t e0, size_t ne, int k0, int kstep,
                             int ncols, double *out, size_t out_elems, hipStream_t st)
{
    const size_t total = ne * (size_t)ncols;
    if (total == 0) return 0;
    hipLaunchKernelGGL(ring_extract_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       st, a, W, e0, ne, k0, kstep, ncols, out, out_elems);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_ring_extract(const StreamArgs &a, int W, int k0, int kstep, int count, double *out,
                        int ldo, size_t out_elems, hipStream_t st)
{
    const size_t total = (size_t)a.cf.nx * a.cf.ny * count;
    if (total == 0) return 0;
    hipLaunchKernelGGL(ring_extract_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       st, a, W, k0, kstep, count, out, ldo, out_elems);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace burg
