// SAE (time surface) + FAST/arc corner detection.
//
// Reference: FCT/metavision_time_surface_periodic_group_track.cpp — per reslicer slice of
// 16384 events the aggregate lambda first writes time_surface.at(y,x) = t for EVERY event
// (:900-923, batch semantics Q14), then runs the eFAST arc test event by event on the CPU
// (:948-1063; circle3 streaks of 3..6 of 16 then circle4 streaks of 4..8 of 20, circles
// :44-45 as {dy,dx}), holding a mutex per event.
//
// Exact batch semantics for a whole batch in few launches.  The arc test of an event in slice
// s must see V(q,s) = t of the last event at pixel q with index < end(s).  Slices are
// processed in GROUPS of G = 32.  For the group being tested we keep
//   mask[q]    : u32 bitmask of the group's slices that touched q
//   M[j][q]    : max t at q within slice j of the group (valid only where mask bit j is set)
//   B[q]       : SAE before the group (the caller's `sae` buffer, updated in place)
// so V(q,s) = M[j*][q] with j* = highest set bit of mask[q] & ((2 << j) - 1), else B[q]
// (timestamps are non-decreasing, so max == last writer; a device check enforces it).
//
// Locality.  The batch is counting-sorted by (group, 16x16-pixel TILE) into 4-byte keys
// (event index within the group << 8 | pixel within the tile) + timestamps:
// per-slice LDS histograms -> scan -> per-slice scatter.  Then per group:
//   tile_build(g): one 1024-lane workgroup per tile OWNS that tile's 256 pixels: it folds group
//                  g-1 into B, accumulates mask/M of its bin with LDS atomics and writes them
//                  back with plain stores — no global atomics and no reset pass (M is only ever
//                  read where the same group's mask bit is set);
//   arc_test(g):   one workgroup per WORK ITEM (<= 4096 events of one tile): it stages the
//                  tile's 24x24 neighbourhood — mask, B and the set M entries compacted per
//                  pixel as u32 offsets from the group's first timestamp — in LDS, then tests
//                  one event per lane against LDS only.  Hot tiles split into several items.
// Two ping-pong buffer sets: tile_build(g) reads set (g-1)&1 and writes set g&1.
//
// Arc test: the reference loop "exists i,s: T[c(i)]>=T[c(i-1)], T[c(i+s-1)]>=T[c(i+s)], and
// every T outside the streak < min(streak)" reduces to "the s largest values are strictly
// greater than the rest and occupy a contiguous arc" (the two >= conditions are implied).
// With cnt[j] = #{k : T[k] > T[j]}, the top-s set is {j : cnt[j] < s}; it is strictly
// separated iff its size is s.  This branch-free form is exact; tests/test_gpu_parity.py
// checks it against the literal loop in oracle/oracle.cpp.
// Algorithmic bytes: 12 B/event in (xy + t) + 1 B/event out (corner flag).
#include "ecc_internal.hpp"

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>

// Development instrumentation (make CORNER_PROFILE=1): per-workgroup s_memrealtime stamps of one
// group launch (ECC_CORNER_TS=<group>, ECC_CORNER_TS_FILE) and phase cut-offs (ECC_CORNER_DBG),
// read by scripts/ts_analyze.py / ts_phases.py.  Compiled out by default.
#ifndef ECC_CORNER_PROFILE
#define ECC_CORNER_PROFILE 0
#endif

namespace {

constexpr int kThreads = 256;
constexpr int kBuildUnroll = 8;
constexpr int kArcThreads = 512;  // 8 waves: one lane per window pixel (484) when staging
constexpr int kItemEvents = 2048;  // events per arc work item
constexpr int kGroup = 32;         // slices per group (mask bits)
constexpr int kTile = 14;          // tile edge (pixels): the 22x22 window fits one 8-wave workgroup
constexpr int kTilePix = kTile * kTile;
constexpr int kHalo = 4;           // circle radius
constexpr int kWin = kTile + 2 * kHalo;  // 22
constexpr int kWinPix = kWin * kWin;     // 484
constexpr int kStageMinEvents = 128;     // smaller work items skip the window staging
constexpr int kMaxTiles = 8191;          // bins per group = n_tiles + 1 (8192 fit an LDS histogram)
constexpr int kMaxSlice = 1 << 19;       // group-local event index must fit 24 bits

struct CornerGeom {
    int W, H, S, margin, border_mode, first_detect;
    int tiles_x, n_tiles;  // bin n_tiles of each group holds the events outside the sensor
    float inv_S;
    int dbg;                 // ECC_CORNER_PROFILE only
    unsigned long long *ts;  // ECC_CORNER_PROFILE only
    int64_t ts_grp;
    int64_t n, n_slices;
};

struct GroupBufs {
    uint32_t *mask;  // [H*W]
    int64_t *M;      // [kGroup][H*W]
};

// Batch sorted by (group, tile): bin b of group g is [bin_off[g*nb+b], bin_off[g*nb+b+1]).
struct Sorted {
    uint32_t *key;       // (event index - first event of the group) << 8 | pixel in tile
    uint32_t *t32;       // t - t(first event of the group), written for groups spanning < 2^32 - 1
    int32_t *bin_count;  // [n_bins]
    int32_t *rel;        // [n_slices * nb] slice's offset inside each bin it touches
    int64_t *bin_off;    // [n_bins + 1]
    int32_t *n_items;    // [n_bins] work items per bin
    int64_t *item_off;   // [n_bins + 1]
    uint4 *items;        // [n_groups][max_items] {tile, first event, end event, -}
    int32_t *grp_items;  // [n_groups] work items per group
    int max_items;       // per-group stride of items
};

__constant__ int8_t c3dy[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
__constant__ int8_t c3dx[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
__constant__ int8_t c4dy[20] = {0, 1, 2, 3, 4, 4, 4, 3, 2, 1, 0, -1, -2, -3, -4, -4, -4, -3, -2, -1};
__constant__ int8_t c4dx[20] = {4, 4, 3, 2, 1, 0, -1, -2, -3, -4, -4, -4, -3, -2, -1, 0, 1, 2, 3, 4};

__device__ __forceinline__ bool is_border(int x, int y, const CornerGeom &g) {
    return x < g.margin || x >= g.W - g.margin || y < g.margin || y >= g.H - g.margin;
}

__device__ __forceinline__ int tile_of(uint32_t v, const CornerGeom &g) {
    const int x = ecc::xy_x(v), y = ecc::xy_y(v);
    if (x >= g.W || y >= g.H) return g.n_tiles;
    return (y / kTile) * g.tiles_x + x / kTile;
}

__device__ __forceinline__ uint32_t tile_key(uint32_t v, uint32_t e_local) {
    return (e_local << 8) | (uint32_t)((ecc::xy_y(v) % kTile) * kTile + ecc::xy_x(v) % kTile);
}

// The group's events span < 2^32 - 1 ticks: t - t(first event) fits a u32 (+1 still fits).
__device__ __forceinline__ bool group_narrow(const int64_t *__restrict__ t, const CornerGeom &g, int64_t grp,
                                             int64_t *t_first) {
    const int64_t first = grp * kGroup * (int64_t)g.S;
    const int64_t end = (grp + 1) * kGroup * (int64_t)g.S;
    *t_first = t[first];
    return (uint64_t)(t[(end < g.n ? end : g.n) - 1] - *t_first) < 0xffffffffull;
}

// floor(el / S) for el < 2^24 (float estimate, then exact correction).
__device__ __forceinline__ int slice_in_group(uint32_t el, const CornerGeom &g) {
    uint32_t q = (uint32_t)((float)el * g.inv_S);
    const uint32_t S = (uint32_t)g.S;
    q = (q * S > el) ? q - 1 : q;
    q = ((q + 1) * S <= el) ? q + 1 : q;
    return (int)q;
}

// 1. Per-slice tile histogram (+ time-order check, first border index per slice for Q11).  The
// value returned by the bin-total atomic is the slice's offset inside the bin (kept in rel[]).
constexpr int kHistUnroll = 8;

__global__ void __launch_bounds__(kThreads)
bin_hist_kernel(const uint32_t *__restrict__ xy, const int64_t *__restrict__ t, CornerGeom g,
                Sorted so, int32_t *__restrict__ first_border, int32_t *__restrict__ err) {
    extern __shared__ int32_t hist[];  // [nb]
    const int64_t s = blockIdx.x;
    const int64_t lo = s * g.S, hi = (lo + g.S < g.n) ? lo + g.S : g.n;
    const int64_t grp = s / kGroup;
    const int nb = g.n_tiles + 1;
    for (int b = threadIdx.x; b < nb; b += kThreads) hist[b] = 0;
    __syncthreads();
    bool bad = false;
    int fb = 0x7fffffff;
    for (int64_t e0 = lo; e0 < hi; e0 += kHistUnroll * kThreads) {
        uint32_t v[kHistUnroll];
        int64_t tc[kHistUnroll], tp[kHistUnroll];
#pragma unroll
        for (int u = 0; u < kHistUnroll; ++u) {
            const int64_t e = e0 + u * kThreads + threadIdx.x;
            v[u] = (e < hi) ? xy[e] : 0u;
            tc[u] = (e < hi) ? t[e] : 0;
            tp[u] = (e < hi && e > 0) ? t[e - 1] : INT64_MIN;
        }
#pragma unroll
        for (int u = 0; u < kHistUnroll; ++u) {
            const int64_t e = e0 + u * kThreads + threadIdx.x;
            if (e < hi) {
                atomicAdd(&hist[tile_of(v[u], g)], 1);
                bad |= tp[u] > tc[u];
                if (is_border(ecc::xy_x(v[u]), ecc::xy_y(v[u]), g)) fb = min(fb, (int)(e - lo));
            }
        }
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) *err = 1;
    if (g.border_mode == 1) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) fb = min(fb, __shfl_xor(fb, o));
        if ((threadIdx.x & 63) == 0 && fb != 0x7fffffff) atomicMin(&first_border[s], fb);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nb; b += kThreads)
        if (hist[b]) so.rel[s * nb + b] = atomicAdd(&so.bin_count[grp * nb + b], hist[b]);
}

// Block-wide exclusive scan of in[0, n) into out (256 threads, each owning a contiguous run).
__device__ __forceinline__ void block_excl_scan(const int32_t *in, int32_t *out, int n, int32_t *wsum) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int per = (n + kThreads - 1) / kThreads;
    const int b0 = min(n, tid * per), b1 = min(n, b0 + per);
    int sum = 0;
    for (int i = b0; i < b1; ++i) sum += in[i];
    int incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int run = incl - sum;
    for (int w = 0; w < wave; ++w) run += wsum[w];
    for (int i = b0; i < b1; ++i) {
        const int c = in[i];
        out[i] = run;
        run += c;
    }
}

// 2. Scatter 4-byte keys (+ 4-byte group-relative timestamps when the group spans < 2^32 - 1
// ticks) into (group, tile) order; order inside a bin is irrelevant.
// The slice's range of every bin comes from bin_hist (rel[]); each chunk of C events is counting-
// sorted by bin in LDS and written out in bin order, so consecutive lanes store to
// consecutive addresses (a direct scatter stores every lane to a different line).
template <int C>
__global__ void __launch_bounds__(kThreads)
bin_scatter_kernel(const uint32_t *__restrict__ xy, const int64_t *__restrict__ t, CornerGeom g, Sorted so) {
    extern __shared__ int64_t lds64[];
    __shared__ int32_t wsum[kThreads / 64];
    const int nb = g.n_tiles + 1;
    int64_t *base = lds64;                                    // [nb] next free slot per bin
    int32_t *cnt = reinterpret_cast<int32_t *>(base + nb);    // [nb]
    int32_t *loff = cnt + nb;                                 // [nb]
    uint32_t *st_key = reinterpret_cast<uint32_t *>(loff + nb);  // [C]
    uint32_t *st_t = st_key + C;                                  // [C]
    uint16_t *st_bin = reinterpret_cast<uint16_t *>(st_t + C);    // [C]
    const int tid = threadIdx.x;
    const int64_t s = blockIdx.x;
    const int64_t lo = s * g.S, hi = (lo + g.S < g.n) ? lo + g.S : g.n;
    const int64_t grp = s / kGroup;
    const int64_t grp_first = grp * kGroup * (int64_t)g.S;
    int64_t t_first;
    const bool narrow = group_narrow(t, g, grp, &t_first);  // uniform
    for (int b = tid; b < nb; b += kThreads) {  // rel[] is only defined for bins the slice touches
        base[b] = so.bin_off[grp * nb + b] + so.rel[s * nb + b];
        cnt[b] = 0;
    }
    __syncthreads();
    constexpr int kPer = C / kThreads;
    for (int64_t c0 = lo; c0 < hi; c0 += C) {
        const int cn = (int)((hi - c0) < C ? (hi - c0) : C);
        uint32_t v[kPer];
        int bb[kPer], rr[kPer];
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int i = u * kThreads + tid;
            v[u] = (i < cn) ? xy[c0 + i] : 0u;
            bb[u] = (i < cn) ? tile_of(v[u], g) : -1;
            rr[u] = (i < cn) ? atomicAdd(&cnt[bb[u]], 1) : 0;
        }
        __syncthreads();
        block_excl_scan(cnt, loff, nb, wsum);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int i = u * kThreads + tid;
            if (i < cn) {
                const int pos = loff[bb[u]] + rr[u];
                st_key[pos] = tile_key(v[u], (uint32_t)(c0 + i - grp_first));
                if (narrow) st_t[pos] = (uint32_t)(t[c0 + i] - t_first);
                st_bin[pos] = (uint16_t)bb[u];
            }
        }
        __syncthreads();
        for (int i = tid; i < cn; i += kThreads) {
            const int b = st_bin[i];
            const int64_t gpos = base[b] + (i - loff[b]);
            so.key[gpos] = st_key[i];
            if (narrow) so.t32[gpos] = st_t[i];
        }
        __syncthreads();
        for (int b = tid; b < nb; b += kThreads) {
            base[b] += cnt[b];
            cnt[b] = 0;
        }
        __syncthreads();
    }
}

// 3a. Work items of the arc test: ceil(count / kItemEvents) per in-sensor bin.
__global__ void __launch_bounds__(kThreads)
item_count_kernel(CornerGeom g, Sorted so, int64_t n_bins) {
    const int64_t gb = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (gb >= n_bins) return;
    const int b = (int)(gb % (g.n_tiles + 1));
    so.n_items[gb] = (b == g.n_tiles) ? 0 : (so.bin_count[gb] + kItemEvents - 1) / kItemEvents;
}

__device__ __forceinline__ int64_t i1_of(int64_t i0, int64_t b1) {
    return (i0 + kItemEvents < b1) ? i0 + kItemEvents : b1;
}

__global__ void __launch_bounds__(kThreads)
item_fill_kernel(CornerGeom g, Sorted so, int64_t n_bins) {
    const int64_t gb = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (gb >= n_bins) return;
    const int nb = g.n_tiles + 1;
    const int64_t grp = gb / nb;
    const uint32_t b = (uint32_t)(gb % nb);
    const int m = so.n_items[gb];
    const int64_t first = so.item_off[grp * nb];
    const int64_t o = so.item_off[gb] - first;
    const int64_t b0 = so.bin_off[gb], b1 = so.bin_off[gb + 1];
    for (int c = 0; c < m; ++c) {
        const int64_t i0 = b0 + (int64_t)c * kItemEvents;
        so.items[grp * so.max_items + o + c] = make_uint4(b, (uint32_t)i0, (uint32_t)(i1_of(i0, b1)), 0u);
    }
    if (b == (uint32_t)(nb - 1)) so.grp_items[grp] = (int32_t)(so.item_off[gb + 1] - first);
}

__device__ __forceinline__ void tile_origin(const CornerGeom &g, int tile, int &x0, int &y0) {
    x0 = (tile % g.tiles_x) * kTile;
    y0 = (tile / g.tiles_x) * kTile;
}

// 3. Build group `grp` for one tile: fold group grp-1 (set `prv`) into B_out = fold(B_in) for
// the tile's pixels (dense; grp > 0), then accumulate mask/M of the tile's bin and store them
// into set `cur`.  The LDS keeps a u32 per (slice, pixel): the max group-relative timestamp + 1
// (narrow groups, from the sorted t32), else the max event index + 1 — timestamps are
// non-decreasing, so the last event carries the max t, gathered once per set pair at the end.
struct BuildLds {
    uint32_t mlast[kGroup][kTilePix];  // value + 1 (0 = none), 24.5 KiB
    uint32_t mask_l[kTilePix];
};

__device__ __forceinline__ void build_tile(const int64_t *__restrict__ t, const CornerGeom &g, int64_t grp,
                                           int tile, const Sorted &so,
                                           const GroupBufs &cur, const GroupBufs &prv,
                                           const int64_t *__restrict__ B_in, int64_t *__restrict__ B_out,
                                           BuildLds &L) {
    constexpr int kHalves = 2;  // 2 lanes per pixel (lanes >= 2 * kTilePix only load events)
    static_assert(kArcThreads >= kHalves * kTilePix, "build lanes");
    constexpr int kPlanes = kGroup / kHalves;
    const int tid = threadIdx.x;
    const int p = tid % kTilePix, part = tid / kTilePix;
    const bool pix_lane = part < kHalves;  // lanes beyond 2 x 256 only help with the events
    int x0, y0;
    tile_origin(g, tile, x0, y0);
    const int px = x0 + p % kTile, py = y0 + p / kTile;
    const bool own = pix_lane && px < g.W && py < g.H;
    const int64_t HW = (int64_t)g.H * g.W;
    const int64_t q = (int64_t)py * g.W + px;
    if (part == 0) {
        if (own && grp > 0) {
            const uint32_t mk = prv.mask[q];
            B_out[q] = mk ? prv.M[(int64_t)(31 - __clz(mk)) * HW + q] : B_in[q];
        }
        L.mask_l[p] = 0u;
    }
    if (pix_lane) {
#pragma unroll
        for (int jj = 0; jj < kPlanes; ++jj) L.mlast[part * kPlanes + jj][p] = 0u;
    }
    __syncthreads();
    const int nb = g.n_tiles + 1;
    const int64_t b0 = so.bin_off[grp * nb + tile], b1 = so.bin_off[grp * nb + tile + 1];
    int64_t t_first;
    const bool narrow = group_narrow(t, g, grp, &t_first);  // uniform
    for (int64_t i0 = b0; i0 < b1; i0 += kBuildUnroll * kArcThreads) {
        uint32_t k[kBuildUnroll], tv32[kBuildUnroll];
#pragma unroll
        for (int u = 0; u < kBuildUnroll; ++u) {
            const int64_t i = i0 + u * kArcThreads + tid;
            k[u] = (i < b1) ? so.key[i] : 0xffffffffu;
            tv32[u] = (i < b1 && narrow) ? so.t32[i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kBuildUnroll; ++u) {
            if (k[u] == 0xffffffffu) continue;
            const int lp = (int)(k[u] & 255u);
            const int j = slice_in_group(k[u] >> 8, g);
            atomicOr(&L.mask_l[lp], 1u << j);
            atomicMax(&L.mlast[j][lp], (narrow ? tv32[u] : (k[u] >> 8)) + 1u);
        }
    }
    __syncthreads();
    if (own) {
        const uint32_t mk_all = L.mask_l[p];
        if (part == 0) cur.mask[q] = mk_all;
        const int64_t grp_first = grp * kGroup * (int64_t)g.S;
        int64_t tv[kPlanes];  // all gathers in flight, then the stores
#pragma unroll
        for (int jj = 0; jj < kPlanes; ++jj) {
            const int j = part * kPlanes + jj;
            const uint32_t m = L.mlast[j][p] - 1u;
            tv[jj] = !((mk_all >> j) & 1u) ? 0 : narrow ? t_first + (int64_t)m : t[grp_first + m];
        }
#pragma unroll
        for (int jj = 0; jj < kPlanes; ++jj) {
            const int j = part * kPlanes + jj;
            if ((mk_all >> j) & 1u) cur.M[(int64_t)j * HW + q] = tv[jj];
        }
    }
}

// Final fold of the last group: B_out = fold(B_in) (dense; may be in place).
__global__ void __launch_bounds__(kThreads)
tile_fold_kernel(CornerGeom g, GroupBufs buf, const int64_t *B_in, int64_t *B_out) {
    int x0, y0;
    tile_origin(g, blockIdx.x, x0, y0);
    if (threadIdx.x >= kTilePix) return;
    const int px = x0 + threadIdx.x % kTile, py = y0 + threadIdx.x / kTile;
    if (px >= g.W || py >= g.H) return;
    const int64_t q = (int64_t)py * g.W + px;
    const uint32_t mk = buf.mask[q];
    B_out[q] = mk ? buf.M[(int64_t)(31 - __clz(mk)) * (int64_t)g.H * g.W + q] : B_in[q];
}

template <int N, int SMIN, int SMAX>
__device__ __forceinline__ bool arc_streak(const int64_t (&v)[N]) {
    int cnt[N];
#pragma unroll
    for (int j = 0; j < N; ++j) cnt[j] = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
#pragma unroll
        for (int k = j + 1; k < N; ++k) {
            cnt[j] += (v[k] > v[j]) ? 1 : 0;
            cnt[k] += (v[j] > v[k]) ? 1 : 0;
        }
    }
    constexpr uint32_t full = (N == 32) ? 0xffffffffu : ((1u << N) - 1u);
    bool ok = false;
#pragma unroll
    for (int s = SMIN; s <= SMAX; ++s) {
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < N; ++j) m |= (cnt[j] < s ? 1u : 0u) << j;
        const uint32_t rot = ((m << 1) | (m >> (N - 1))) & full;  // bit j <- bit j-1
        const uint32_t starts = m & ~rot;
        ok |= (__popc(m) == s) && (__popc(starts) == 1);
    }
    return ok;
}

// ---- fast arc test on 32-bit keys ------------------------------------------------------------
// Values are mapped to v' = clamp(v - L, 0, 2^27 - 1) with L = t_last(group) - (2^27 - 1) and
// keyed as (v' << IB) | position.  Clamping merges the values <= L into ties at 0.  This cannot
// change the outcome when at least SMAX+1 values are unclamped: a witness k (the largest value
// outside the arc) has <= SMAX values above it, so it and its arc are unclamped and compare as
// before, while a clamped k' has every unclamped value (> SMAX of them) above it in both
// forms.  Otherwise (or when some value exceeds t_last) the exact int64 test runs.
constexpr int kVBits = 27;
constexpr uint32_t kVMax = (1u << kVBits) - 1u;

// Batcher odd-even merge sort, descending; with compile-time padding and only the top outputs
// used, dead compare-exchanges fold away.
template <int N>
__device__ __forceinline__ void sort_desc(uint32_t (&k)[N]) {
#pragma unroll
    for (int p = 1; p < N; p += p) {
#pragma unroll
        for (int kk = p; kk > 0; kk /= 2) {
#pragma unroll
            for (int j = kk % p; j + kk < N; j += kk + kk) {
#pragma unroll
                for (int i = 0; i < kk; ++i) {
                    if (i + j + kk < N && (i + j) / (p + p) == (i + j + kk) / (p + p)) {
                        const uint32_t a = k[i + j], b = k[i + j + kk];
                        k[i + j] = a > b ? a : b;
                        k[i + j + kk] = a > b ? b : a;
                    }
                }
            }
        }
    }
}

// 1 = arc found, 0 = none, -1 = undecidable on clamped keys (fewer than SMAX+1 unclamped and
// the clamped values not all equal).
template <int N, int NP, int IB, int SMIN, int SMAX>
__device__ __forceinline__ int arc_keys(uint32_t (&k)[NP], bool ties_exact) {
    sort_desc<NP>(k);
    if (!ties_exact && (k[SMAX] >> IB) == 0u) return -1;
    constexpr uint32_t full = (1u << N) - 1u;
    uint32_t m = 0;
    bool ok = false;
#pragma unroll
    for (int s = 1; s <= SMAX; ++s) {
        m |= 1u << (k[s - 1] & ((1u << IB) - 1u));
        if (s >= SMIN) {
            const bool sep = (k[s - 1] >> IB) > (k[s] >> IB);
            const uint32_t rot = ((m << 1) | (m >> (N - 1))) & full;
            ok |= sep && (__popc(m & ~rot) == 1);
        }
    }
    return ok ? 1 : 0;
}

// Staged neighbourhood of one work item: T[j][wp] = V'(window pixel wp, slice j of the group) —
// the clamped value the arc test of an event in slice j sees — so every circle lookup is one
// independent LDS read.  mask[] (the group mask per window pixel) serves the exact fallback.
struct ArcLds {
    uint32_t T[kGroup][kWinPix];  // 60.5 KiB
    union {
        uint32_t mask[kWinPix];  // staging: group mask per window pixel
        struct {                 // tests: bit j*256 + pixel-in-tile
            uint32_t pairs[kGroup * kTilePix / 32];  // (slice, pixel) pairs with an eligible event
            uint32_t res[kGroup * kTilePix / 32];    // ... that are corners
        } bits;
    } u;
    uint16_t word_off[kGroup * kTilePix / 32];  // exclusive prefix of popc(pairs)
    uint16_t q4[kItemEvents];                    // pairs that passed circle 3
    int64_t wave_min[kArcThreads / 64];
    int32_t wave_tot[kArcThreads / 64];
    int32_t exact_only;  // a value above t_last: clamped keys unusable
    int32_t mixed;       // clamped values not all equal to the window minimum of B
    int32_t q4n;
    int32_t n_tasks;
};

__device__ __forceinline__ uint32_t clamp_rel(int64_t v, int64_t L, int64_t vz, int32_t *exact_flag,
                                              int32_t *mixed_flag) {
    if (v <= L) {
        if (v != vz) *mixed_flag = 1;
        return 0u;
    }
    const int64_t d = v - L;
    if (d > (int64_t)kVMax) { *exact_flag = 1; return kVMax; }
    return (uint32_t)d;
}

// Exact int64 V(q_k, j) of N circle pixels from the global images in two dependent levels:
// all masks, then one selected address per pixel (no branch between a mask and its load).
template <int N>
__device__ __forceinline__ void sae_gather(int64_t q0, const int8_t *dy, const int8_t *dx, int W, uint32_t below,
                                           const GroupBufs &cur, const int64_t *__restrict__ B, int64_t HW,
                                           int64_t (&v)[N]) {
    uint32_t mk[N];
#pragma unroll
    for (int k = 0; k < N; ++k) mk[k] = cur.mask[q0 + (int64_t)dy[k] * W + dx[k]] & below;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const int64_t q = q0 + (int64_t)dy[k] * W + dx[k];
        const int64_t *p = mk[k] ? cur.M + (int64_t)(31 - __clz(mk[k])) * HW + q : B + q;
        v[k] = *p;
    }
}

// Exact int64 arc test of one circle from the global images (rare fallback; out of line so its
// registers do not raise the pressure of the main kernel body).
__device__ __noinline__ bool exact_circle_test(int x, int y, int j, bool c3, int W, const GroupBufs cur,
                                               const int64_t *__restrict__ B, int64_t HW) {
    const uint32_t below = (j == 31) ? 0xffffffffu : ((2u << j) - 1u);
    const int64_t q0 = (int64_t)y * W + x;
    if (c3) {
        int64_t v3[16];
        sae_gather<16>(q0, c3dy, c3dx, W, below, cur, B, HW, v3);
        return arc_streak<16, 3, 6>(v3);
    }
    int64_t v4[20];
    sae_gather<20>(q0, c4dy, c4dx, W, below, cur, B, HW, v4);
    return arc_streak<20, 4, 8>(v4);
}

// 4. Arc test of one work item (<= kItemEvents tile-sorted events of group `grp`).
#define ARC_STAMP(k)                                                                              \
    do {                                                                                          \
        if (ECC_CORNER_PROFILE && g.ts && grp == g.ts_grp && threadIdx.x == 0)                    \
            g.ts[(size_t)item_idx * 16 + 4 + (k)] = __builtin_amdgcn_s_memrealtime();             \
    } while (0)
__device__ __forceinline__ void arc_item(const int64_t *__restrict__ t, const CornerGeom &g, int64_t grp,
                                         int item_idx, const Sorted &so, const GroupBufs &cur,
                                         const int64_t *__restrict__ B, const int32_t *__restrict__ first_border,
                                         uint8_t *__restrict__ flags, ArcLds &L) {
    const uint4 rec = so.items[grp * so.max_items + item_idx];  // one load resolves the item
    if (item_idx >= so.grp_items[grp]) return;
    const int tile = (int)rec.x;
    const int64_t i0 = rec.y, i1 = rec.z;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t HW = (int64_t)g.H * g.W;
    int x0, y0;
    tile_origin(g, tile, x0, y0);
    const int wx0 = x0 - kHalo, wy0 = y0 - kHalo;
    const int64_t grp_first = grp * kGroup * (int64_t)g.S;
    const int64_t grp_end = (grp + 1) * kGroup * (int64_t)g.S;
    const int64_t Lt = t[(grp_end < g.n ? grp_end : g.n) - 1] - (int64_t)kVMax;
    if (ECC_CORNER_PROFILE && (g.dbg & 4)) return;
    if (i1 - i0 < kStageMinEvents) {
        // small item (sparse tile): staging 576 pixels would cost more than the events — exact
        // int64 test straight from the global images, one event per lane
        for (int64_t i = i0 + tid; i < i1; i += kArcThreads) {
            const uint32_t key = so.key[i];
            const int lp = (int)(key & 255u);
            const uint32_t el = key >> 8;
            const int x = x0 + lp % kTile, y = y0 + lp / kTile;
            const int j = slice_in_group(el, g);
            const int64_t s = grp * kGroup + j;
            bool test = s >= g.first_detect && !is_border(x, y, g);
            if (test && g.border_mode == 1) test = (int64_t)el - (int64_t)j * g.S < first_border[s];
            if (!test) continue;
            if (exact_circle_test(x, y, j, true, g.W, cur, B, HW) && exact_circle_test(x, y, j, false, g.W, cur, B, HW))
                flags[grp_first + el] = 1;
        }
        return;
    }
    if (tid == 0) {
        L.exact_only = 0;
        L.mixed = 0;
    }

    // keys of the item (preloaded; the loads overlap the staging)
    constexpr int kPerLane = (kItemEvents + kArcThreads - 1) / kArcThreads;
    uint32_t keys[kPerLane];
#pragma unroll
    for (int u = 0; u < kPerLane; ++u) {
        const int64_t i = i0 + tid + (int64_t)u * kArcThreads;
        keys[u] = (i < i1) ? so.key[i] : 0xffffffffu;
    }
    // (a) one lane per window pixel: its group mask and B, then the low 32 bits of its set M
    //     planes, issued before the barrier.  When the group spans < 2^27 ticks every M lies in
    //     (Lt, t_last], so M' = M - Lt is exact from the low words.  (Loading all 32 planes
    //     without waiting for the mask was measured slower: ~73 KB of extra L2 traffic per item.)
    static_assert(kArcThreads >= kWinPix, "one lane per window pixel");
    const int wp = tid;
    const bool win_lane = wp < kWinPix;
    const int wx = wx0 + wp % kWin, wy = wy0 + wp / kWin;
    const bool in = win_lane && wx >= 0 && wy >= 0 && wx < g.W && wy < g.H;
    const int64_t qq = (int64_t)wy * g.W + wx;
    const uint32_t mk = in ? cur.mask[qq] : 0u;
    const int64_t bq = in ? B[qq] : INT64_MAX;  // INT64_MAX: outside the sensor (never read)
    uint32_t v[kGroup];
    {  // only the planes whose mask bit is set (issued before the barrier below)
        const uint32_t *M32 = reinterpret_cast<const uint32_t *>(cur.M + (in ? qq : 0));
#pragma unroll
        for (int j = 0; j < kGroup; ++j) v[j] = ((mk >> j) & 1u) ? M32[(int64_t)j * HW * 2] : 0u;
    }
    if (win_lane) L.u.mask[wp] = mk;
    int64_t bmin = bq;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t x = __shfl_xor(bmin, o);
        bmin = x < bmin ? x : bmin;
    }
    if (lane == 0) L.wave_min[wave] = bmin;
    __syncthreads();
    int64_t vz = INT64_MAX;
#pragma unroll
    for (int w = 0; w < kArcThreads / 64; ++w) vz = L.wave_min[w] < vz ? L.wave_min[w] : vz;
    ARC_STAMP(0);
    if (ECC_CORNER_PROFILE && (g.dbg & 2)) return;
    // (b) forward fill along j in registers: T[j] = bit j set ? M'_j : T[j-1], T[-1] = B'
    const int64_t t_first = t[grp_first];
    const bool narrow = (Lt + (int64_t)kVMax) - t_first < (int64_t)kVMax;  // uniform
    uint32_t cur_v = (bq == INT64_MAX) ? 0u : clamp_rel(bq, Lt, vz, &L.exact_only, &L.mixed);
    if (!win_lane) {
    } else if (narrow) {
        const uint32_t lt32 = (uint32_t)Lt;
#pragma unroll
        for (int j = 0; j < kGroup; ++j) {
            cur_v = ((mk >> j) & 1u) ? v[j] - lt32 : cur_v;
            L.T[j][wp] = cur_v;
        }
    } else {
#pragma unroll 4
        for (int j = 0; j < kGroup; ++j) {
            if ((mk >> j) & 1u) cur_v = clamp_rel(cur.M[(int64_t)j * HW + qq], Lt, vz, &L.exact_only, &L.mixed);
            L.T[j][wp] = cur_v;
        }
    }
    __syncthreads();
    const bool fast = !L.exact_only;
    ARC_STAMP(1);
    if (ECC_CORNER_PROFILE && (g.dbg & 1)) return;
    const bool ties_exact = !L.mixed;
    // (d) the test depends only on (slice j, pixel): eligible events mark their pair in a bitmap,
    //     each distinct pair is tested once (one per lane; ~2.5x fewer tests than events on
    //     dense tiles), circle-3 survivors are queued so circle 4 runs densely, and every event
    //     finally reads its pair's result.  Eligibility (first slice, border, the border-mode-1
    //     cut at the slice's first border event) stays per event.
    constexpr int kPairWords = kGroup * kTilePix / 32;  // 196
    for (int w = tid; w < 2 * kPairWords; w += kArcThreads) (&L.u.bits.pairs[0])[w] = 0u;
    if (tid == 0) L.q4n = 0;
    __syncthreads();
    uint32_t pidx[kPerLane];
#pragma unroll
    for (int u = 0; u < kPerLane; ++u) {
        pidx[u] = 0xffffffffu;
        const uint32_t key = keys[u];
        if (key == 0xffffffffu) continue;
        const int lp = (int)(key & 255u);
        const uint32_t el = key >> 8;
        const int j = slice_in_group(el, g);
        const int64_t s = grp * kGroup + j;
        bool test = s >= g.first_detect && !is_border(x0 + lp % kTile, y0 + lp / kTile, g);
        if (test && g.border_mode == 1) test = (int64_t)el - (int64_t)j * g.S < first_border[s];
        if (!test) continue;
        pidx[u] = (uint32_t)(j * kTilePix + lp);
        atomicOr(&L.u.bits.pairs[pidx[u] >> 5], 1u << (pidx[u] & 31u));
    }
    __syncthreads();
    int wcnt = 0, wincl = 0;
    if (tid < kPairWords) {  // exclusive prefix of the words' popcounts (waves 0-3)
        wcnt = __popc(L.u.bits.pairs[tid]);
        wincl = wcnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(wincl, o);
            if (lane >= o) wincl += v;
        }
        if (lane == 63) L.wave_tot[wave] = wincl;
    }
    __syncthreads();
    if (tid < kPairWords) {
        int before = 0;
        for (int w = 0; w < wave; ++w) before += L.wave_tot[w];
        L.word_off[tid] = (uint16_t)(before + wincl - wcnt);
        if (tid == kPairWords - 1) L.n_tasks = before + wincl;
    }
    __syncthreads();
    const int n_tasks = L.n_tasks;
    ARC_STAMP(2);
    auto task_pair = [&](int ti) {  // ti-th set bit of the pair bitmap
        int lo = 0, hi = kPairWords;
#pragma unroll
        for (int step = 0; step < 8; ++step) {  // 2^8 >= kPairWords
            const int mid = (lo + hi) >> 1;
            if ((int)L.word_off[mid] <= ti) lo = mid; else hi = mid;
        }
        uint32_t m = L.u.bits.pairs[lo];
        for (int r = ti - (int)L.word_off[lo]; r > 0; --r) m &= m - 1;
        return lo * 32 + (__ffs(m) - 1);
    };
    auto exact_circle = [&](int x, int y, int j, bool c3) {
        return exact_circle_test(x, y, j, c3, g.W, cur, B, HW);
    };
    for (int ti = tid; ti < n_tasks; ti += kArcThreads) {
        const int pi = task_pair(ti);
        const int j = pi / kTilePix, lp = pi % kTilePix;
        const int x = x0 + lp % kTile, y = y0 + lp / kTile;
        const int wp0 = (y - wy0) * kWin + (x - wx0);
        int res = -1;
        if (fast) {
            const uint32_t *Tj = L.T[j];
            uint32_t k3[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) k3[k] = (Tj[wp0 + c3dy[k] * kWin + c3dx[k]] << 4) | k;
            res = arc_keys<16, 16, 4, 3, 6>(k3, ties_exact);
        }
        if (res < 0) res = exact_circle(x, y, j, true) ? 1 : 0;
        if (res == 1) L.q4[atomicAdd(&L.q4n, 1)] = (uint16_t)pi;
    }
    __syncthreads();
    const int n4 = L.q4n;
    ARC_STAMP(3);
    for (int qi = tid; qi < n4; qi += kArcThreads) {
        const int pi = L.q4[qi];
        const int j = pi / kTilePix, lp = pi % kTilePix;
        const int x = x0 + lp % kTile, y = y0 + lp / kTile;
        const int wp0 = (y - wy0) * kWin + (x - wx0);
        int res = -1;
        if (fast) {
            const uint32_t *Tj = L.T[j];
            uint32_t k4[32];
#pragma unroll
            for (int k = 0; k < 20; ++k) k4[k] = (Tj[wp0 + c4dy[k] * kWin + c4dx[k]] << 5) | k;
#pragma unroll
            for (int k = 20; k < 32; ++k) k4[k] = 0u;
            res = arc_keys<20, 32, 5, 4, 8>(k4, ties_exact);
        }
        if (res < 0) res = exact_circle(x, y, j, false) ? 1 : 0;
        if (res == 1) atomicOr(&L.u.bits.res[pi >> 5], 1u << (pi & 31));
    }
    __syncthreads();
    ARC_STAMP(4);
#pragma unroll
    for (int u = 0; u < kPerLane; ++u)
        if (pidx[u] != 0xffffffffu && ((L.u.bits.res[pidx[u] >> 5] >> (pidx[u] & 31u)) & 1u))
            flags[grp_first + (keys[u] >> 8)] = 1;
}

// One launch per group g: workgroups [0, n_arc) test the work items of group g, the rest build
// group g+1 (one tile each).  Both read set g&1; the build writes set (g+1)&1 and
// B_{g+1} = fold(B_g) into the other B buffer, so nothing the arc test reads changes under it.
union GroupLds {
    ArcLds arc;
    BuildLds build;
};

__global__ void __launch_bounds__(kArcThreads, 4)  // two 8-wave workgroups per CU
group_kernel(const int64_t *__restrict__ t, CornerGeom g, int64_t grp, int n_arc, Sorted so,
             GroupBufs cur, GroupBufs nxt, const int64_t *B_in, int64_t *B_out,
             const int32_t *__restrict__ first_border, uint8_t *__restrict__ flags) {
    __shared__ GroupLds L;
    const bool rec = ECC_CORNER_PROFILE && g.ts && grp == g.ts_grp && threadIdx.x == 0;
    unsigned long long t_start = rec ? __builtin_amdgcn_s_memrealtime() : 0;
    if ((int)blockIdx.x < n_arc) {  // long arc items first, short build workgroups fill in after
        if (!(ECC_CORNER_PROFILE && (g.dbg & 8))) arc_item(t, g, grp, (int)blockIdx.x, so, cur, B_in, first_border, flags, L.arc);
    } else {
        build_tile(t, g, grp + 1, (int)blockIdx.x - n_arc, so, nxt, cur, B_in, B_out, L.build);
    }
    if (rec) {
        unsigned int hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        unsigned int xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g.ts[blockIdx.x * 16 + 0] = t_start;
        g.ts[blockIdx.x * 16 + 1] = __builtin_amdgcn_s_memrealtime();
        g.ts[blockIdx.x * 16 + 2] = ((int)blockIdx.x < n_arc && (int)blockIdx.x < so.grp_items[grp])
                                       ? (so.items[grp * so.max_items + blockIdx.x].z - so.items[grp * so.max_items + blockIdx.x].y)
                                       : 0xfffff;
        g.ts[blockIdx.x * 16 + 3] = xcc;
    }
}

// Plain final-SAE scatter (no detection): sae[q] = max t.
__global__ void __launch_bounds__(kThreads)
sae_scatter_kernel(const uint32_t *__restrict__ xy, const int64_t *__restrict__ t, int64_t n,
                   int W, int H, int64_t *__restrict__ sae) {
    for (int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x; e < n;
         e += (int64_t)gridDim.x * kThreads) {
        const uint32_t v = xy[e];
        const int x = ecc::xy_x(v), y = ecc::xy_y(v);
        if (x < W && y < H)
            atomicMax(reinterpret_cast<long long *>(&sae[(int64_t)y * W + x]), (long long)t[e]);
    }
}

__global__ void __launch_bounds__(kThreads)
sae_max_combine_kernel(const int64_t *__restrict__ images, int n_images, int64_t hw,
                       int64_t *__restrict__ out) {
    for (int64_t q = (int64_t)blockIdx.x * kThreads + threadIdx.x; q < hw;
         q += (int64_t)gridDim.x * kThreads) {
        int64_t m = images[q];
        for (int i = 1; i < n_images; ++i) m = max(m, images[(int64_t)i * hw + q]);
        out[q] = m;
    }
}

// Per-context corner workspace: group images (sized by the sensor) and the sorted batch with
// its bin tables (sized by the batch; grown, never shrunk).
struct CornerState {
    int W = 0, H = 0;
    void *img = nullptr;
    GroupBufs set[2]{};
    int64_t *b_alt = nullptr;  // second SAE buffer (B ping-pong with the caller's `sae`)
    void *evt = nullptr;
    size_t evt_bytes = 0;
};

std::mutex g_state_mu;
std::map<const ecc_ctx *, CornerState *> g_states;

CornerState *state_of(const ecc_ctx *ctx) {
    std::lock_guard<std::mutex> lk(g_state_mu);
    auto it = g_states.find(ctx);
    if (it != g_states.end()) return it->second;
    auto *s = new CornerState();
    g_states[ctx] = s;
    return s;
}

// Sequential carve of one allocation; with base == nullptr it only measures.
struct Carve {
    char *base;
    size_t used = 0;
    template <class T> T *take(size_t count) {
        T *r = base ? reinterpret_cast<T *>(base + used) : nullptr;
        used += ecc::align_up(count * sizeof(T), 256);
        return r;
    }
};

Sorted carve_sorted(Carve &cv, const CornerGeom &g, int64_t n_bins, int32_t **first_border,
                    int64_t **scan_scratch) {
    Sorted so{};
    so.key = cv.take<uint32_t>((size_t)g.n);
    so.t32 = cv.take<uint32_t>((size_t)g.n);
    so.bin_count = cv.take<int32_t>((size_t)n_bins);
    so.rel = cv.take<int32_t>((size_t)g.n_slices * (g.n_tiles + 1));
    so.bin_off = cv.take<int64_t>((size_t)n_bins + 1);
    so.n_items = cv.take<int32_t>((size_t)n_bins);
    so.item_off = cv.take<int64_t>((size_t)n_bins + 1);
    const int64_t n_groups = (g.n_slices + kGroup - 1) / kGroup;
    so.max_items = (int)(g.n_tiles + std::min<int64_t>((int64_t)kGroup * g.S, g.n) / kItemEvents);
    so.items = cv.take<uint4>((size_t)n_groups * so.max_items);
    so.grp_items = cv.take<int32_t>((size_t)n_groups);
    *first_border = cv.take<int32_t>((size_t)g.n_slices);
    *scan_scratch = cv.take<int64_t>((ecc::scan_scratch_bytes(n_bins) + 7) / 8);
    return so;
}

int corner_state_reserve(ecc_ctx *ctx, CornerState *st, const CornerGeom &g, size_t evt_need) {
    if (st->W != g.W || st->H != g.H || !st->img) {
        if (st->img) {
            ECC_CHECK_HIP(ctx, hipDeviceSynchronize(), "sync(corner images)");
            (void)hipFree(st->img);
            st->img = nullptr;
        }
        const size_t HW = (size_t)g.W * g.H;
        const size_t mask_b = ecc::align_up(HW * 4, 256);
        const size_t m_b = ecc::align_up(HW * 8 * kGroup, 256);
        const size_t b_b = ecc::align_up(HW * 8, 256);
        hipError_t e = hipMalloc(&st->img, 2 * mask_b + 2 * m_b + b_b);
        if (e != hipSuccess) {
            st->img = nullptr;
            ecc::hip_fail(ctx, e, "hipMalloc(corner images)");
            return ECC_ERR_NOMEM;
        }
        char *p = static_cast<char *>(st->img);
        for (int b = 0; b < 2; ++b) {
            st->set[b].mask = reinterpret_cast<uint32_t *>(p + b * mask_b);
            st->set[b].M = reinterpret_cast<int64_t *>(p + 2 * mask_b + b * m_b);
        }
        st->b_alt = reinterpret_cast<int64_t *>(p + 2 * mask_b + 2 * m_b);
        st->W = g.W;
        st->H = g.H;
    }
    if (evt_need > st->evt_bytes) {
        if (st->evt) {
            ECC_CHECK_HIP(ctx, hipDeviceSynchronize(), "sync(corner batch)");
            (void)hipFree(st->evt);
            st->evt = nullptr;
            st->evt_bytes = 0;
        }
        const size_t want = ecc::align_up(evt_need + evt_need / 8, 1 << 20);
        hipError_t e = hipMalloc(&st->evt, want);
        if (e != hipSuccess) {
            st->evt = nullptr;
            ecc::hip_fail(ctx, e, "hipMalloc(corner batch)");
            return ECC_ERR_NOMEM;
        }
        st->evt_bytes = want;
    }
    return ECC_OK;
}

unsigned blocks_for(int64_t n, int threads) { return (unsigned)((n + threads - 1) / threads); }

}  // namespace

namespace ecc {
void corner_state_release(const ecc_ctx *ctx) {
    CornerState *st = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_state_mu);
        auto it = g_states.find(ctx);
        if (it == g_states.end()) return;
        st = it->second;
        g_states.erase(it);
    }
    if (st->img) (void)hipFree(st->img);
    if (st->evt) (void)hipFree(st->evt);
    delete st;
}
}  // namespace ecc

ECC_API void ecc_corner_cfg_default(ecc_corner_cfg *cfg) {
    if (!cfg) return;
    cfg->width = 1280;            // hard-coded bounds of the reference arc test (:952-953)
    cfg->height = 720;
    cfg->slice_events = 16384;    // make_n_events(nevents = ARRAY_SIZE), :745, :772-774
    cfg->margin = 4;              // cs = max_scale * 4, :948-951
    cfg->border_mode = 0;         // fixed; 1 = ref_compat `break` (Q11)
    cfg->first_detect_slice = 1;  // time_surface_flag (Q15)
}

ECC_API int ecc_fast_detect(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n,
                            const ecc_corner_cfg *cfg, int64_t *sae, uint8_t *corner_flags,
                            ecc_stream_t stream) {
    if (!ctx || !cfg || !sae || n < 0) return ECC_ERR_INVALID;
    if (n > 0 && (!xy || !t || !corner_flags)) return ECC_ERR_INVALID;
    if (cfg->width < 1 || cfg->height < 1 || cfg->width > 65536 || cfg->height > 65536)
        return ECC_ERR_INVALID;
    if (cfg->margin < 4 || 2 * cfg->margin >= cfg->width || 2 * cfg->margin >= cfg->height)
        return ECC_ERR_INVALID;  // the circles reach 4 px from the event
    if (cfg->slice_events < 1 || cfg->slice_events > kMaxSlice ||
        (cfg->border_mode != 0 && cfg->border_mode != 1))
        return ECC_ERR_INVALID;
    CornerGeom g{};
    g.W = cfg->width;
    g.H = cfg->height;
    g.S = cfg->slice_events;
    g.inv_S = 1.0f / (float)g.S;
    g.dbg = 0;
    g.ts = nullptr;
    g.ts_grp = -1;
#if ECC_CORNER_PROFILE
    g.dbg = getenv("ECC_CORNER_DBG") ? atoi(getenv("ECC_CORNER_DBG")) : 0;
    static unsigned long long *ts_buf = nullptr;
    g.ts_grp = getenv("ECC_CORNER_TS") ? atoi(getenv("ECC_CORNER_TS")) : -1;
    if (g.ts_grp >= 0) {
        if (!ts_buf) (void)hipMalloc(&ts_buf, 1 << 20);
        (void)hipMemset(ts_buf, 0, 1 << 20);
        g.ts = ts_buf;
    }
#endif
    g.margin = cfg->margin;
    g.border_mode = cfg->border_mode;
    g.first_detect = cfg->first_detect_slice;
    g.tiles_x = (g.W + kTile - 1) / kTile;
    g.n_tiles = g.tiles_x * ((g.H + kTile - 1) / kTile);
    if (g.n_tiles > kMaxTiles) return ECC_ERR_INVALID;  // > 8191 16x16 tiles (~2.1 Mpixel)
    g.n = n;
    g.n_slices = (n + g.S - 1) / g.S;
    if (g.n_slices > INT32_MAX) return ECC_ERR_INVALID;
    hipStream_t s = ecc::as_stream(stream);
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    ECC_CHECK_HIP(ctx, hipMemsetAsync(ctx->flags, 0, 4, s), "memset(err flag)");
    if (n == 0) return ECC_OK;
    const int nb = g.n_tiles + 1;
    const int64_t n_groups = (g.n_slices + kGroup - 1) / kGroup;
    const int64_t n_bins = n_groups * nb;
    CornerState *st = state_of(ctx);
    int32_t *first_border = nullptr;
    int64_t *scan_scratch = nullptr;
    Carve measure{nullptr};
    carve_sorted(measure, g, n_bins, &first_border, &scan_scratch);
    int rc = corner_state_reserve(ctx, st, g, measure.used);
    if (rc) return rc;
    Carve cv{static_cast<char *>(st->evt)};
    const Sorted so = carve_sorted(cv, g, n_bins, &first_border, &scan_scratch);

    ECC_CHECK_HIP(ctx, hipMemsetAsync(corner_flags, 0, (size_t)n, s), "memset(flags)");
    ECC_CHECK_HIP(ctx, hipMemsetAsync(so.bin_count, 0, (size_t)n_bins * 4, s), "memset(bins)");
    if (g.border_mode == 1)
        ECC_CHECK_HIP(ctx, hipMemsetAsync(first_border, 0x7f, (size_t)g.n_slices * 4, s), "memset(fb)");
    {
        ECC_TIMED(ctx, s, "bin_hist_kernel");
        hipLaunchKernelGGL(bin_hist_kernel, dim3((unsigned)g.n_slices), dim3(kThreads), nb * 4, s, xy, t,
                           g, so, first_border, ctx->flags);
    }
    rc = ecc::exclusive_scan_i32_i64(ctx, so.bin_count, n_bins, so.bin_off, scan_scratch, s);
    if (rc) return rc;
    {
        ECC_TIMED(ctx, s, "bin_scatter_kernel");
        const size_t lds_big = (size_t)nb * 16 + 2048 * 10, lds_small = (size_t)nb * 16 + 1024 * 10;
        if (lds_big <= 40 * 1024)  // 4 workgroups per CU
            hipLaunchKernelGGL(bin_scatter_kernel<2048>, dim3((unsigned)g.n_slices), dim3(kThreads), lds_big, s, xy,
                               t, g, so);
        else
            hipLaunchKernelGGL(bin_scatter_kernel<1024>, dim3((unsigned)g.n_slices), dim3(kThreads), lds_small, s,
                               xy, t, g, so);
    }
    {
        ECC_TIMED(ctx, s, "item_count_kernel");
        hipLaunchKernelGGL(item_count_kernel, dim3(blocks_for(n_bins, kThreads)), dim3(kThreads), 0, s, g,
                           so, n_bins);
    }
    rc = ecc::exclusive_scan_i32_i64(ctx, so.n_items, n_bins, so.item_off, scan_scratch, s);
    if (rc) return rc;
    {
        ECC_TIMED(ctx, s, "item_fill_kernel");
        hipLaunchKernelGGL(item_fill_kernel, dim3(blocks_for(n_bins, kThreads)), dim3(kThreads), 0, s, g,
                           so, n_bins);
    }
    // upper bound of the work items of one group: one partial item per tile + full items
    const int64_t grp_events = std::min<int64_t>((int64_t)kGroup * g.S, n);
    const int64_t arc_blocks = g.n_tiles + grp_events / kItemEvents;
    if (arc_blocks > INT32_MAX) return ECC_ERR_INVALID;
    // B_g lives in bufB[g & 1]: B_0 = the caller's sae, B_1 = b_alt, ...
    int64_t *bufB[2] = {sae, st->b_alt};
    {
        ECC_TIMED(ctx, s, "group_kernel");  // build(0) only
        hipLaunchKernelGGL(group_kernel, dim3(g.n_tiles), dim3(kArcThreads), 0, s, t, g, (int64_t)-1, 0, so, st->set[1], st->set[0], (const int64_t *)bufB[0], bufB[1], (const int32_t *)first_border,
                           corner_flags);
    }
    for (int64_t gi = 0; gi < n_groups; ++gi) {
        const int n_build = (gi + 1 < n_groups) ? g.n_tiles : 0;
        ECC_TIMED(ctx, s, "group_kernel");
        hipLaunchKernelGGL(group_kernel, dim3((unsigned)(n_build + arc_blocks)), dim3(kArcThreads), 0, s, t, g, gi,
                           (int)arc_blocks, so, st->set[gi & 1], st->set[(gi + 1) & 1], (const int64_t *)bufB[gi & 1],
                           bufB[(gi + 1) & 1], (const int32_t *)first_border, corner_flags);
    }
    {
        ECC_TIMED(ctx, s, "tile_fold_kernel");  // B_G into the caller's buffer
        hipLaunchKernelGGL(tile_fold_kernel, dim3(g.n_tiles), dim3(kThreads), 0, s, g, st->set[(n_groups - 1) & 1],
                           (const int64_t *)bufB[(n_groups - 1) & 1], sae);
    }
    ECC_CHECK_LAUNCH(ctx, "fast_detect");
#if ECC_CORNER_PROFILE
    if (g.ts) {
        (void)hipStreamSynchronize(s);
        static unsigned long long hb[1 << 17];
        (void)hipMemcpy(hb, g.ts, 1 << 20, hipMemcpyDeviceToHost);
        FILE *f = fopen(getenv("ECC_CORNER_TS_FILE") ? getenv("ECC_CORNER_TS_FILE") : "/tmp/ts.bin", "wb");
        if (f) { fwrite(hb, 1, 1 << 20, f); fclose(f); }
    }
#endif
    return ECC_OK;
}

ECC_API int ecc_fast_detect_status(ecc_ctx *ctx, ecc_stream_t stream) {
    if (!ctx) return ECC_ERR_INVALID;
    int32_t f = 0;
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(&f, ctx->flags, 4, hipMemcpyDeviceToHost, ecc::as_stream(stream)),
                  "read err flag");
    ECC_CHECK_HIP(ctx, hipStreamSynchronize(ecc::as_stream(stream)), "sync");
    return f ? ECC_ERR_UNSORTED_TIME : ECC_OK;
}

ECC_API int ecc_sae_scatter(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n,
                            int32_t width, int32_t height, int64_t *sae, ecc_stream_t stream) {
    if (!ctx || !sae || n < 0 || width < 1 || height < 1) return ECC_ERR_INVALID;
    if (n == 0) return ECC_OK;
    if (!xy || !t) return ECC_ERR_INVALID;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    const int64_t blocks = std::min<int64_t>((n + kThreads - 1) / kThreads, 4096);
    {
        ECC_TIMED(ctx, ecc::as_stream(stream), "sae_scatter_kernel");
        hipLaunchKernelGGL(sae_scatter_kernel, dim3((unsigned)blocks), dim3(kThreads), 0,
                           ecc::as_stream(stream), xy, t, n, width, height, sae);
    }
    ECC_CHECK_LAUNCH(ctx, "sae_scatter");
    return ECC_OK;
}

ECC_API int ecc_sae_max_combine(ecc_ctx *ctx, const int64_t *images, int32_t n_images, int64_t hw,
                                int64_t *out, ecc_stream_t stream) {
    if (!ctx || !out || hw < 0 || n_images < 0 || (n_images > 0 && !images)) return ECC_ERR_INVALID;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    if (n_images == 0) {
        ECC_CHECK_HIP(ctx, hipMemsetAsync(out, 0, hw * 8, s), "memset(sae)");
        return ECC_OK;
    }
    if (hw == 0) return ECC_OK;
    const int64_t blocks = std::min<int64_t>((hw + kThreads - 1) / kThreads, 4096);
    {
        ECC_TIMED(ctx, s, "sae_max_combine_kernel");
        hipLaunchKernelGGL(sae_max_combine_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s, images,
                           n_images, hw, out);
    }
    ECC_CHECK_LAUNCH(ctx, "sae_max_combine");
    return ECC_OK;
}
