// SAE (time surface) + FAST/arc corner detection.
//
// Reference: FCT/metavision_time_surface_periodic_group_track.cpp — per reslicer slice of
// 16384 events the aggregate lambda first writes time_surface.at(y,x) = t for EVERY event
// (:900-923, batch semantics Q14), then runs the eFAST arc test event by event on the CPU
// (:948-1063; circle3 streaks of 3..6 of 16 then circle4 streaks of 4..8 of 20, circles
// :44-45 as {dy,dx}), holding a mutex per event.
//
// Exact batch semantics for a whole batch with no per-slice (or per-group) launches.  The arc
// test of an event in slice s must see V(q,s) = t of the last event at pixel q with index
// < end(s).  Slices are taken in GROUPS of G = 32; with B_g = the SAE before group g,
// V(q,s) = the last t at q in slices j' <= j of the group (j = s mod 32), else B_g[q]
// (timestamps are non-decreasing, so max == last writer; a device check enforces it).
//
// Pipeline (every launch covers the whole batch):
//   bin_hist / scan / bin_scatter: counting sort by (group, 14x14-pixel TILE) into 4-byte keys
//       (event index within the group << 8 | pixel within the tile) + group-relative timestamps;
//   pair_build: per (group, tile) the distinct (slice, pixel) pairs with the value an arc test
//               reads there, in sub-region order; the slices that touched each pixel and its
//               last timestamp;
//   sae_prefix: per pixel, B_g for every group (prefix over groups) and the final SAE;
//   arc:        one 512-lane workgroup per (group, tile) for ALL groups at once: it stores the
//               pairs of the sub-regions its 22x22 window covers into per-slice LDS planes,
//               forward-fills them from B_g, and tests each distinct (slice, pixel) pair of
//               its tile once against LDS only;
//   flags:      per event in stream order, eligibility (Q11, Q15, border) && its pair's result.
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

namespace {

constexpr int kThreads = 256;
constexpr int kBuildUnroll = 8;
// ctx->flags[10]: the tag of the last sort phase that saw decreasing time (every sort phase gets
// a fresh host-side tag, so a stale word never matches a later call); flags[0]: the verdict
// sae_prefix_kernel published for the last finished call (pending word == its prepare's tag)
constexpr int kSortPendingWord = 10;
// the flag pass's dynamic LDS limit: 160 KiB less its static LDS (ctot[kFlagQuads][4], 128 B)
constexpr size_t kFlagDynLdsMax = 160 * 1024 - 256;
constexpr int kArcThreads = 512;  // 8 waves: one lane per window pixel (484) when staging
constexpr int kGroup = 32;         // slices per group (mask bits)
constexpr int kTile = 14;          // tile edge (pixels): the 22x22 window fits one 8-wave workgroup
constexpr int kTilePix = kTile * kTile;
constexpr int kHalo = 4;           // circle radius
constexpr int kWin = kTile + 2 * kHalo;  // 22
constexpr int kWinPix = kWin * kWin;     // 484
constexpr int kMaxTiles = 8191;          // bins per group = n_tiles + 1 (8192 fit an LDS histogram)
constexpr int kMaxSlice = 1 << 19;       // group-local event index must fit 24 bits

struct CornerGeom {
    int W, H, S, margin, border_mode, first_detect;
    int any_order;         // timestamps in any order: every group wide (index values, exact tests)
    int dedup_words;       // slice_sort's dedup bitmap: n_tiles * 196 bits (0: off, too large)
    int tiles_x, n_tiles;  // bin n_tiles of each group holds the events outside the sensor
    int seg_stride;        // words per slice of the slice-major corner pairs: n_tiles * 7, to 16 B
    float inv_S;
    int64_t n, n_slices;
};

// Batch sorted per slice by tile: slice s keeps its own range [s*S, s*S + len_s), and tile b of
// slice s is [s*S + toff[s][b], s*S + toff[s][b+1]) (row length n_tiles + 2: the outside-sensor
// bin n_tiles, then len_s).  A (group, tile) item's events are the 32 segments of its slices.
struct Sorted {
    uint32_t *key;   // (event index - first event of the group) << 8 | pixel in tile
    uint32_t *t32;   // t - t(first event of the group), written for groups spanning < 2^32 - 1
    int32_t *toff;   // [n_slices][n_tiles + 2]
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

__device__ __forceinline__ void tile_origin(const CornerGeom &g, int tile, int &x0, int &y0) {
    x0 = (tile % g.tiles_x) * kTile;
    y0 = (tile / g.tiles_x) * kTile;
}

// The group's events span < 2^32 - 1 ticks: t - t(first event) fits a u32 (+1 still fits).
__device__ __forceinline__ bool group_narrow(const int64_t *__restrict__ t, const CornerGeom &g, int64_t grp,
                                             int64_t *t_first) {
    const int64_t first = grp * kGroup * (int64_t)g.S;
    const int64_t end = (grp + 1) * kGroup * (int64_t)g.S;
    *t_first = t[first];
    if (g.any_order) return false;
    return (uint64_t)(t[(end < g.n ? end : g.n) - 1] - *t_first) < 0xffffffffull;
}

// Groups spanning < 2^24 - 1 ticks (the common case: 524288 events in under 16.7 s) are sorted
// into ONE 4-byte key per event, (t - t(first event of the group)) << 8 | pixel in tile: the
// slice an event belongs to is the slice segment it is read from.  Other groups keep the event
// index in the key and the relative timestamp in t32.
__device__ __forceinline__ bool group_fmt4(const int64_t *__restrict__ t, const CornerGeom &g, int64_t grp) {
    const int64_t first = grp * kGroup * (int64_t)g.S;
    const int64_t end = (grp + 1) * kGroup * (int64_t)g.S;
    if (g.any_order) return false;
    return (uint64_t)(t[(end < g.n ? end : g.n) - 1] - t[first]) < 0xFFFFFFull;
}

// floor(el / S) for el < 2^24 (float estimate, then exact correction).
__device__ __forceinline__ int slice_in_group(uint32_t el, const CornerGeom &g) {
    uint32_t q = (uint32_t)((float)el * g.inv_S);
    const uint32_t S = (uint32_t)g.S;
    q = (q * S > el) ? q - 1 : q;
    q = ((q + 1) * S <= el) ? q + 1 : q;
    return (int)q;
}

// 1. Per slice, one 1024-lane workgroup: counting sort of the slice's events by tile into the
// slice's own range (keys + group-relative timestamps), the per-slice tile offsets, the
// time-order check (Metavision stream order: t non-decreasing) and, for Q11, the slice's first
// border event.  Slices of <= 16384 events stay in registers (one read); longer ones take a
// counting pass and a placing pass.
// Two 1024-lane workgroups per CU (64 VGPRs: only each event's final key and tile/rank stay in
// registers), so one workgroup's loads overlap the other's LDS phases (one workgroup per CU left
// the CU idle outside its load phase).
constexpr int kSortThreads = 1024;
constexpr int kSortEPT = 16;
#ifndef ECC_SORT_FENCE
#define ECC_SORT_FENCE 4
#endif
constexpr int kSortFence = ECC_SORT_FENCE;  // events whose loads may be in flight together
constexpr int kSortChunk = kSortThreads * kSortEPT;
constexpr int kSortWaves = kSortThreads / 64;

// Per-slice (slice, pixel) dedup of the keys (groups with 4-byte keys, slices in one chunk, time
// order intact): an arc test reads, per (slice, pixel), only the largest timestamp, i.e. the key
// of the pixel's LAST event in the slice; pair_build takes the maximum of what it receives.  The
// slice's events are taken in kSortEPT rounds from the last (round u = events [1024 u, 1024 u +
// 1024)): an event is dropped when a LATER round already set its tile pixel's bit in an LDS
// bitmap (the staging area, not yet in use).  Events of one round at one pixel all stay (no
// ordering inside a round), so the maximum always survives.  ~46 % of the events remain on the
// bench's stream (40 % are distinct (slice, pixel) pairs), and pair_build reads only those.
#ifndef ECC_SORT_DEDUP_STEP
#define ECC_SORT_DEDUP_STEP 1  // event slots per dedup round (a divisor of kSortEPT)
#endif
constexpr int kSortDedupStep = ECC_SORT_DEDUP_STEP;
#ifndef ECC_SORT_DEDUP
#define ECC_SORT_DEDUP 1
#endif

// Block-wide exclusive scan in place of a[0, n) (kSortThreads threads, each a contiguous run);
// returns the total to every thread.
__device__ __forceinline__ int block_excl_scan_inplace(int32_t *a, int n, int32_t *wsum) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int per = (n + kSortThreads - 1) / kSortThreads;
    const int b0 = min(n, tid * per), b1 = min(n, b0 + per);
    int sum = 0;
    for (int i = b0; i < b1; ++i) sum += a[i];
    const int incl = ecc::wave_incl_scan(sum);  // DPP
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int run = incl - sum, total = 0;
    for (int w = 0; w < kSortThreads / 64; ++w) {
        run += w < wave ? wsum[w] : 0;
        total += wsum[w];
    }
    for (int i = b0; i < b1; ++i) {
        const int c = a[i];
        a[i] = run;
        run += c;
    }
    return total;
}

__global__ void __launch_bounds__(kSortThreads, 8)  // 8 waves/SIMD: two workgroups per CU
slice_sort_kernel(const uint32_t *__restrict__ xy, const int64_t *__restrict__ t, CornerGeom g, Sorted so,
                  int32_t *__restrict__ first_border, int32_t *__restrict__ err, int32_t tag,
                  uint32_t *__restrict__ zero0, int32_t *__restrict__ zero1) {
    extern __shared__ int32_t hist[];  // [nb]: counts, then offsets, then (long slices) cursors;
                                       // then [kSortChunk] staging (single slices: the keys in
                                       // event order, then in tile order); then the dedup bitmap
    __shared__ int32_t wsum[kSortThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63;
    const int64_t s = blockIdx.x;
    // the call's counters that later kernels of the call start from (a 4-B memset each was a
    // fill launch on the critical path): arc_kernel's overflow count, the NMS error word.  The
    // sort verdict needs no reset: a workgroup that sees decreasing time writes this call's tag.
    if (s == 0 && tid == 0) {
        if (zero0) *zero0 = 0u;
        if (zero1) *zero1 = 0;
    }
    const int64_t lo = s * g.S;
    const int len = (int)((lo + g.S < g.n ? lo + g.S : g.n) - lo);
    const int64_t grp = s / kGroup;
    const int64_t grp_first = grp * kGroup * (int64_t)g.S;
    int64_t t_first;
    const bool narrow = group_narrow(t, g, grp, &t_first);  // uniform
    const bool fmt4 = group_fmt4(t, g, grp);                // uniform
    const int nb = g.n_tiles + 1;
    const bool single = len <= kSortChunk;
    const bool dedup = ECC_SORT_DEDUP && single && fmt4 && g.dedup_words > 0;  // uniform
    uint32_t *stage = reinterpret_cast<uint32_t *>(hist + nb);
    uint32_t *bm = stage + kSortChunk;  // the dedup bitmap
    for (int b = tid; b < nb; b += kSortThreads) hist[b] = 0;
    if (dedup)
        for (int w = tid; w < g.dedup_words; w += kSortThreads) bm[w] = 0u;
    __syncthreads();
    bool bad = false;
    int fb = 0x7fffffff;
    // per event only tile << 16 | rank stays in registers (single slices: rank < 2^14); the key,
    // formed at load time, waits in the staging area in event order (in registers, it held 16
    // VGPRs through the load phase)
    uint32_t br[kSortEPT];
    const uint32_t *__restrict__ xs = xy + lo;
    const int64_t *__restrict__ ts = t + lo;
    for (int c0 = 0; c0 < len; c0 += kSortChunk) {  // one iteration for single slices
#pragma unroll
        for (int u = 0; u < kSortEPT; ++u) {
            // a compiler fence every kSortFence events keeps later loads from being hoisted above
            // earlier uses (all 16 events' loads in flight would spill)
            if (u > 0 && u % kSortFence == 0) asm volatile("" ::: "memory");
            const int i = c0 + u * kSortThreads + tid;
            const bool ok = i < len;
            const int ic = ok ? i : len - 1;  // clamped: unconditional loads off uniform bases
            const uint32_t v = xs[ic];
            const int64_t tc = ts[ic];
            // the previous event's t: a coalesced load of the neighbouring element (cache hit)
            const int64_t tp = (ic > 0 || lo > 0) ? ts[ic - 1] : INT64_MIN;
            bad |= ok && tp > tc;
            if (single) stage[u * kSortThreads + tid] = tile_key(v, fmt4 ? (uint32_t)(tc - t_first) : (uint32_t)(lo + i - grp_first));
            br[u] = ok ? (uint32_t)tile_of(v, g) << 16 : 0xffffffffu;
            if (ok && is_border(ecc::xy_x(v), ecc::xy_y(v), g)) fb = min(fb, i);
        }
        if (dedup && !__syncthreads_or(bad)) {  // uniform (single slices: one pass of this loop)
            // rounds of kSortDedupStep event slots, latest first: an event is dropped when a later
            // round already holds its (slice, pixel); events of one round are not compared with
            // each other (pair_build's atomicMax keeps the last of what remains)
#pragma unroll
            for (int u0 = kSortEPT - 1; u0 >= 0; u0 -= kSortDedupStep) {
                bool drop[kSortDedupStep];
                uint32_t tp[kSortDedupStep];
                bool cand[kSortDedupStep];
#pragma unroll
                for (int d = 0; d < kSortDedupStep; ++d) {
                    const int u = u0 - d;
                    const uint32_t b = br[u] >> 16;  // 0xffff: no event; n_tiles: outside the sensor (kept)
                    cand[d] = b < (uint32_t)g.n_tiles;
                    tp[d] = b * kTilePix + (stage[u * kSortThreads + tid] & 255u);  // own key
                    drop[d] = u0 < kSortEPT - 1 && cand[d] && ((bm[tp[d] >> 5] >> (tp[d] & 31u)) & 1u);
                }
                if (u0 < kSortEPT - 1) __syncthreads();  // every check of the round before its bits are set
#pragma unroll
                for (int d = 0; d < kSortDedupStep; ++d) {
                    if (drop[d]) br[u0 - d] = 0xffffffffu;
                    else if (cand[d]) atomicOr(&bm[tp[d] >> 5], 1u << (tp[d] & 31u));
                }
                if (u0 - kSortDedupStep >= 0) __syncthreads();  // the round's bits before the next checks
            }
        }
#pragma unroll
        for (int u = 0; u < kSortEPT; ++u) {
            if (br[u] == 0xffffffffu) continue;
            br[u] |= (uint32_t)atomicAdd(&hist[br[u] >> 16], 1) & 0xffffu;
        }
    }
    if (__any(bad) && lane == 0 && !g.any_order) *err = tag;  // pending: published by sae_prefix_kernel
    fb = ecc::wave_min_i32(fb);  // DPP
    if (lane == 0) wsum[tid >> 6] = fb;
    __syncthreads();
    if (tid == 0) {
        int m = 0x7fffffff;
        for (int w = 0; w < kSortThreads / 64; ++w) m = min(m, wsum[w]);
        first_border[s] = m;
    }
    __syncthreads();
    const int kept = block_excl_scan_inplace(hist, nb, wsum);  // len, less the dropped events
    __syncthreads();
    int32_t *row = so.toff + s * (int64_t)(nb + 1);
    for (int b = tid; b < nb; b += kSortThreads) row[b] = hist[b];
    if (tid == 0) row[nb] = kept;
    if (single) {  // place keys, then timestamps, in tile order in LDS; write both out contiguously
        uint32_t kv[kSortEPT];
#pragma unroll
        for (int u = 0; u < kSortEPT; ++u) kv[u] = stage[u * kSortThreads + tid];  // own keys
        __syncthreads();  // every key read before the stage is permuted
#pragma unroll
        for (int u = 0; u < kSortEPT; ++u)
            if (br[u] != 0xffffffffu) stage[hist[br[u] >> 16] + (br[u] & 0xffffu)] = kv[u];
        __syncthreads();
        for (int i = tid; i < kept; i += kSortThreads) so.key[lo + i] = stage[i];
        if (fmt4 || !narrow) return;  // (no dedup below: kept == len)
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kSortEPT; ++u)  // rare (groups spanning >= 2^24 ticks): t read again
            if (br[u] != 0xffffffffu) stage[hist[br[u] >> 16] + (br[u] & 0xffffu)] = (uint32_t)(t[lo + u * kSortThreads + tid] - t_first);
        __syncthreads();
        for (int i = tid; i < len; i += kSortThreads) so.t32[lo + i] = stage[i];
        return;
    }
    __syncthreads();  // row written before the offsets turn into cursors
    for (int c0 = 0; c0 < len; c0 += kSortThreads) {
        const int i = c0 + tid;
        if (i >= len) continue;
        const uint32_t vv = xy[lo + i];
        const int64_t pos = lo + atomicAdd(&hist[tile_of(vv, g)], 1);
        if (fmt4) {
            so.key[pos] = tile_key(vv, (uint32_t)(t[lo + i] - t_first));
        } else {
            so.key[pos] = tile_key(vv, (uint32_t)(lo + i - grp_first));
            if (narrow) so.t32[pos] = (uint32_t)(t[lo + i] - t_first);
        }
    }
}

// The 32 slice segments of one (group, tile) item, built by wave 0 into LDS (caller syncs):
// segment r = slice grp*32 + r; events are addressed by a flattened index i in [0, pref[32]).
// base = sum over the slices of toff[s][tile] = the item's offset inside the group's range when
// the group's items are laid out in tile order (used for its pair entries).
struct TileSegs {
    int64_t start[kGroup];
    int32_t pref[kGroup + 1];
    int64_t base;
};

__device__ __forceinline__ void tile_segs(const CornerGeom &g, const Sorted &so, int64_t grp, int tile, TileSegs &T) {
    const int tid = threadIdx.x;
    if (tid >= 64) return;
    const int64_t s = grp * kGroup + tid;
    int a = 0, len = 0;
    if (tid < kGroup && s < g.n_slices) {
        const int32_t *row = so.toff + s * (int64_t)(g.n_tiles + 2);
        a = row[tile];
        len = row[tile + 1] - a;
    }
    const int incl = ecc::wave_incl_scan(len);         // DPP (wave 0: all 64 lanes)
    const int asum = ecc::wave_sum_i32(a);  // < 32 * S <= 2^24: a 32-bit sum
    if (tid < kGroup) {
        T.start[tid] = s * g.S + a;
        T.pref[tid + 1] = incl;
    }
    if (tid == 0) {
        T.pref[0] = 0;
        T.base = asum;
    }
}

__device__ __forceinline__ int64_t seg_at(const TileSegs &T, int i, int &r) {
    r = 0;
#pragma unroll
    for (int step = kGroup / 2; step > 0; step >>= 1)
        if (T.pref[r + step] <= i) r += step;
    return T.start[r] + (i - T.pref[r]);
}

// Group time reference: L = t_last(group) - (2^27 - 1).  In a narrow group (span < 2^27 - 1
// ticks) every value v of the group maps exactly to v' = v - L in [1, 2^27 - 1]; in a wide group
// the stored value is the event index within the group + 1 (the exact test gathers t).
constexpr int kVBits = 27;
constexpr uint32_t kVMax = (1u << kVBits) - 1u;

struct GroupRef {
    int64_t first, t_first, Lt;
    bool narrow;
    uint32_t dlt;  // t32 + dlt = t - Lt (narrow)
};

__device__ __forceinline__ GroupRef group_ref(const int64_t *__restrict__ t, const CornerGeom &g, int64_t grp) {
    GroupRef r;
    r.first = grp * kGroup * (int64_t)g.S;
    const int64_t end = (grp + 1) * kGroup * (int64_t)g.S;
    r.t_first = t[r.first];
    r.Lt = t[(end < g.n ? end : g.n) - 1] - (int64_t)kVMax;
    // any order: the span of the first and last timestamps says nothing about the others
    r.narrow = !g.any_order && (r.Lt + (int64_t)kVMax) - r.t_first < (int64_t)kVMax;
    r.dlt = r.narrow ? (uint32_t)(r.t_first - r.Lt) : 0u;
    return r;
}

static_assert(kWin == kTile + 2 * kHalo, "window = tile + halo on both sides");
static_assert(kHalo >= 4, "the circles reach 4 px from the pixel under test");

// 3. Per (group, tile): the distinct (slice, pixel) pairs the tile's events touch, each with the
// value an arc test reads there (max over the slice's events at the pixel: v' or index + 1),
// stored PER PIXEL so that an arc workgroup stages a window pixel from its own fixed addresses,
// with no per-item offset table between its loads:
//   gmask[grp][q]  the slices that touched the pixel (bit j = slice j of the group),
//   pv[grp][q]     its values in ascending j: {v0, v1, v2, v3} when it has <= 4 of them, else
//                  {v0, v1, v2, x} with v3, v4, ... at ovf[4x], ovf[4x + 1], ... (16-B aligned, so
//                  an arc workgroup reads them as whole uint4s),
//   glast[grp][q]  its last timestamp.
// Item i's overflow values go to its own part of ovf: from (its place in the group's range with
// the group's items in tile order) + 4i, rounded up to 16 B.  A pixel with p > 4 values takes
// p - 3 rounded up to 4 words, at most p, and an item has at least as many events as pairs, so
// the 4 words per item cover the rounding and ovf needs n + 4 * n_items words.
constexpr int kRecVals = 4;  // values a pixel record holds inline

__global__ void __launch_bounds__(kThreads)
pair_build_kernel(const int64_t *__restrict__ t, CornerGeom g, Sorted so, uint32_t *__restrict__ ovf,
                  uint4 *__restrict__ pv, uint32_t *__restrict__ gmask, int64_t *__restrict__ glast) {
    __shared__ uint32_t tab[kGroup][kTilePix];  // 24.5 KiB
    __shared__ uint32_t pmask[kTilePix];        // slices that touched each tile pixel
    __shared__ int32_t wtot[kThreads / 64];
    __shared__ TileSegs segs;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t item = blockIdx.x;
    const int64_t grp = (int)item / g.n_tiles;  // n_items < 2^31 (host check): 32-bit division
    const int tile = (int)item % g.n_tiles;
    const int lp = tid < kTilePix ? tid : 0;  // this lane's tile pixel
    {
        uint4 *z = reinterpret_cast<uint4 *>(&tab[0][0]);
        for (int i = tid; i < (int)(sizeof(tab) / 16); i += kThreads) z[i] = make_uint4(0u, 0u, 0u, 0u);
        if (tid < kTilePix) pmask[tid] = 0u;
    }
    tile_segs(g, so, grp, tile, segs);
    const GroupRef gr = group_ref(t, g, grp);
    const bool fmt4 = group_fmt4(t, g, grp);  // uniform; the same test as slice_sort's
    __syncthreads();
    const int total = segs.pref[kGroup];
    if (fmt4) {  // 4-byte keys: slice = the segment, value = relative t + dlt
        for (int i0 = 0; i0 < total; i0 += kBuildUnroll * kThreads) {
            uint32_t k[kBuildUnroll];
            int r[kBuildUnroll];
#pragma unroll
            for (int u = 0; u < kBuildUnroll; ++u) {
                const int i = i0 + u * kThreads + tid;
                const int64_t gi = (i < total) ? seg_at(segs, i, r[u]) : 0;
                k[u] = (i < total) ? so.key[gi] : 0xffffffffu;
            }
#pragma unroll
            for (int u = 0; u < kBuildUnroll; ++u) {
                if (k[u] == 0xffffffffu) continue;
                atomicMax(&tab[r[u]][k[u] & 255u], (k[u] >> 8) + gr.dlt);
                atomicOr(&pmask[k[u] & 255u], 1u << r[u]);
            }
        }
    } else {
        for (int i0 = 0; i0 < total; i0 += kBuildUnroll * kThreads) {
            uint32_t k[kBuildUnroll], tv[kBuildUnroll];
#pragma unroll
            for (int u = 0; u < kBuildUnroll; ++u) {
                const int i = i0 + u * kThreads + tid;
                int r_unused;
                const int64_t gi = (i < total) ? seg_at(segs, i, r_unused) : 0;
                k[u] = (i < total) ? so.key[gi] : 0xffffffffu;
                tv[u] = (i < total && gr.narrow) ? so.t32[gi] : 0u;
            }
#pragma unroll
            for (int u = 0; u < kBuildUnroll; ++u) {
                if (k[u] == 0xffffffffu) continue;
                const uint32_t el = k[u] >> 8;
                const int jr = slice_in_group(el, g);
                atomicMax(&tab[jr][k[u] & 255u], gr.narrow ? tv[u] + gr.dlt : el + 1u);
                atomicOr(&pmask[k[u] & 255u], 1u << jr);
            }
        }
    }
    __syncthreads();
    // lane lp owns tile pixel lp: its slice mask, kept by one LDS atomicOr per event beside its
    // atomicMax (reading the pixel's 32 table words instead cost 32 LDS reads per pixel lane)
    const uint32_t m = tid < kTilePix ? pmask[lp] : 0u;
    const int cnt = __popc(m);
    const int nov = cnt > kRecVals ? (cnt - (kRecVals - 1) + 3) & ~3 : 0;  // past the first three, to 16 B
    const int incl = ecc::wave_incl_scan(nov);                  // DPP (all lanes active)
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    int off = incl - nov;
    for (int w = 0; w < wave; ++w) off += wtot[w];
    if (tid >= kTilePix) return;
    int x0, y0;
    tile_origin(g, tile, x0, y0);
    const int px = x0 + lp % kTile, py = y0 + lp / kTile;
    if (px >= g.W || py >= g.H) return;
    const int64_t q = grp * (int64_t)g.H * g.W + (int64_t)py * g.W + px;
    gmask[q] = m;
    if (!m) return;  // no slice touched it: arc workgroups never read its record
    // the pixel's overflow values at 16-B index x4 (off is a multiple of 4)
    const uint32_t x4 = (uint32_t)(((gr.first + segs.base + 4 * item + 3) >> 2) + (off >> 2));
    uint32_t *xo = ovf + 4 * (int64_t)x4 - (kRecVals - 1);
    static_assert(kRecVals == 4, "the record is one uint4");
    uint32_t r0 = 0u, r1 = 0u, r2 = 0u, r3 = x4;  // selects, not a register array indexed by k
    uint32_t v = 0u;
    int k = 0;
    for (uint32_t mm = m; mm; mm &= mm - 1u, ++k) {
        v = tab[__ffs(mm) - 1][lp];
        if (k == 0) r0 = v;
        else if (k == 1) r1 = v;
        else if (k == 2) r2 = v;
        else if (cnt == kRecVals) r3 = v;
        else xo[k] = v;
    }
    pv[q] = make_uint4(r0, r1, r2, r3);
    glast[q] = gr.narrow ? gr.Lt + (int64_t)v : t[gr.first + v - 1u];  // v: the newest slice's value
}

// 4. Per pixel, in place over the groups: gB[g] := B_g, the SAE before group g (the caller's
// `sae` for g = 0, then overwritten by the last event of every group that touched the pixel —
// the reference's `sae.at(y,x) = t`, :921-923); the caller's `sae` receives the final surface.
// The prefix is a "last value set" scan, which is associative: a workgroup takes 64 pixels (one
// per lane) and splits each run of 64 groups over its 4 waves (16 groups each); a wave finds the
// last value its groups set, the waves exchange those through LDS, and each then writes its
// groups' B_g from its incoming value.  (One thread per pixel walking all groups left 90 K
// threads for 256 CUs at 346x260: latency-bound at 31 us.)
constexpr int kPrefixPix = 64;
constexpr int kPrefixPer = 16;  // groups per wave per round
constexpr int kPrefixRound = kPrefixPer * (kThreads / 64);

__global__ void __launch_bounds__(kThreads)
sae_prefix_kernel(CornerGeom g, int64_t n_groups, const uint32_t *__restrict__ gmask, int64_t *__restrict__ gB,
                  int64_t *__restrict__ sae, int32_t *__restrict__ err_status,
                  int32_t *__restrict__ err_pending, int32_t tag,
                  uint32_t *__restrict__ zero0, int32_t *__restrict__ zero1) {
    // the call's sort verdict: its sort phase (finished before this kernel, in this call or in
    // the prepare it finishes) wrote its tag into the pending word iff it saw decreasing time;
    // publish it and consume the pending word (a captured graph replays the same tag, so each
    // replay must start from a clean word; a stale word from an abandoned prepare carries another
    // tag and never matches).
    // A finish-only call also zeroes the counters of its later kernels here (the arc kernels'
    // overflow count, the NMS error word), as slice_sort does in a one-call detection.
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *err_status = *err_pending == tag ? 1 : 0;
        *err_pending = 0;
        if (zero0) *zero0 = 0u;
        if (zero1) *zero1 = 0;
    }
    __shared__ int64_t s_last[kThreads / 64][kPrefixPix];
    __shared__ uint8_t s_has[kThreads / 64][kPrefixPix];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t HW = (int64_t)g.H * g.W;
    const int64_t q = (int64_t)blockIdx.x * kPrefixPix + lane;
    const bool in = q < HW;
    int64_t carry = in ? sae[q] : 0;  // B_0 = the caller's surface
    for (int64_t r0 = 0; r0 < n_groups; r0 += kPrefixRound) {
        const int64_t g0 = r0 + (int64_t)wave * kPrefixPer;
        uint32_t m[kPrefixPer];
        int64_t lt[kPrefixPer];
#pragma unroll
        for (int u = 0; u < kPrefixPer; ++u) m[u] = (in && g0 + u < n_groups) ? gmask[(g0 + u) * HW + q] : 0u;
#pragma unroll
        for (int u = 0; u < kPrefixPer; ++u) lt[u] = m[u] ? gB[(g0 + u) * HW + q] : 0;
        bool has = false;
        int64_t last = 0;
#pragma unroll
        for (int u = 0; u < kPrefixPer; ++u) {
            if (m[u]) { has = true; last = lt[u]; }
        }
        s_last[wave][lane] = last;
        s_has[wave][lane] = has ? 1 : 0;
        __syncthreads();
        int64_t run = carry;  // the value before this wave's first group
        for (int w = 0; w < wave; ++w)
            if (s_has[w][lane]) run = s_last[w][lane];
#pragma unroll
        for (int u = 0; u < kPrefixPer; ++u) {
            if (!in || g0 + u >= n_groups) break;
            gB[(g0 + u) * HW + q] = run;
            if (m[u]) run = lt[u];
        }
#pragma unroll
        for (int w = 0; w < kThreads / 64; ++w)
            if (s_has[w][lane]) carry = s_last[w][lane];
        __syncthreads();  // s_last reused by the next round
    }
    if (in && wave == 0) sae[q] = carry;
}

// The shard's own final time surface for the multi-GPU hand-off (ecc_fast_detect_prepare): per
// pixel the last timestamp of the batch, 0 where no event touched it — from the per-group images,
// no global atomics.
__global__ void __launch_bounds__(kThreads)
sae_local_last_kernel(CornerGeom g, int64_t n_groups, const uint32_t *__restrict__ gmask,
                      const int64_t *__restrict__ glast, int64_t *__restrict__ out) {
    const int64_t HW = (int64_t)g.H * g.W;
    for (int64_t q = (int64_t)blockIdx.x * kThreads + threadIdx.x; q < HW; q += (int64_t)gridDim.x * kThreads) {
        int64_t run = 0;
        for (int64_t gi = n_groups - 1; gi >= 0; --gi)
            if (gmask[gi * HW + q]) { run = glast[gi * HW + q]; break; }
        out[q] = run;
    }
}

__device__ __forceinline__ void tile_origin_xy(const CornerGeom &g, int tile, int &tx, int &ty) {
    tx = tile % g.tiles_x;
    ty = tile / g.tiles_x;
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
        m |= 1u << (k[s - 1] & ((1u << IB) - 1u));  // IB = 5: the shift's own 5-bit mask, no AND
        if (s >= SMIN) {
            // (a >> IB) > (b >> IB)  <=>  a > (b | low IB bits): one OR, one compare
            const bool sep = k[s - 1] > (k[s] | ((1u << IB) - 1u));
            const uint32_t rot = ((m << 1) | (m >> (N - 1))) & full;
            ok |= sep && (__popc(m & ~rot) == 1);
        }
    }
    return ok ? 1 : 0;
}

// Staged neighbourhood of one (group, tile) item.  T[j][wp] holds the value set at window pixel
// wp by slice j of the group — v' = t - L (narrow groups, exact) or the event index + 1 (wide
// groups) — and is valid only where bit j of mb[wp].mask is set; mb[wp].bc is the clamped B_g.
// The value an event of slice j sees at wp is T[j*][wp] with j* the highest set bit of
// mask & ((2 << j) - 1), else bc: no forward fill, and T is never cleared.
constexpr int kPairWords = kGroup * kTilePix / 32;  // 196: one bit per (slice, tile pixel)
constexpr int kSegWords = (kTilePix + 31) / 32;     // 7: one slice's 196 bits of a tile

// The corner pairs leave the arc kernels SLICE-major: res[group][j][tile][kSegWords], bit lp of
// word w = pair (j, pixel 32 w + lp), so that the flag pass of slice j stages its segment of every
// tile as one contiguous run (item-major words put one 4-B read of each tile in its own 128-B
// line, and the 32 slices of a group, on 8 XCDs, fetched every line ~8 times: ~90 MB per step).
// Lane w < 32 * 7 of an item's workgroup writes word w from the item's LDS bits `bits`
// (pair j * 196 + lp); neighbouring tiles' words are adjacent, so the writes combine in L2.
__device__ __forceinline__ void store_res_slice_major(const uint32_t *bits, int64_t grp, int tile, const CornerGeom &g,
                                                      uint32_t *__restrict__ res, int tid) {
    if (tid >= kGroup * kSegWords) return;
    const int j = tid / kSegWords, w = tid % kSegWords;
    const int b0 = j * kTilePix + 32 * w, w0 = b0 >> 5, sh = b0 & 31;
    uint32_t v = bits[w0] >> sh;
    if (sh && w0 + 1 < kPairWords) v |= bits[w0 + 1] << (32 - sh);
    if (w == kSegWords - 1) v &= (1u << (kTilePix - 32 * (kSegWords - 1))) - 1u;  // 4 bits of the last word
    res[(grp * kGroup + j) * g.seg_stride + tile * kSegWords + w] = v;
}
constexpr int kWaves = kArcThreads / 64;
constexpr int kQ4Cap = 1024;  // two 8-wave workgroups per CU fit the 160 KiB LDS

struct MaskB {
    uint32_t mask;
    uint32_t bc;
};

struct ArcLds {
    uint32_t T[kGroup][kWinPix];      // 60.5 KiB
    MaskB mb[kWinPix];
    uint32_t res[kPairWords];         // corner (slice, pixel) pairs of the tile
    uint16_t tasks[kGroup * kTilePix]; // the tile's eligible pairs (j << 9 | window pixel)
    uint16_t q4[kQ4Cap];               // circle-3 survivors (beyond the cap: tested inline)
    int64_t wave_min[16];  // per wave (up to 16 waves: arc_dense_kernel's workgroup size is a switch)
    int32_t exact_only;  // a value above t_last: clamped keys unusable
    int32_t mixed;       // clamped values not all equal to the window minimum of B
    int32_t q4n;
    int32_t n_exact;      // some task needs the exact int64 test
    int32_t wave_own[16];  // the wave's own-tile pixels have pairs
    int32_t wave_tasks[16];  // the wave's eligible pairs (task-list offsets by a scan)
};

// arc_dense_kernel's clamp: v <= L maps to 0 (mixed_flag set when v is not the window minimum vz)
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

// The clamped B_g values (at or below L) are "mixed" when not all equal: ties among their keys may
// then be artefacts of the clamp.  Per wave: its first clamped value c0 and flags cf (bit 1: it has
// one, bit 0: another differs), by ballots and readlanes (no 64-bit reductions); bq = INT64_MAX
// outside the sensor.
__device__ __forceinline__ int64_t readlane_i64(int64_t v, int l) {
    return (int64_t)((uint64_t)__builtin_amdgcn_readlane((uint32_t)((uint64_t)v >> 32), l) << 32 |
                     (uint64_t)__builtin_amdgcn_readlane((uint32_t)v, l));
}
__device__ __forceinline__ void clamp_wave_flags(int64_t bq, int64_t Lt, int64_t &c0, int &cf) {
    const bool clp = bq <= Lt;
    const uint64_t cball = __ballot(clp);
    c0 = 0;
    cf = 0;
    if (cball) {  // uniform
        c0 = readlane_i64(bq, __ffsll((unsigned long long)cball) - 1);
        cf = 2 | (__ballot(clp && bq != c0) != 0ull ? 1 : 0);
    }
}
// Wave 0 after the barrier: lane w takes wave w's (c0, cf); the window's "mixed" flag.
template <int W>
__device__ __forceinline__ bool clamp_mixed(const int64_t *wc0, const int32_t *wcf, int lane) {
    const int wf = lane < W ? wcf[lane] : 0;
    const int64_t wv = lane < W ? wc0[lane] : 0;
    const uint64_t has = __ballot(wf & 2);
    bool mixed = __ballot(wf & 1) != 0ull;
    if (has) {  // uniform
        const int64_t v0 = readlane_i64(wv, __ffsll((unsigned long long)has) - 1);
        mixed = mixed || __ballot((wf & 2) && wv != v0) != 0ull;
    }
    return mixed;
}
// clamp(B_g - L, 0, 2^27 - 1); above the range the window goes to the exact test (*exact_flag)
__device__ __forceinline__ uint32_t clamp_value(int64_t bq, int64_t Lt, bool narrow, int32_t *exact_flag) {
    if (!narrow || bq == INT64_MAX || bq <= Lt) return 0u;
    const int64_t d = bq - Lt;
    if (d > (int64_t)kVMax) {
        *exact_flag = 1;
        return kVMax;
    }
    return (uint32_t)d;
}

// slices 0 .. j (j <= 31: 2u << 31 is 0 in 32 bits, so j = 31 gives all ones without a select)
__device__ __forceinline__ uint32_t below_mask(int j) { return (2u << j) - 1u; }

// Clamped value at window pixel wp for slice j (fast path).
__device__ __forceinline__ uint32_t win_value(const ArcLds &L, int wp, uint32_t below) {
    const MaskB m = L.mb[wp];
    const uint32_t mk = m.mask & below;
    return mk ? L.T[31 - __clz(mk)][wp] : m.bc;
}

// Exact int64 arc test of one circle around window pixel wp0 (global pixel q0) for slice j:
// V = the group value (v' + L, or the timestamp of the stored event index) where a slice <= j of
// the group touched the pixel, else B_g.  Rare fallback; out of line so its registers do not
// raise the pressure of the main kernel body.
struct ExactCtx {
    const int64_t *Bg;  // B_g image of the group
    const int64_t *t;
    int64_t grp_first, Lt;
    int W;
    bool narrow;
};

template <int N>
__device__ __forceinline__ void exact_values(const ArcLds *L, int wp0, int64_t q0, uint32_t below,
                                             const int8_t *dy, const int8_t *dx, const ExactCtx &c, int64_t (&v)[N]) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
        // four neighbours' loads in flight at a time: all of them at once spilled (rare path)
        if (k > 0 && k % 4 == 0) __builtin_amdgcn_sched_barrier(0);
        const int wp = wp0 + dy[k] * kWin + dx[k];
        const uint32_t mk = L->mb[wp].mask & below;
        const uint32_t tv = mk ? L->T[31 - __clz(mk)][wp] : 0u;
        v[k] = !mk      ? c.Bg[q0 + (int64_t)dy[k] * c.W + dx[k]]
               : c.narrow ? c.Lt + (int64_t)tv
                          : c.t[c.grp_first + tv - 1u];
    }
}


// Both circles exactly (circle 3 skipped when it already passed on keys).  Out of line, called
// only from arc_dense_item's exact phase, where nothing else is live.
__device__ __noinline__ bool exact_pair_test(const ArcLds *L, int wp0, int64_t q0, uint32_t below, bool c3_passed,
                                             const int64_t *Bg, const int64_t *t, int64_t grp_first, int64_t Lt, int W,
                                             bool narrow) {
    const ExactCtx c{Bg, t, grp_first, Lt, W, narrow};  // scalars in registers, not a by-value struct on the stack
    if (!c3_passed) {
        int64_t v3[16];
        exact_values<16>(L, wp0, q0, below, c3dy, c3dx, c, v3);
        if (!arc_streak<16, 3, 6>(v3)) return false;
    }
    int64_t v4[20];
    exact_values<20>(L, wp0, q0, below, c4dy, c4dx, c, v4);
    return arc_streak<20, 4, 8>(v4);
}

// 5. Arc test of one (group, tile) item, all items of all groups in one launch.  The item's
// corner pairs go to res (slice-major, store_res_slice_major); flags_event_kernel applies them.
//
// Staging: window pixel wp of the item (lane wp < 484) reads its slice mask, its value record and
// its B_g from fixed per-pixel addresses (pair_build's gmask / pv images, sae_prefix's B), three
// independent loads in flight together; only a pixel with more than four values reads the rest
// of them from the overflow array, at the address its record names.

// The slices of group grp whose pairs are tested (Q15: slices before first_detect are not).
__device__ __forceinline__ uint32_t eligible_slices(const CornerGeom &g, int64_t grp) {
    const int64_t j0 = (int64_t)g.first_detect - grp * kGroup;
    return j0 <= 0 ? 0xffffffffu : (j0 >= kGroup ? 0u : (0xffffffffu << (int)j0));
}

// The values v3 .. v_{p-1} (p > 4) of a pixel whose record is r, from the overflow array:
// the run starts 16-B aligned at line r.w, so line l holds
// v_{3 + 4l} .. v_{6 + 4l}.  Lines l0 .. of the run, four lines (16 values) in flight per trip
// (clamped to the last line, no load under a lane condition): a pixel with 32 values costs two
// dependent round trips instead of seven 4-value ones.
template <class Put>
__device__ __forceinline__ void overflow_lines(const uint32_t *__restrict__ ovf, const uint4 &r, int l0, int p, Put put) {
    const uint4 *__restrict__ x4 = reinterpret_cast<const uint4 *>(ovf) + r.w;
    const int nl = (p - (kRecVals - 1) + 3) >> 2;
    for (; l0 < nl; l0 += 4) {
        uint4 a[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] = x4[min(l0 + u, nl - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = (kRecVals - 1) + 4 * (l0 + u);
            if (k < p) put(k, a[u].x);
            if (k + 1 < p) put(k + 1, a[u].y);
            if (k + 2 < p) put(k + 2, a[u].z);
            if (k + 3 < p) put(k + 3, a[u].w);
        }
    }
}

#ifndef ECC_ARC_PROFILE
#define ECC_ARC_PROFILE 0
#endif
#if ECC_ARC_PROFILE
// profiling builds: arc_dense_kernel's per-item phases summed (thread 0), [5] = the longest item,
// [6] = tasks, [7] = items
__device__ unsigned long long g_dense_prof[8];
#define DENSE_MARK(k)                                                                \
    do {                                                                             \
        if (tid == 0) {                                                              \
            const unsigned long long now_ = wall_clock64();                          \
            atomicAdd(&g_dense_prof[k], now_ - dense_t_);                            \
            dense_t_ = now_;                                                         \
        }                                                                            \
    } while (0)
#else
#define DENSE_MARK(k) do { } while (0)
#endif

template <int NT>
__device__ __forceinline__ void arc_dense_item(ArcLds &L, int64_t item, const int64_t *__restrict__ t, const CornerGeom &g,
                                               const uint32_t *__restrict__ ovf, const uint4 *__restrict__ pv,
                                               const int64_t *__restrict__ gB, const uint32_t *__restrict__ gmask,
                                               uint32_t *__restrict__ res) {
    const int64_t grp = (int)item / g.n_tiles;  // n_items < 2^31 (host check): 32-bit division
    const int tile = (int)item % g.n_tiles;
    if ((grp + 1) * kGroup <= g.first_detect) return;  // every slice of the group precedes detection
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#if ECC_ARC_PROFILE
    const unsigned long long dense_t0_ = wall_clock64();
    unsigned long long dense_t_ = dense_t0_;
#endif
    const int64_t HW = (int64_t)g.H * g.W;
    int tx, ty;
    tile_origin_xy(g, tile, tx, ty);
    const int x0 = tx * kTile, y0 = ty * kTile;
    const GroupRef gr = group_ref(t, g, grp);
    const int64_t grp_first = gr.first, Lt = gr.Lt;
    const bool narrow = gr.narrow;
    const int64_t *Bg = gB + grp * HW;

    // (a) window pixel wp (lane wp < 484): its B_g, slice mask and value record, three loads in
    //     flight together; its values go to the dense planes T[j][wp], the own tile's eligible
    //     pairs (slice and pixel; the per-event cut of border mode 1 is applied when flagging)
    //     are the test tasks
    static_assert(NT >= kWinPix, "one lane per window pixel");
    const int wp = tid;
    const bool win_lane = wp < kWinPix;
    const int ox = wp % kWin - kHalo, oy = wp / kWin - kHalo;  // pixel relative to the tile origin
    const int wx = x0 + ox, wy = y0 + oy;
    const bool in = win_lane && wx >= 0 && wy >= 0 && wx < g.W && wy < g.H;
    const int64_t q = grp * HW + (int64_t)wy * g.W + wx;
    int64_t bq = INT64_MAX;  // INT64_MAX: outside (never read)
    uint32_t mk = 0u;
    uint4 rec = make_uint4(0u, 0u, 0u, 0u);
    if (in) {
        bq = gB[q];
        mk = gmask[q];
        rec = pv[q];
    }
    for (int w = tid; w < kPairWords; w += NT) L.res[w] = 0u;
    if (tid == 0) {
        L.exact_only = narrow ? 0 : 1;  // wide groups: every test exact
        L.mixed = 0;
        L.q4n = 0;
        L.n_exact = 0;
    }
    const bool own = win_lane && ox >= 0 && oy >= 0 && ox < kTile && oy < kTile;
    const uint64_t own_pairs = __ballot(own && mk != 0u);
    if (lane == 0) L.wave_own[wave] = own_pairs != 0ull;
    // the own tile's eligible pairs, placed by a scan (one returning LDS atomic per pair on one
    // counter serialised a heavy item's ~3 000 tasks)
    const uint32_t tm0 = (own && !is_border(wx, wy, g)) ? (mk & eligible_slices(g, grp)) : 0u;
    const int tcnt = __popc(tm0);
    const int tincl = ecc::wave_incl_scan(tcnt);  // DPP
    if (lane == 63) L.wave_tasks[wave] = tincl;
    __syncthreads();
    if (win_lane) {
        L.mb[wp].mask = mk;
        const int p = __popc(mk);
        uint32_t mm = mk;
        for (int k = 0; mm && k < kRecVals - 1; ++k, mm &= mm - 1u)
            L.T[__ffs(mm) - 1][wp] = k == 0 ? rec.x : (k == 1 ? rec.y : rec.z);
        if (mm && p == kRecVals) {
            L.T[__ffs(mm) - 1][wp] = rec.w;
        } else if (mm) {  // v3.. from the overflow array, ascending j as the bits
            overflow_lines(ovf, rec, 0, p, [&](int, uint32_t v) {
                L.T[__ffs(mm) - 1][wp] = v;
                mm &= mm - 1u;
            });
        }
    }
    int toff = tincl - tcnt, n_tasks = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        const int c = L.wave_tasks[w];
        toff += w < wave ? c : 0;
        n_tasks += c;
    }
    for (uint32_t tm = tm0; tm; tm &= tm - 1u) L.tasks[toff++] = (uint16_t)((__ffs(tm) - 1) << 9 | wp);  // j << 9 | window pixel
    const int64_t bmin = ecc::wave_min_i64(bq);  // DPP
    if (lane == 0) L.wave_min[wave] = bmin;
    __syncthreads();
    DENSE_MARK(0);  // (a) staging
    {
        int any = 0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) any |= L.wave_own[w];
        if (!any) return;  // uniform: no events in the tile, nothing to flag
    }
    DENSE_MARK(1);

    // (c) clamped B_g per window pixel
    if (win_lane) {
        int64_t vz = INT64_MAX;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) vz = L.wave_min[w] < vz ? L.wave_min[w] : vz;
        L.mb[wp].bc = (!narrow || bq == INT64_MAX) ? 0u : clamp_rel(bq, Lt, vz, &L.exact_only, &L.mixed);
    }
    __syncthreads();
    DENSE_MARK(2);  // (c)

    // (d) each eligible pair of the tile is tested once, in three phases so that no phase holds
    //     another's registers (and no call): circle 3 on clamped keys, its survivors queued so
    //     that circle 4 runs on as few waves as possible; circle 4 on clamped keys; then the
    //     exact int64 tests of whatever the keys could not decide, marked in the task list
    //     itself (bit 14: circle 3 undecided; bit 15: circle 3 passed, circle 4 still open).
    //     Wide groups and values above t_last (exact_only) take every task exactly.
    const bool fast = !L.exact_only;
    const bool ties_exact = !L.mixed;
    constexpr uint16_t kOpen3 = 0x4000, kOpen4 = 0x8000;
    if (fast) {
        for (int ti = tid; ti < n_tasks; ti += NT) {
            const int pi = L.tasks[ti];  // j << 9 | window pixel
            const int wp0 = pi & 511;
            const uint32_t below = below_mask(pi >> 9);
            uint32_t k3[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) k3[k] = (win_value(L, wp0 + c3dy[k] * kWin + c3dx[k], below) << 5) | k;
            const int r3 = arc_keys<16, 16, 5, 3, 6>(k3, ties_exact);
            if (r3 > 0) {
                const int qi = atomicAdd(&L.q4n, 1);
                if (qi < kQ4Cap) L.q4[qi] = (uint16_t)ti;
                else { L.tasks[ti] = (uint16_t)(pi | kOpen4); L.n_exact = 1; }  // queue full (rare)
            } else if (r3 < 0) {
                L.tasks[ti] = (uint16_t)(pi | kOpen3);
                L.n_exact = 1;
            }
        }
    }
    __syncthreads();
    DENSE_MARK(3);  // circle 3
    const int n4 = min(L.q4n, kQ4Cap);
    for (int qi = tid; qi < n4; qi += NT) {
        const int ti = L.q4[qi];
        const int pi = L.tasks[ti];
        const int j = pi >> 9, wp0 = pi & 511;
        const uint32_t below = below_mask(j);
        uint32_t k4[32];
#pragma unroll
        for (int k = 0; k < 20; ++k) k4[k] = (win_value(L, wp0 + c4dy[k] * kWin + c4dx[k], below) << 5) | k;
#pragma unroll
        for (int k = 20; k < 32; ++k) k4[k] = 0u;
        const int r4 = arc_keys<20, 32, 5, 4, 8>(k4, ties_exact);
        if (r4 > 0) {  // the pair's bit: slice j, tile pixel (wp0's row and column less the halo)
            const int rb = j * kTilePix + (wp0 / kWin - kHalo) * kTile + (wp0 % kWin - kHalo);
            atomicOr(&L.res[rb >> 5], 1u << (rb & 31));
        } else if (r4 < 0) {
            L.tasks[ti] = (uint16_t)(pi | kOpen4);
            L.n_exact = 1;
        }
    }
    __syncthreads();
    DENSE_MARK(4);  // circle 4
    if (!fast || L.n_exact) {  // uniform; rare: the exact int64 tests
        for (int ti = tid; ti < n_tasks; ti += NT) {
            const int e = L.tasks[ti], pi = e & 0x3fff;
            if (fast && !(e & (kOpen3 | kOpen4))) continue;
            const int j = pi >> 9, wp0 = pi & 511;
            const int ly = wp0 / kWin - kHalo, lx = wp0 % kWin - kHalo;
            const int64_t q0 = (int64_t)(y0 + ly) * g.W + (x0 + lx);
            const uint32_t below = below_mask(j);
            if (exact_pair_test(&L, wp0, q0, below, (e & kOpen4) != 0, Bg, t, grp_first, Lt, g.W, narrow)) {
                const int rb = j * kTilePix + ly * kTile + lx;
                atomicOr(&L.res[rb >> 5], 1u << (rb & 31));
            }
        }
        __syncthreads();
    }
#if ECC_ARC_PROFILE
    if (tid == 0) {
        atomicMax(&g_dense_prof[5], wall_clock64() - dense_t0_);
        atomicAdd(&g_dense_prof[6], (unsigned long long)n_tasks);
        atomicAdd(&g_dense_prof[7], 1ull);
    }
#endif
    store_res_slice_major(L.res, grp, tile, g, res, tid);
}

// ---- compact window values (the common case) -------------------------------------------------
// Window pixel wp keeps its clamped B_g followed by the values of the slices that touched it,
// ascending j, at vals[pix[wp].off ...]; the value an event of slice j sees is
// vals[off + popc(mask & ((2 << j) - 1))] — index off (the B_g slot) when no slice <= j touched
// the pixel, so a lookup is one 8-B pixel read and one value read, no select.  ~34 KB of LDS
// instead of the dense planes' ~80 KB: four 8-wave workgroups per CU.  Windows with more than
// kValCap values go to the overflow list (arc_dense_kernel).
#ifndef ECC_ARC_VALCAP
#define ECC_ARC_VALCAP 4096
#endif
constexpr int kValCap = ECC_ARC_VALCAP;

struct PixInfo {
    uint32_t mask;  // slices of the group that touched the pixel
    uint32_t off;   // its B_g slot in vals[], the slice values follow
};

struct SparseLds {
    uint32_t vals[kValCap + kWinPix];   // 17.9 KiB: the pairs + one B_g slot per window pixel
    PixInfo pix[kWinPix];               // 3.8 KiB
    uint32_t res[kPairWords];
    uint16_t tasks[kValCap];  // the tile's eligible pairs (j << 9 | window pixel): at most the window's pairs
    uint16_t q4[kQ4Cap];
    int64_t wave_c0[kWaves];    // the wave's first B_g at or below L (clamped to 0) ...
    int32_t wave_cf[kWaves];    // ... bit 1: it has one, bit 0: another differs from it
    int32_t wave_tot[kWaves];
    int32_t wave_own[kWaves];  // the wave's own-tile pixels have pairs
    int32_t exact_only, mixed, q4n, redo;
};

// Branch-free by layout: one 8-B pixel read and one value read (a conditional read compiles to
// an exec-mask branch per circle pixel: scalar-unit bookkeeping, serialised LDS round trips).
static_assert(sizeof(PixInfo) == 8, "one 8-B LDS read per pixel");
__device__ __forceinline__ uint32_t sparse_value(const SparseLds &L, int wp, uint32_t below) {
    const uint2 p = reinterpret_cast<const uint2 *>(L.pix)[wp];  // {mask, off}
    return L.vals[p.y + __popc(p.x & below)];
}

#ifndef ECC_ARC_SKIP_OVF
#define ECC_ARC_SKIP_OVF 0  // timing experiments only (wrong results): 1 = no overflow loads past the first line
#endif
#ifndef ECC_ARC_WAVES
#define ECC_ARC_WAVES 8
#endif

#if ECC_ARC_PROFILE
// profiling builds: per-workgroup wall-clock of arc_kernel's phases, summed (thread 0); [7] = items
// per item (no global atomics on shared words: 18 K workgroups adding to 8 words serialised at
// the memory side and distorted the very phases they timed); summed on the host
constexpr int kProfItems = 1 << 15;
__device__ unsigned long long g_arc_items[kProfItems][8];
#define ARC_MARK(k)                                                                  \
    do {                                                                             \
        if (tid == 0) {                                                              \
            const unsigned long long now_ = wall_clock64();                          \
            arc_ph_[k] = now_ - arc_t_;                                              \
            arc_t_ = now_;                                                           \
        }                                                                            \
    } while (0)
#else
#define ARC_MARK(k) do { } while (0)
#endif

// One item's phase-A loads: window pixel `tid`'s B_g, slice mask and value record, from fixed
// per-pixel addresses (no offset table in between), so the three are in flight together.
struct ArcPre {
    int64_t bq;   // B_g (INT64_MAX outside the sensor / past the window)
    uint32_t mk;  // slices of the group that touched the pixel
    uint4 rec;    // its values (pair_build's record)
};

__device__ __forceinline__ void arc_prefetch(ArcPre &p, int64_t item, const CornerGeom &g, const uint4 *__restrict__ pv,
                                             const int64_t *__restrict__ gB, const uint32_t *__restrict__ gmask) {
    const int tid = threadIdx.x;
    p.bq = INT64_MAX;
    p.mk = 0u;
    p.rec = make_uint4(0u, 0u, 0u, 0u);
    const int64_t HW = (int64_t)g.H * g.W;
    const int64_t grp = (int)item / g.n_tiles;  // n_items < 2^31 (host check): 32-bit division
    const int tile = (int)item % g.n_tiles;
    const int tx = tile % g.tiles_x, ty = tile / g.tiles_x;
    const int wx = tx * kTile - kHalo + tid % kWin, wy = ty * kTile - kHalo + tid / kWin;
    if (tid < kWinPix && wx >= 0 && wy >= 0 && wx < g.W && wy < g.H) {
        const int64_t q = grp * HW + (int64_t)wy * g.W + wx;
        p.bq = gB[q];
        p.mk = gmask[q];
        p.rec = pv[q];
    }
}

// The arc tests of one (group, tile) item from its phase-A loads `pre`.
//   A: wave scans of the value counts and task counts, wave minimum of B_g    -> barrier 1
//   B: pixel records, clamped B_g slots, values (overflow loads), tasks       -> barrier 2
//   circle 3 -> barrier 3 -> circle 4 -> barrier 4
// Every lane knows its own pixel's values, so the list offsets, the task offsets and the window
// minimum of B_g are all wave scans before the first barrier, and each lane writes its pixel's
// list and tasks itself (no scatter, no LDS atomics).
__device__ __forceinline__ void arc_item(SparseLds &L, int64_t item, const ArcPre &pre,
                                         const int64_t *__restrict__ t, const CornerGeom &g,
                                         const uint32_t *__restrict__ ovf, uint32_t *__restrict__ res,
                                         int64_t *__restrict__ over, uint32_t *__restrict__ n_over) {
    const int64_t grp = (int)item / g.n_tiles;  // n_items < 2^31 (host check): 32-bit division
    const int tile = (int)item % g.n_tiles;
    if ((grp + 1) * kGroup <= g.first_detect) return;  // every slice of the group precedes detection
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#if ECC_ARC_PROFILE
    unsigned long long arc_t_ = wall_clock64(), arc_ph_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    int tx, ty;
    tile_origin_xy(g, tile, tx, ty);
    const int x0 = tx * kTile, y0 = ty * kTile;
    const GroupRef gr = group_ref(t, g, grp);
    const int64_t Lt = gr.Lt;
    const bool narrow = gr.narrow;
    const int wp = tid;
    const bool win_lane = wp < kWinPix;
    const int64_t bq = pre.bq;
    const uint32_t mk_w = pre.mk;
    const int ox = wp % kWin - kHalo, oy = wp / kWin - kHalo;  // pixel relative to the tile origin
    const bool own = win_lane && ox >= 0 && oy >= 0 && ox < kTile && oy < kTile;
    for (int w = tid; w < kPairWords; w += kArcThreads) L.res[w] = 0u;
    if (tid == 0) {
        L.exact_only = narrow ? 0 : 1;  // wide groups: every test exact
        L.q4n = 0;
        L.redo = 0;
    }
    // the own tile's eligible pairs of this pixel (Q15 slices; border pixels are never corners)
    const uint32_t tm = (own && !is_border(x0 + ox, y0 + oy, g)) ? (mk_w & eligible_slices(g, grp)) : 0u;
    const int cnt = win_lane ? __popc(mk_w) + 1 : 0;  // the pixel's values + its B_g slot
    const int tcnt = __popc(tm);
    // wave scans and the wave minimum of B_g by DPP moves
    // one scan of both counts, packed (task count << 16 | value count: a workgroup's sums stay
    // below 2^16, at most 484 * 33 values and 196 * 32 tasks)
    const int both = ecc::wave_incl_scan(tcnt << 16 | cnt);
    const int incl = both & 0xffff, tincl = both >> 16;
    const uint64_t own_pairs = __ballot(own && mk_w != 0u);
    int64_t c0;
    int cf;
    clamp_wave_flags(bq, Lt, c0, cf);  // the window's "mixed" clamp, per wave
    // a pixel with more than 4 values: v3 .. v6 as one 16-B load, issued now (its address is in
    // the record) so that it flies during the scans and the barrier; the other lanes of the wave
    // load the first line of ovf (no per-lane branch around the load)
    const int p = cnt - 1;
#ifndef ECC_ARC_XPF
#define ECC_ARC_XPF 1  // 16-B overflow lines loaded before barrier 1 (0: none, after it)
#endif
    constexpr int kXpf = ECC_ARC_XPF > 0 ? ECC_ARC_XPF : 1;
    uint4 xs[kXpf];
#pragma unroll
    for (int u = 0; u < kXpf; ++u) xs[u] = make_uint4(0u, 0u, 0u, 0u);
    if (ECC_ARC_XPF && __ballot(p > kRecVals)) {  // uniform
        const bool o = p > kRecVals;
        const uint4 *x4 = reinterpret_cast<const uint4 *>(ovf) + (o ? pre.rec.w : 0u);
        const int nl = o ? (p - (kRecVals - 1) + 3) >> 2 : 1;  // lines of the lane's run
#pragma unroll
        for (int u = 0; u < kXpf; ++u) xs[u] = x4[min(u, nl - 1)];  // no load past the run
    }
    if (lane == 63) L.wave_tot[wave] = both;
    if (lane == 0) {
        L.wave_c0[wave] = c0;
        L.wave_cf[wave] = cf;
        L.wave_own[wave] = own_pairs != 0ull;
    }
    __syncthreads();  // 1
    ARC_MARK(0);  // A
    int total = 0, n_tasks = 0, any_own = 0, off = incl - cnt, toff = tincl - tcnt;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {  // uniform reads, in flight together
        const int wb = L.wave_tot[w], wt = wb & 0xffff, tt = wb >> 16;
        total += wt;
        n_tasks += tt;
        off += w < wave ? wt : 0;
        toff += w < wave ? tt : 0;
        any_own |= L.wave_own[w];
    }
    if (wave == 0) {  // L.mixed is read after barrier 2
        const bool mixed = clamp_mixed<kWaves>(L.wave_c0, L.wave_cf, lane);
        if (lane == 0) L.mixed = mixed;
    }
    if (!any_own || total > kValCap + kWinPix) {  // uniform
        // no events in the tile: nothing to flag; too many values for the compact list: the
        // dense kernel takes it
        if (any_own && tid == 0) over[atomicAdd(n_over, 1u)] = item;
        return;
    }
    if (win_lane) {
        const uint32_t bcv = clamp_value(bq, Lt, narrow, &L.exact_only);  // above the range: the exact kernel
        reinterpret_cast<uint2 *>(L.pix)[wp] = make_uint2(mk_w, (uint32_t)off);
        uint32_t *dst = L.vals + off;
        dst[0] = bcv;
        if (p > 0) dst[1] = pre.rec.x;
        if (p > 1) dst[2] = pre.rec.y;
        if (p > 2) dst[3] = pre.rec.z;
        if (p == kRecVals) {
            dst[4] = pre.rec.w;
        } else if (!ECC_ARC_XPF && p > kRecVals) {
            overflow_lines(ovf, pre.rec, 0, p, [&](int k, uint32_t v) { dst[1 + k] = v; });
        } else if (p > kRecVals) {  // v3 .. v6 from the prefetched line, the rest loaded now
            // v_k goes to dst[1 + k] for k < p (here p >= 5); line u holds v_{3+4u} .. v_{6+4u}
#pragma unroll
            for (int u = 0; u < kXpf; ++u) {
                const int k = (kRecVals - 1) + 4 * u;
                if (k < p) dst[1 + k] = xs[u].x;
                if (k + 1 < p) dst[2 + k] = xs[u].y;
                if (k + 2 < p) dst[3 + k] = xs[u].z;
                if (k + 3 < p) dst[4 + k] = xs[u].w;
            }
            if (!ECC_ARC_SKIP_OVF && p > kRecVals + 4 * ECC_ARC_XPF - 1)
                overflow_lines(ovf, pre.rec, ECC_ARC_XPF, p, [&](int k, uint32_t v) { dst[1 + k] = v; });
        }
        // a task is (slice j, window pixel) as j << 9 | wp: the tests decode it with a shift and
        // a mask (no division by the tile and window widths)
        for (uint32_t m = tm; m; m &= m - 1u) L.tasks[toff++] = (uint16_t)((__ffs(m) - 1) << 9 | wp);
    }
    __syncthreads();  // 2
    ARC_MARK(1);  // B
    if (L.exact_only) {  // uniform: a wide group or a value above t_last — the exact kernel takes it
        if (tid == 0) over[atomicAdd(n_over, 1u)] = item;
        return;
    }
    // Tests through the compact lists, on clamped 32-bit keys only.  No exact int64 path and no
    // call: an item its keys cannot decide (a wide group, a value above t_last, a tie the clamping
    // may have merged) or whose circle-3 survivors overflow the queue goes whole to
    // arc_dense_kernel, which redoes it exactly.  So the kernel fits 64 VGPRs without spills.
#ifndef ECC_ARC_SKIP
#define ECC_ARC_SKIP 0  // timing experiments only (wrong results): 1 = no circle 4, 2 = no tests
#endif
    if (ECC_ARC_SKIP >= 2) n_tasks = 0;
    const bool ties_exact = !L.mixed;
    for (int ti = tid; ti < n_tasks; ti += kArcThreads) {
        const int pi = L.tasks[ti];  // j << 9 | window pixel
        const int wp0 = pi & 511;
        const uint32_t below = below_mask(pi >> 9);
        uint32_t k3[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) k3[k] = (sparse_value(L, wp0 + c3dy[k] * kWin + c3dx[k], below) << 5) | k;
        const int r3 = arc_keys<16, 16, 5, 3, 6>(k3, ties_exact);
        if (r3 > 0) {
            const int qi = atomicAdd(&L.q4n, 1);
            if (qi < kQ4Cap) L.q4[qi] = (uint16_t)pi;
            else L.redo = 1;
        } else if (r3 < 0) {
            L.redo = 1;
        }
    }
    __syncthreads();  // 3
    ARC_MARK(3);  // circle 3
    if (L.redo) {  // uniform
        if (tid == 0) over[atomicAdd(n_over, 1u)] = item;
        return;
    }
    const int n4 = ECC_ARC_SKIP >= 1 ? 0 : L.q4n;
#if ECC_ARC_PROFILE
    if (tid == 0) {
        arc_ph_[5] = (unsigned long long)n_tasks;
        arc_ph_[6] = (unsigned long long)n4;
    }
#endif
    for (int qi = tid; qi < n4; qi += kArcThreads) {
        const int pt = L.q4[qi];  // j << 9 | window pixel
        const int j = pt >> 9, wp0 = pt & 511;
        const uint32_t below = below_mask(j);
        uint32_t k4[32];
#pragma unroll
        for (int k = 0; k < 20; ++k) k4[k] = (sparse_value(L, wp0 + c4dy[k] * kWin + c4dx[k], below) << 5) | k;
#pragma unroll
        for (int k = 20; k < 32; ++k) k4[k] = 0u;
        const int r4 = arc_keys<20, 32, 5, 4, 8>(k4, ties_exact);
        if (r4 > 0) {  // the pair's bit: slice j, tile pixel (wp0's row and column less the halo)
            const int pi = j * kTilePix + (wp0 / kWin - kHalo) * kTile + (wp0 % kWin - kHalo);
            atomicOr(&L.res[pi >> 5], 1u << (pi & 31));
        } else if (r4 < 0) {
            L.redo = 1;
        }
    }
    __syncthreads();  // 4
    ARC_MARK(4);  // circle 4
#if ECC_ARC_PROFILE
    if (tid == 0 && item < kProfItems) {
        arc_ph_[7] = 1ull;
        for (int k = 0; k < 8; ++k) g_arc_items[item][k] = arc_ph_[k];
    }
#endif
    if (L.redo) {  // uniform: a circle-4 tie the clamped keys cannot decide
        if (tid == 0) over[atomicAdd(n_over, 1u)] = item;
        return;
    }
    store_res_slice_major(L.res, grp, tile, g, res, tid);
}

// One workgroup per item, all items of all groups in one launch, in XCD-aware order: workgroup b
// runs on XCD b % 8, so XCD x takes the contiguous item range [x * per, (x + 1) * per) —
// neighbouring tiles of one group share that XCD's L2.
__global__ void __launch_bounds__(kArcThreads, ECC_ARC_WAVES)  // waves/SIMD: 8 = four 8-wave workgroups per CU
arc_kernel(const int64_t *__restrict__ t, CornerGeom g, int64_t n_items, const uint32_t *__restrict__ ovf,
           const uint4 *__restrict__ pv, const int64_t *__restrict__ gB, const uint32_t *__restrict__ gmask,
           uint32_t *__restrict__ res, int64_t *__restrict__ over, uint32_t *__restrict__ n_over) {
    __shared__ SparseLds L;
    const int per = (int)(gridDim.x / 8);
    const int64_t item = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
    if (item >= n_items) return;
    ArcPre pre;
    arc_prefetch(pre, item, g, pv, gB, gmask);
    arc_item(L, item, pre, t, g, ovf, res, over, n_over);
}


// The windows above the compact list's capacity (arc_kernel's overflow list), each with the
// dense per-slice planes.
#ifndef ECC_DENSE_THREADS
#define ECC_DENSE_THREADS 512  // arc_dense_kernel's workgroup: 512 = two per CU, 1024 = one per CU
#endif
constexpr int kDenseThreads = ECC_DENSE_THREADS;
__global__ void __launch_bounds__(kDenseThreads, 4)  // 4 waves/SIMD (128 VGPRs)
arc_dense_kernel(const int64_t *__restrict__ t, CornerGeom g, const int64_t *__restrict__ over,
                 const uint32_t *__restrict__ n_over, const uint32_t *__restrict__ ovf, const uint4 *__restrict__ pv,
                 const int64_t *__restrict__ gB, const uint32_t *__restrict__ gmask, uint32_t *__restrict__ res) {
    __shared__ ArcLds L;
    const uint32_t n = *n_over;
    for (uint32_t li = blockIdx.x; li < n; li += gridDim.x) {
        arc_dense_item<kDenseThreads>(L, over[li], t, g, ovf, pv, gB, gmask, res);
        __syncthreads();
    }
}

// 6. Corner flags in event order: one workgroup per slice.  Event i of slice s (group g, slice j
// of the group) is a corner iff its (slice, pixel) pair's bit is set in the result words of its
// (g, tile) item.  The workgroup first stages slice j's 196-bit segment of every tile's result
// vector in LDS (7 words per tile), so each event's lookup is an LDS read; every flag is then
// written, 0 or 1, four per lane and store.  The per-event eligibility of the reference loop: the
// first-detect rule (Q15) and, in ref_compat mode (Q11), "before the slice's first border event";
// corner pairs are never border pixels.
#ifndef ECC_FLAG_THREADS
#define ECC_FLAG_THREADS 256
#endif
constexpr int kFlagThreads = ECC_FLAG_THREADS;  // 256: every slice's workgroup resident at once (8 per CU)
#ifndef ECC_FLAG_QUADS
#define ECC_FLAG_QUADS 8
#endif
constexpr int kFlagQuads = ECC_FLAG_QUADS;  // 4-event quads a lane has in flight per batch
constexpr int kFlagBatch = kFlagQuads * kFlagThreads;  // quads per batch
constexpr int kFlagCandMax = 16384;  // slices up to this many events take the candidate-list form

// kStaged: bit lp of tile in the LDS segments; otherwise (sensors whose segments exceed the
// LDS) straight from the group's result words.
template <bool kStaged>
__device__ __forceinline__ uint32_t corner_bit(uint32_t v, const CornerGeom &g, const uint32_t *sb,
                                               const uint32_t *__restrict__ rg, int j) {
    const int x = ecc::xy_x(v), y = ecc::xy_y(v);
    if (x >= g.W || y >= g.H) return 0u;
    const int tile = (y / kTile) * g.tiles_x + x / kTile;
    const int lp = (y % kTile) * kTile + x % kTile;
    if (kStaged) return (sb[tile * kSegWords + (lp >> 5)] >> (lp & 31)) & 1u;
    return (rg[(int64_t)tile * kSegWords + (lp >> 5)] >> (lp & 31)) & 1u;
}

// kCand (ecc_fast_detect_nms): the pass also writes each slice's NMS candidate list — the
// flagged events' xy in event order at cand[s * S ...], their count in n_cand[s] — which is
// what nms_compact_kernel would rebuild from the flags (the host takes this form only for
// slices of at most kFlagCandMax events, a multiple of 4).
// 256-lane workgroups, one per slice, so that all 1221 slices of the bench batch are resident at
// once (eight per CU; 512-lane ones left a second round of 197 workgroups as a tail).  A slice's
// quads are taken in batches of kFlagQuads per lane: the first batch's loads are issued before
// the staging of the result segments, so the two latencies overlap.
template <bool kStaged, bool kCand>
__global__ void __launch_bounds__(kFlagThreads)
flags_event_kernel(const uint32_t *__restrict__ xy, CornerGeom g, const uint32_t *__restrict__ res,
                   const int32_t *__restrict__ first_border, uint8_t *__restrict__ flags, uint32_t *__restrict__ cand,
                   int32_t *__restrict__ n_cand) {
    extern __shared__ uint32_t sb[];  // [n_tiles][kSegWords]: bit lp of tile = pair (j, lp)
    __shared__ int ctot[kFlagQuads][kFlagThreads / 64];
    const int64_t s = blockIdx.x;
    const int64_t lo = s * g.S;
    const int len = (int)((lo + g.S < g.n ? lo + g.S : g.n) - lo);
    const int j = (int)(s % kGroup);
    // events [0, live_end) of the slice can be corners
    const int live_end = s < g.first_detect ? 0 : (g.border_mode == 1 ? min(len, max(first_border[s], 0)) : len);
    const uint32_t *rg = res + s * g.seg_stride;  // slice s's segment of every tile (16-B aligned)
    const bool vec = (lo & 3) == 0;  // 4-event quads: 16-B loads, 4-B flag stores
    const int n4 = vec ? len / 4 : 0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // all loads unconditional through a buffer view of the slice's whole quads (0 past them): a
    // load under a per-lane condition made each quad wait for the previous one
    const __amdgpu_buffer_rsrc_t vq = ecc::buffer_view(xy + lo, (uint32_t)n4 * 16u);
    uint4 pre[kFlagQuads];
    auto load_batch = [&](int q0) {
#pragma unroll
        for (int u = 0; u < kFlagQuads; ++u)
            pre[u] = ecc::buffer_load_u128(vq, threadIdx.x * 16u, (uint32_t)(q0 + u * kFlagThreads) * 16u);
        __builtin_amdgcn_sched_barrier(0);
    };
    load_batch(0);
    if (kStaged && live_end > 0) {
        // the slice's words of every tile are one contiguous run: 16-B loads, four per lane per
        // trip, unconditional through a buffer view (0 past the run)
        const int total = g.n_tiles * kSegWords;
        const __amdgpu_buffer_rsrc_t vr = ecc::buffer_view(rg, (uint32_t)total * 4u);
        for (int k0 = 0; k0 < total; k0 += 16 * kFlagThreads) {
            uint4 a[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) a[b] = ecc::buffer_load_u128(vr, (uint32_t)(k0 + 4 * (b * kFlagThreads + (int)threadIdx.x)) * 4u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int k = k0 + 4 * (b * kFlagThreads + (int)threadIdx.x);
                if (k + 3 < total) {
                    *reinterpret_cast<uint4 *>(sb + k) = a[b];
                } else {
                    if (k < total) sb[k] = a[b].x;
                    if (k + 1 < total) sb[k + 1] = a[b].y;
                    if (k + 2 < total) sb[k + 2] = a[b].z;
                }
            }
        }
    }
    __syncthreads();
    auto quad_flags = [&](int i, const uint4 v) {
        return corner_bit<kStaged>(v.x, g, sb, rg, j) | (i + 1 < live_end ? corner_bit<kStaged>(v.y, g, sb, rg, j) << 8 : 0u) |
               (i + 2 < live_end ? corner_bit<kStaged>(v.z, g, sb, rg, j) << 16 : 0u) |
               (i + 3 < live_end ? corner_bit<kStaged>(v.w, g, sb, rg, j) << 24 : 0u);
    };
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    int base = 0;  // candidates written so far (uniform)
    uint32_t *dst = cand + lo;
    for (int q0 = 0; q0 < n4; q0 += kFlagBatch) {  // uniform
        if (q0 > 0) load_batch(q0);
        uint32_t f[kFlagQuads];
        int pfx[kFlagQuads];
#pragma unroll
        for (int u = 0; u < kFlagQuads; ++u) {
            const int q = q0 + u * kFlagThreads + (int)threadIdx.x;
            const int i = 4 * q;
            f[u] = (q < n4 && i < live_end) ? quad_flags(i, pre[u]) : 0u;
            if (q < n4) *reinterpret_cast<uint32_t *>(flags + lo + i) = f[u];
            if constexpr (kCand) {
                // quad u of lane tid holds events 4 (q0 + u * T + tid) .. + 3: event order is u,
                // then lane; a quad has <= 4 flags, so three ballots give each lane its prefix
                const int c = __popc(f[u]);  // flag bytes are 0 or 1
                const uint64_t b0 = __ballot(c & 1), b1 = __ballot(c & 2), b2 = __ballot(c & 4);
                pfx[u] = __popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt);
                if (lane == 0) ctot[u][wave] = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
            }
        }
        if constexpr (kCand) {
            __syncthreads();
#pragma unroll
            for (int u = 0; u < kFlagQuads; ++u) {
                int off = base + pfx[u];
#pragma unroll
                for (int w = 0; w < kFlagThreads / 64; ++w) {
                    const int tw = ctot[u][w];
                    off += w < wave ? tw : 0;
                    base += tw;
                }
                if (f[u]) {
                    if (f[u] & 0x1u) dst[off++] = pre[u].x;
                    if (f[u] & 0x100u) dst[off++] = pre[u].y;
                    if (f[u] & 0x10000u) dst[off++] = pre[u].z;
                    if (f[u] & 0x1000000u) dst[off++] = pre[u].w;
                }
            }
            __syncthreads();  // ctot is rewritten by the next batch
        }
    }
    if constexpr (kCand) {
        if (threadIdx.x == 0) {
            for (int i = 4 * n4; i < len; ++i) {  // the batch's last < 4 events, in order
                const uint32_t v = xy[lo + i];
                const uint32_t fb = i < live_end ? corner_bit<kStaged>(v, g, sb, rg, j) : 0u;
                flags[lo + i] = (uint8_t)fb;
                if (fb) dst[base++] = v;
            }
            n_cand[s] = base;
        }
    } else {
        for (int i = 4 * n4 + threadIdx.x; i < len; i += kFlagThreads)  // last < 4 events, or unaligned slices
            flags[lo + i] = (uint8_t)(i < live_end ? corner_bit<kStaged>(xy[lo + i], g, sb, rg, j) : 0u);
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

// Per-context corner workspace: the sorted batch with its offset tables and the per-group images
// (sized by batch and sensor; grown, never shrunk).
struct CornerState {
    void *evt = nullptr;
    size_t evt_bytes = 0;
    // diagnostics of the last detection (ecc_fast_detect_stats)
    const uint32_t *n_over = nullptr;
    int64_t n_items = 0, n_slices = 0, n_groups = 0;
    // the unsorted-time verdict (ecc_fast_detect_status): every sort phase takes a fresh tag;
    // status_src says what the last call left to report (0: nothing, an empty call -> OK;
    // 1: a prepare-only call -> the pending word against prep_tag; 2: a finished call -> flags[0])
    int32_t next_tag = 0, prep_tag = 0;
    int status_src = 0;
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

struct GroupImages {
    uint32_t *mask;       // [n_groups][H*W] slices of the group that touched the pixel
    int64_t *B;           // [n_groups][H*W] last t of the group, then (in place) B_g
    uint32_t *res;        // [n_groups][32][n_tiles][kSegWords] corner (slice, pixel) pairs, slice-major
    uint4 *pv;            // [n_groups][H*W] value record of each (group, pixel) (pair_build)
    uint32_t *ovf;        // [n] the values past a record's first three, in each item's part of the range
    int64_t *over;        // [n_items] items arc_kernel leaves to arc_dense_kernel (heavy or undecidable)
    uint32_t *n_over;     // [0]: their count
};

Sorted carve_sorted(Carve &cv, const CornerGeom &g, int64_t n_items, int64_t n_groups, int32_t **first_border,
                    GroupImages *gi) {
    Sorted so{};
    so.key = cv.take<uint32_t>((size_t)g.n);
    so.t32 = cv.take<uint32_t>((size_t)g.n);
    so.toff = cv.take<int32_t>((size_t)g.n_slices * (g.n_tiles + 2));
    *first_border = cv.take<int32_t>((size_t)g.n_slices);
    const size_t img = (size_t)n_groups * g.W * g.H;
    gi->mask = cv.take<uint32_t>(img);
    gi->B = cv.take<int64_t>(img);
    gi->res = cv.take<uint32_t>((size_t)n_groups * kGroup * g.seg_stride);
    gi->pv = cv.take<uint4>(img);
    gi->ovf = cv.take<uint32_t>((size_t)g.n + 4 * (size_t)n_items + 8);
    gi->over = cv.take<int64_t>((size_t)n_items);
    gi->n_over = cv.take<uint32_t>(64);
    return so;
}

int corner_state_reserve(ecc_ctx *ctx, CornerState *st, size_t evt_need) {
    if (evt_need > st->evt_bytes) {
        if (st->evt) {
            ECC_CHECK_HIP(ctx, hipDeviceSynchronize(), "sync(corner batch)");
            (void)hipFree(st->evt);
            st->evt = nullptr;
            st->evt_bytes = 0;
            st->n_over = nullptr;
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
    cfg->any_order = 0;           // Metavision stream order (checked)
}

// phase bit 1: sort + pair entries (+ the shard-local last-t image when local_last != null);
// phase bit 2: SAE prefix from `sae` + arc tests + flags.  Both phases see the same workspace
// carve (same n and cfg), so prepare/finish may be separate calls with a collective between.
static int fast_detect_phases(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n,
                              const ecc_corner_cfg *cfg, int64_t *sae, uint8_t *corner_flags, int64_t *local_last,
                              int phases, ecc_stream_t stream, uint32_t *cand = nullptr, int32_t *n_cand = nullptr,
                              int32_t *zero_nms_err = nullptr) {
    if (!ctx || !cfg || n < 0) return ECC_ERR_INVALID;
    if ((phases & 2) && !sae) return ECC_ERR_INVALID;
    if (n > 0 && (!xy || !t || ((phases & 2) && !corner_flags))) return ECC_ERR_INVALID;
    if (cfg->width < 1 || cfg->height < 1 || cfg->width > 65536 || cfg->height > 65536)
        return ECC_ERR_INVALID;
    if (cfg->margin < 4 || 2 * cfg->margin >= cfg->width || 2 * cfg->margin >= cfg->height)
        return ECC_ERR_INVALID;  // the circles reach 4 px from the event
    if (cfg->slice_events < 1 || cfg->slice_events > kMaxSlice ||
        (cfg->border_mode != 0 && cfg->border_mode != 1))
        return ECC_ERR_INVALID;
    if (cfg->any_order != 0 && (cfg->any_order != 1 || phases != 3)) return ECC_ERR_INVALID;
    CornerGeom g{};
    g.W = cfg->width;
    g.H = cfg->height;
    g.S = cfg->slice_events;
    g.inv_S = 1.0f / (float)g.S;
    g.margin = cfg->margin;
    g.border_mode = cfg->border_mode;
    g.first_detect = cfg->first_detect_slice;
    g.any_order = cfg->any_order;
    g.tiles_x = (g.W + kTile - 1) / kTile;
    g.n_tiles = g.tiles_x * ((g.H + kTile - 1) / kTile);
    g.seg_stride = (g.n_tiles * kSegWords + 3) & ~3;
    if (g.n_tiles > kMaxTiles) return ECC_ERR_INVALID;  // > 8191 16x16 tiles (~2.1 Mpixel)
    // slice_sort's dedup bitmap (one bit per tile pixel), kept only while two of its workgroups
    // still fit a CU's LDS (sensors up to ~400 tiles of 14x14 pixels, e.g. 346x260)
    g.dedup_words = (int)(((int64_t)g.n_tiles * kTilePix + 31) / 32);
    if (((size_t)g.n_tiles + 1 + kSortChunk + g.dedup_words) * 4 + 256 > 80 * 1024) g.dedup_words = 0;
    g.n = n;
    g.n_slices = (n + g.S - 1) / g.S;
    if (g.n_slices > INT32_MAX) return ECC_ERR_INVALID;
    hipStream_t s = ecc::as_stream(stream);
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    CornerState *st = state_of(ctx);
    if (phases & 1) {  // a fresh tag for this sort phase (never 0: the pending word starts at 0)
        st->next_tag = st->next_tag == INT32_MAX ? 1 : st->next_tag + 1;
        st->prep_tag = st->next_tag;
    }
    if (n == 0) {
        st->status_src = 0;  // an empty call reports OK, whatever earlier calls saw
        if (local_last) ECC_CHECK_HIP(ctx, hipMemsetAsync(local_last, 0, (size_t)g.W * g.H * 8, s), "memset(local)");
        return ECC_OK;
    }
    const int nb = g.n_tiles + 1;
    const int64_t n_groups = (g.n_slices + kGroup - 1) / kGroup;
    const int64_t n_items = n_groups * g.n_tiles;  // work items: (group, tile)
    if (n_items > (int64_t)INT32_MAX - 8) return ECC_ERR_INVALID;
    if ((n + 4 * n_items) / 4 >= (int64_t)UINT32_MAX) return ECC_ERR_INVALID;  // 16-B overflow index in a u32
    int32_t *first_border = nullptr;
    GroupImages gi{};
    Carve measure{nullptr};
    carve_sorted(measure, g, n_items, n_groups, &first_border, &gi);
    if (!(phases & 1) && measure.used > st->evt_bytes) return ECC_ERR_INVALID;  // finish without prepare
    int rc = (phases & 1) ? corner_state_reserve(ctx, st, measure.used) : ECC_OK;
    if (rc) return rc;
    Carve cv{static_cast<char *>(st->evt)};
    const Sorted so = carve_sorted(cv, g, n_items, n_groups, &first_border, &gi);

    if (phases & 1) {
    {
        // > 64 KiB: opt in (gfx950 has 160 KiB); the dedup bitmap only while two workgroups fit a CU
        const size_t lds = ((size_t)nb + kSortChunk + g.dedup_words) * 4;
        static int lds_set = 0;
        if ((int)lds > lds_set) {
            ECC_CHECK_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void *>(&slice_sort_kernel),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   (int)((size_t)kMaxTiles * 4 + 4 + kSortChunk * 4)),
                          "slice_sort LDS");
            lds_set = kMaxTiles * 4 + 4 + kSortChunk * 4;
        }
        ECC_TIMED(ctx, s, "slice_sort_kernel");
        hipLaunchKernelGGL(slice_sort_kernel, dim3((unsigned)g.n_slices), dim3(kSortThreads), lds, s, xy, t, g,
                           so, first_border, ctx->flags + kSortPendingWord, st->prep_tag,
                           (phases & 2) ? gi.n_over : nullptr, zero_nms_err);
    }
    {
        ECC_TIMED(ctx, s, "pair_build_kernel");
        hipLaunchKernelGGL(pair_build_kernel, dim3((unsigned)n_items), dim3(kThreads), 0, s, t, g, so, gi.ovf, gi.pv,
                           gi.mask, gi.B);
    }
    if (local_last) {
        ECC_TIMED(ctx, s, "sae_local_last_kernel");
        const int64_t HW = (int64_t)g.W * g.H;
        const unsigned blocks = (unsigned)std::min<int64_t>((HW + kThreads - 1) / kThreads, 8192);
        hipLaunchKernelGGL(sae_local_last_kernel, dim3(blocks), dim3(kThreads), 0, s, g, n_groups,
                           (const uint32_t *)gi.mask, (const int64_t *)gi.B, local_last);
    }
    }  // phase 1
    if (!(phases & 2)) {
        st->status_src = 1;
        ECC_CHECK_LAUNCH(ctx, "fast_detect_prepare");
        return ECC_OK;
    }
    st->status_src = 2;
    st->n_over = gi.n_over;
    st->n_items = n_items;
    st->n_slices = g.n_slices;
    st->n_groups = n_groups;
    {
        ECC_TIMED(ctx, s, "sae_prefix_kernel");
        const int64_t HW = (int64_t)g.W * g.H;
        const unsigned blocks = (unsigned)((HW + kPrefixPix - 1) / kPrefixPix);
        hipLaunchKernelGGL(sae_prefix_kernel, dim3(blocks), dim3(kThreads), 0, s, g, n_groups,
                           (const uint32_t *)gi.mask, gi.B, sae, ctx->flags, ctx->flags + kSortPendingWord,
                           st->prep_tag, (phases & 1) ? nullptr : gi.n_over, (phases & 1) ? nullptr : zero_nms_err);
    }
    {
        ECC_TIMED(ctx, s, "arc_kernel");
        {
            const unsigned grid = (unsigned)(8 * ((n_items + 7) / 8));  // multiple of 8 (XCD-aware order)
            hipLaunchKernelGGL(arc_kernel, dim3(grid), dim3(kArcThreads), 0, s, t, g, n_items,
                               (const uint32_t *)gi.ovf, (const uint4 *)gi.pv, (const int64_t *)gi.B, (const uint32_t *)gi.mask, gi.res, gi.over, gi.n_over);
        }
    }
    {
        ECC_TIMED(ctx, s, "arc_dense_kernel");  // the items arc_kernel left: dense planes, exact tests
        hipLaunchKernelGGL(arc_dense_kernel, dim3(kDenseThreads == 512 ? 512 : ctx->n_cu), dim3(kDenseThreads), 0, s, t, g, (const int64_t *)gi.over,
                           (const uint32_t *)gi.n_over, (const uint32_t *)gi.ovf, (const uint4 *)gi.pv,
                           (const int64_t *)gi.B, (const uint32_t *)gi.mask, gi.res);
    }
    {
        ECC_TIMED(ctx, s, "flags_kernel");
        constexpr size_t kLdsMax = kFlagDynLdsMax;
        const size_t lds = (size_t)g.n_tiles * kSegWords * sizeof(uint32_t);
        if (lds <= kLdsMax) {
            static bool lds_set[2] = {false, false};
            const void *fn = cand ? reinterpret_cast<const void *>(&flags_event_kernel<true, true>)
                                  : reinterpret_cast<const void *>(&flags_event_kernel<true, false>);
            if (lds > 65536 && !lds_set[cand ? 1 : 0]) {
                ECC_CHECK_HIP(ctx, hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsMax),
                              "flags LDS");
                lds_set[cand ? 1 : 0] = true;
            }
            if (cand)
                hipLaunchKernelGGL((flags_event_kernel<true, true>), dim3((unsigned)g.n_slices), dim3(kFlagThreads), lds, s,
                                   xy, g, (const uint32_t *)gi.res, (const int32_t *)first_border, corner_flags, cand,
                                   n_cand);
            else
                hipLaunchKernelGGL((flags_event_kernel<true, false>), dim3((unsigned)g.n_slices), dim3(kFlagThreads), lds,
                                   s, xy, g, (const uint32_t *)gi.res, (const int32_t *)first_border, corner_flags,
                                   nullptr, nullptr);
        } else {
            if (cand) return ECC_ERR_INVALID;  // the caller checks ecc_fast_detect_nms' conditions
            hipLaunchKernelGGL((flags_event_kernel<false, false>), dim3((unsigned)g.n_slices), dim3(kFlagThreads), 0, s,
                               xy, g, (const uint32_t *)gi.res, (const int32_t *)first_border, corner_flags, nullptr,
                               nullptr);
        }
    }
    ECC_CHECK_LAUNCH(ctx, "fast_detect");
    return ECC_OK;
}

#if ECC_ARC_PROFILE
// Profiling builds only (make ARC_PROFILE=1): arc_kernel's summed per-workgroup phase ticks
// since the last call (reset after reading); out[7] = items timed; ticks_per_us from the device.
ECC_API int ecc_arc_dense_profile(unsigned long long *out8, double *ticks_per_us) {
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_dense_prof), 8 * sizeof(unsigned long long)) != hipSuccess) return ECC_ERR_HIP;
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_dense_prof), z, sizeof(z));
    int khz = 0;
    hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    *ticks_per_us = khz / 1000.0;
    return ECC_OK;
}

ECC_API int ecc_arc_profile(unsigned long long *out8, double *ticks_per_us) {
    std::vector<unsigned long long> h((size_t)kProfItems * 8);
    if (hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_arc_items), h.size() * 8) != hipSuccess) return ECC_ERR_HIP;
    for (int k = 0; k < 8; ++k) out8[k] = 0;
    for (size_t it = 0; it < (size_t)kProfItems; ++it)
        if (h[it * 8 + 7])
            for (int k = 0; k < 8; ++k) out8[k] += h[it * 8 + k];
    std::fill(h.begin(), h.end(), 0ull);
    hipMemcpyToSymbol(HIP_SYMBOL(g_arc_items), h.data(), h.size() * 8);
    int khz = 0;
    hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    *ticks_per_us = khz / 1000.0;
    return ECC_OK;
}
#endif

ECC_API int ecc_fast_detect(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n,
                            const ecc_corner_cfg *cfg, int64_t *sae, uint8_t *corner_flags,
                            ecc_stream_t stream) {
    return fast_detect_phases(ctx, xy, t, n, cfg, sae, corner_flags, nullptr, 3, stream);
}

// detection (phases 3: sort + tests; 2: the finish half) followed by the per-slice NMS
static int fast_detect_nms_phases(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n,
                                  const ecc_corner_cfg *cfg, int64_t *sae, uint8_t *corner_flags, int32_t box_size,
                                  int32_t cap, ecc_corner *out, int32_t *out_count, int phases, ecc_stream_t stream) {
    if (!ctx || !cfg) return ECC_ERR_INVALID;
    if (ecc::nms_check_args(n, cfg->slice_events, cfg->width, cfg->height, box_size, cap)) return ECC_ERR_INVALID;
    if (n > 0 && (!out_count || (cap > 0 && !out))) return ECC_ERR_INVALID;
    const int64_t tiles = (int64_t)((cfg->width + kTile - 1) / kTile) * ((cfg->height + kTile - 1) / kTile);
    uint32_t *cand = nullptr;
    int32_t *n_cand = nullptr;
    if (n > 0 && cfg->slice_events % 4 == 0 && cfg->slice_events <= kFlagCandMax &&
        tiles * kSegWords * 4 <= (int64_t)kFlagDynLdsMax) {
        int rc = ecc::nms_candidates(ctx, n, cfg->slice_events, cfg->width, cfg->height, box_size, &cand, &n_cand);
        if (rc) return rc;
    }
    if (!cand) {  // the two calls
        int rc = phases == 3 ? ecc_fast_detect(ctx, xy, t, n, cfg, sae, corner_flags, stream)
                             : ecc_fast_detect_finish(ctx, xy, t, n, cfg, sae, corner_flags, stream);
        if (rc) return rc;
        return ecc_corner_nms(ctx, xy, corner_flags, n, cfg->slice_events, cfg->width, cfg->height, box_size, cap, out,
                              out_count, stream);
    }
    hipStream_t s = ecc::as_stream(stream);
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    // the NMS error word is zeroed by the call's first kernel (n > 0 here: nms_candidates gave a
    // buffer): the sort kernel, or in a finish-only call the SAE prefix
    int rc = fast_detect_phases(ctx, xy, t, n, cfg, sae, corner_flags, nullptr, phases, stream, cand, n_cand,
                                ctx->flags + 1);
    if (rc) return rc;
    rc = ecc::nms_greedy(ctx, cand, n_cand, n, cfg->slice_events, cfg->width, cfg->height, box_size, cap, out,
                         out_count, s);
    if (rc) return rc;
    ECC_CHECK_LAUNCH(ctx, "fast_detect_nms");
    return ECC_OK;
}

ECC_API int ecc_fast_detect_nms(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n,
                                const ecc_corner_cfg *cfg, int64_t *sae, uint8_t *corner_flags, int32_t box_size,
                                int32_t cap, ecc_corner *out, int32_t *out_count, ecc_stream_t stream) {
    return fast_detect_nms_phases(ctx, xy, t, n, cfg, sae, corner_flags, box_size, cap, out, out_count, 3, stream);
}

ECC_API int ecc_fast_detect_finish_nms(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n,
                                       const ecc_corner_cfg *cfg, int64_t *sae, uint8_t *corner_flags,
                                       int32_t box_size, int32_t cap, ecc_corner *out, int32_t *out_count,
                                       ecc_stream_t stream) {
    return fast_detect_nms_phases(ctx, xy, t, n, cfg, sae, corner_flags, box_size, cap, out, out_count, 2, stream);
}

ECC_API int ecc_fast_detect_prepare(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n,
                                    const ecc_corner_cfg *cfg, int64_t *local_last, ecc_stream_t stream) {
    return fast_detect_phases(ctx, xy, t, n, cfg, nullptr, nullptr, local_last, 1, stream);
}

ECC_API int ecc_fast_detect_finish(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n,
                                   const ecc_corner_cfg *cfg, int64_t *sae, uint8_t *corner_flags,
                                   ecc_stream_t stream) {
    return fast_detect_phases(ctx, xy, t, n, cfg, sae, corner_flags, nullptr, 2, stream);
}

ECC_API int ecc_fast_detect_status(ecc_ctx *ctx, ecc_stream_t stream) {
    if (!ctx) return ECC_ERR_INVALID;
    // the verdict of the last call on this context (CornerState::status_src)
    const CornerState *st = state_of(ctx);
    if (st->status_src == 0) return ECC_OK;
    int32_t w = 0;
    const int32_t *src = st->status_src == 1 ? ctx->flags + kSortPendingWord : ctx->flags;
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(&w, src, 4, hipMemcpyDeviceToHost, ecc::as_stream(stream)), "read err flag");
    ECC_CHECK_HIP(ctx, hipStreamSynchronize(ecc::as_stream(stream)), "sync");
    const bool bad = st->status_src == 1 ? w == st->prep_tag : w != 0;
    return bad ? ECC_ERR_UNSORTED_TIME : ECC_OK;
}

ECC_API int ecc_fast_detect_stats(ecc_ctx *ctx, int64_t *out, int32_t n_out, ecc_stream_t stream) {
    if (!ctx || n_out < 0 || (n_out > 0 && !out)) return ECC_ERR_INVALID;
    CornerState *st = state_of(ctx);
    uint32_t ov = 0;
    if (st->n_over) {
        ECC_CHECK_HIP(ctx, hipMemcpyAsync(&ov, st->n_over, 4, hipMemcpyDeviceToHost, ecc::as_stream(stream)),
                      "read overflow count");
        ECC_CHECK_HIP(ctx, hipStreamSynchronize(ecc::as_stream(stream)), "sync");
    }
    const int64_t v[4] = {st->n_items, (int64_t)ov, st->n_slices, st->n_groups};
    for (int i = 0; i < n_out && i < 4; ++i) out[i] = v[i];
    return ECC_OK;
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
