// Exact (x, y) deduplication per window.
//
// Reference: analyzeCoordinates / findCoordinate, FCT/metavision_time_surface_periodic.cpp:
// 56-120 (also …periodic_corner.cpp:306-379): for the ARRAY_SIZE = 16384 ints of a window
// (8192 (x, y) pairs), a linear search of the unique list so far per pair — O(n·u) — that appends
// a new coordinate with count 1 or bumps the count of an existing one, then prints the number of
// unique coordinates.  Its only call site is commented out (:214), but the function is the exact
// counterpart of the lossy bucket downsampler (process_coordinates, rows a1-a2).
//
// MI355X design: one workgroup (4 wave64) per window, all windows in ONE launch.  The window's
// packed-xy events (16-B loads, registers) go into an LDS open-addressing table of 2x the window
// size whose 64-bit slots hold (xy << 32 | first index): ds_cmpst_b64 claims an empty slot and
// ds_min_u64 keeps the smallest event index of a coordinate (its first occurrence — the order of
// the reference's list).  The first occurrences then reset their slot's low word to 0 and every
// event adds 1 (ds_add_u64): the per-coordinate counts.  First occurrences are compacted in
// event order with wave ballots (as downsample.hip).  Algorithmic bytes: 4 B/event in + 8 B per
// unique coordinate (index + count) + 4 B/window.
#include "ecc_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kChunk = kThreads * 4;  // events per chunk: 4 consecutive per lane
constexpr int kMaxChunks = 8;         // window <= 8192 pairs (the reference's ARRAY_SIZE / 2)
constexpr int kSlots = 16384;         // 2x the largest window: load factor <= 1/2
constexpr unsigned long long kEmptySlot = ~0ull;

__device__ __forceinline__ uint32_t slot_hash(uint32_t v) { return (v * 0x9E3779B1u) >> 18; }  // 14 bits

__global__ void __launch_bounds__(kThreads)
dedup_exact_kernel(const uint32_t *__restrict__ xy, int64_t n, int window, int n_chunks, uint32_t *__restrict__ uniq_idx,
                   int32_t *__restrict__ uniq_cnt, int32_t *__restrict__ n_unique) {
    __shared__ unsigned long long table[kSlots];  // 128 KiB
    __shared__ int wave_tot[kMaxChunks][kWaves];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int64_t wbase = blockIdx.x * (int64_t)window;
    const int64_t wend = (wbase + window < n) ? wbase + window : n;
    const int m = (int)(wend - wbase);
    for (int i = tid; i < kSlots; i += kThreads) table[i] = kEmptySlot;
    uint32_t v[kMaxChunks][4];
    int slot[kMaxChunks][4];
#pragma unroll
    for (int c = 0; c < kMaxChunks; ++c) {
        if (c >= n_chunks) continue;
        const int li = c * kChunk + 4 * tid;
        const int64_t g = wbase + li;
        if (li + 3 < m && (g & 3) == 0) {
            const uint4 q = *reinterpret_cast<const uint4 *>(xy + g);
            v[c][0] = q.x; v[c][1] = q.y; v[c][2] = q.z; v[c][3] = q.w;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) v[c][k] = li + k < m ? xy[g + k] : 0u;
        }
    }
    __syncthreads();
    // 1. claim / find the coordinate's slot; keep the smallest event index in its low word
#pragma unroll
    for (int c = 0; c < kMaxChunks; ++c) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int li = c * kChunk + 4 * tid + k;
            slot[c][k] = -1;
            if (c >= n_chunks || li >= m) continue;
            const unsigned long long mine = ((unsigned long long)v[c][k] << 32) | (uint32_t)li;
            uint32_t h = slot_hash(v[c][k]);
            for (;;) {
                const unsigned long long prev = atomicCAS(&table[h], kEmptySlot, mine);
                if (prev == kEmptySlot) break;
                if ((uint32_t)(prev >> 32) == v[c][k]) {
                    atomicMin(&table[h], mine);
                    break;
                }
                h = (h + 1) & (kSlots - 1);
            }
            slot[c][k] = (int)h;
        }
    }
    __syncthreads();
    // 2. first occurrences (slot minimum == own index); ranks for the event-order compaction
    uint32_t firstmask[kMaxChunks];
    int lane_prefix[kMaxChunks];
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int c = 0; c < kMaxChunks; ++c) {
        firstmask[c] = 0;
        lane_prefix[c] = 0;
        if (c >= n_chunks) continue;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (slot[c][k] >= 0 && (uint32_t)table[slot[c][k]] == (uint32_t)(c * kChunk + 4 * tid + k))
                firstmask[c] |= 1u << k;
        const int r = __popc(firstmask[c]);
        const uint64_t b0 = __ballot(r & 1), b1 = __ballot(r & 2), b2 = __ballot(r & 4);
        lane_prefix[c] = __popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt);
        if (lane == 0) wave_tot[c][wave] = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
    }
    __syncthreads();
    // 3. counts: the first occurrence clears its slot's low word, then every event adds one
#pragma unroll
    for (int c = 0; c < kMaxChunks; ++c)
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (firstmask[c] & (1u << k)) table[slot[c][k]] = (unsigned long long)v[c][k] << 32;
    __syncthreads();
#pragma unroll
    for (int c = 0; c < kMaxChunks; ++c)
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (slot[c][k] >= 0) atomicAdd(&table[slot[c][k]], 1ull);
    __syncthreads();
    // 4. compacted write-out in ascending event order
    int base = 0;
#pragma unroll
    for (int c = 0; c < kMaxChunks; ++c) {
        if (c >= n_chunks) continue;
        int off = base + lane_prefix[c];
        for (int ww = 0; ww < kWaves; ++ww) {
            const int t = wave_tot[c][ww];
            if (ww < wave) off += t;
            base += t;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!(firstmask[c] & (1u << k))) continue;
            if (uniq_idx) uniq_idx[wbase + off] = (uint32_t)(wbase + c * kChunk + 4 * tid + k);
            if (uniq_cnt) uniq_cnt[wbase + off] = (int32_t)(uint32_t)table[slot[c][k]];
            ++off;
        }
    }
    if (tid == 0 && n_unique) n_unique[blockIdx.x] = base;
}

}  // namespace

ECC_API int ecc_dedup_exact(ecc_ctx *ctx, const uint32_t *xy, int64_t n, int32_t window, uint32_t *uniq_idx,
                            int32_t *uniq_cnt, int32_t *n_unique, ecc_stream_t stream) {
    if (!ctx || n < 0 || (n > 0 && !xy) || window < 1 || window > kMaxChunks * kChunk) return ECC_ERR_INVALID;
    if (n == 0) return ECC_OK;
    const int64_t n_win = (n + window - 1) / window;
    if (n_win > INT32_MAX) return ECC_ERR_INVALID;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    const int n_chunks = (window + kChunk - 1) / kChunk;
    {
        ECC_TIMED(ctx, ecc::as_stream(stream), "dedup_exact_kernel");
        hipLaunchKernelGGL(dedup_exact_kernel, dim3((unsigned)n_win), dim3(kThreads), 0, ecc::as_stream(stream), xy, n,
                           window, n_chunks, uniq_idx, uniq_cnt, n_unique);
    }
    ECC_CHECK_LAUNCH(ctx, "dedup_exact_kernel");
    return ECC_OK;
}
