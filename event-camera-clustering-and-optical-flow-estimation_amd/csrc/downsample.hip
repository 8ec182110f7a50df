// Hash-map downsampler.
//
// Reference: __kernel process_coordinates, SMP/build/coordinate_processor.cl:16-89 — ONE
// work-group of 1024 lanes whose lane 0 zeroes an 8192-int LDS table serially, then lanes
// race with atomic_inc: the first hit of a bucket appends (x,y) to unique_coords (racy winner
// and order, Q2), the second hit bumps repeated_count.
//
// MI355X design: one workgroup (8 wave64) per 8192-event window, all windows of a batch in
// ONE launch.  The window's packed-xy events are loaded with 16-B loads straight into
// registers (HBM-bound stream, 4 B/event), each bucket keeps the MINIMUM local event index via
// ds_min_u32 (canonical deterministic representative), a second pass marks repeated buckets
// with ds_or (bit 31), and representatives are compacted in ascending event order with
// wave ballots + a per-chunk wave-total table in LDS.  Algorithmic bytes: 4 B/event in,
// 4 B/representative out (rep_xy; +4 with rep_idx), 8 B/window of counts.
#include "ecc_internal.hpp"

namespace {

// 8 waves per window (16 events per lane at 8192): four workgroups per CU by waves (33 KB of LDS
// each).  Measured per kernel on the bench stream: 256 lanes 50 us (five per CU by LDS, each
// window's phases on 4 waves), 512 lanes 42 us, 1024 lanes 48 us (two per CU).
constexpr int kThreads = 512;
constexpr int kMaxWindow = 16384;
constexpr int kBuckets = 8192;            // LDS table (32 KiB)
constexpr uint32_t kEmpty = 0x7fffffffu;
constexpr uint32_t kRepeatBit = 0x80000000u;

// Four consecutive events per lane.  kQuads (window and n multiples of 4, xy 16-B aligned): one
// 16-B load per lane, clamped to the last quad; otherwise four clamped 4-B loads.  Values past the
// window are masked by the caller.  No load is conditional: a per-lane choice between a 16-B and
// four 4-B loads into the same registers made the compiler wait for each chunk's load before
// issuing the next (four HBM round trips per window instead of one).
template <bool kQuads>
__device__ inline void load4(const uint32_t *__restrict__ xy, int64_t g, int64_t n, uint32_t (&v)[4]) {
    if constexpr (kQuads) {
        const int64_t n4 = n >> 2, qi = g >> 2;
        const uint4 q = reinterpret_cast<const uint4 *>(xy)[qi < n4 ? qi : n4 - 1];
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = xy[g + k < n ? g + k : n - 1];
    }
}

template <int NT, int MAXC, bool kQuads>
__global__ void __launch_bounds__(NT)
downsample_hash_kernel(const uint32_t *__restrict__ xy, int64_t n, int window, int n_chunks,
                       int x_max, int y_max, int mult_x, int mult_y,
                       uint32_t *__restrict__ rep_xy, uint32_t *__restrict__ rep_idx,
                       int32_t *__restrict__ win_unique, int32_t *__restrict__ win_repeated) {
    __shared__ __attribute__((aligned(16))) uint32_t table[kBuckets];
    constexpr int kWaves = NT / 64, kChunk = NT * 4;  // events per chunk: 4 consecutive per lane
    __shared__ int wave_tot[MAXC][kWaves];
    __shared__ int red[kWaves];

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & 63;
    const int64_t w = blockIdx.x;
    const int64_t wbase = w * (int64_t)window;
    const int64_t wend = (wbase + window < n) ? wbase + window : n;

    // 1. zero the bucket table (vectorised; the reference's lane-0 serial loop, :35-44)
    {
        uint4 *t4 = reinterpret_cast<uint4 *>(table);
        const uint4 e = make_uint4(kEmpty, kEmpty, kEmpty, kEmpty);
        for (int i = tid; i < kBuckets / 4; i += NT) t4[i] = e;
    }

    // 2. load the window into registers: lane owns events wbase + c*1024 + 4*tid + k
    uint32_t v[MAXC][4];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        if (c < n_chunks) {
            load4<kQuads>(xy, wbase + (int64_t)c * kChunk + 4 * tid, n, v[c]);
        }
    }
    __syncthreads();

    // bucket of an event (:11) or 0xffffffff when out of range / past the window end (:56)
    auto bucket = [&](int c, int k) -> uint32_t {
        const int li = c * kChunk + 4 * tid + k;
        const int x = ecc::xy_x(v[c][k]), y = ecc::xy_y(v[c][k]);
        const bool ok = (wbase + li < wend) && x <= x_max && y <= y_max;
        return ok ? (uint32_t)((x * mult_x + y * mult_y) & (kBuckets - 1)) : 0xffffffffu;
    };

    // 3. first-hit = minimum local index per bucket (:62 atomic_inc race -> ds_min_u32)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        if (c < n_chunks) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t h = bucket(c, k);
                if (h != 0xffffffffu) atomicMin(&table[h], (uint32_t)(c * kChunk + 4 * tid + k));
            }
        }
    }
    __syncthreads();

    // 4. representatives (bucket min == own index) and repeated marks (:65-75); a bucket is
    //    repeated (hit >= 2 times) iff some non-first event's ds_or finds bit 31 clear: exactly
    //    one such ds_or per repeated bucket, so the returned old values count them
    uint32_t repmask[MAXC];
    int rp = 0;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        repmask[c] = 0;
        if (c < n_chunks) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t h = bucket(c, k);
                if (h != 0xffffffffu) {
                    const int li = c * kChunk + 4 * tid + k;
                    const uint32_t first = table[h] & kEmpty;
                    if (first == (uint32_t)li) repmask[c] |= 1u << k;
                    else rp += (atomicOr(&table[h], kRepeatBit) & kRepeatBit) ? 0 : 1;
                }
            }
        }
    }

    // 5. per chunk, rank of this lane's first rep among the wave (3 ballots on the 0..4 count)
    int lane_prefix[MAXC];
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        lane_prefix[c] = 0;
        if (c < n_chunks) {
            const int r = __popc(repmask[c]);
            const uint64_t b0 = __ballot(r & 1), b1 = __ballot(r & 2), b2 = __ballot(r & 4);
            lane_prefix[c] = __popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt);
            if (lane == 0) wave_tot[c][wave] = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
        }
    }
    __syncthreads();

    // 6. repeated count per wave (unique = occupied buckets = the representatives: step 7's total)
    rp = ecc::wave_sum_i32(rp);  // DPP
    if (lane == 0) red[wave] = rp;

    // 7. compacted write-out in ascending event order
    int base = 0;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        if (c < n_chunks) {
            int off = base + lane_prefix[c];
            for (int ww = 0; ww < kWaves; ++ww) {
                const int t = wave_tot[c][ww];
                if (ww < wave) off += t;
                base += t;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (repmask[c] & (1u << k)) {
                    const int li = c * kChunk + 4 * tid + k;
                    if (rep_xy) rep_xy[wbase + off] = v[c][k];
                    if (rep_idx) rep_idx[wbase + off] = (uint32_t)(wbase + li);
                    ++off;
                }
            }
        }
    }
    __syncthreads();
    if (tid == 0) {
        int r = 0;
        for (int ww = 0; ww < kWaves; ++ww) r += red[ww];
        if (win_unique) win_unique[w] = base;  // every lane's `base` is the window's total
        if (win_repeated) win_repeated[w] = r;
    }
}

}  // namespace

ECC_API void ecc_hash_cfg_default(ecc_hash_cfg *cfg) {
    if (!cfg) return;
    cfg->window = 8192;     // SMP/…opencl_store.cpp:34-38 (ARRAY_SIZE 16384 ints = 8192 pairs)
    cfg->x_max = 1280;      // coordinate_processor.cl:56
    cfg->y_max = 720;
    cfg->mult_x = 1619;     // coordinate_processor.cl:11
    cfg->mult_y = 31;
    cfg->n_buckets = 8192;
}

ECC_API int ecc_downsample_hash(ecc_ctx *ctx, const uint32_t *xy, int64_t n,
                                const ecc_hash_cfg *cfg, uint32_t *rep_xy, uint32_t *rep_idx,
                                int32_t *win_unique, int32_t *win_repeated, ecc_stream_t stream) {
    if (!ctx || !cfg || n < 0 || (n > 0 && !xy)) return ECC_ERR_INVALID;
    if (cfg->window < 1 || cfg->window > kMaxWindow) return ECC_ERR_INVALID;
    if (cfg->n_buckets != kBuckets) return ECC_ERR_INVALID;
    if (cfg->x_max < 0 || cfg->y_max < 0 || cfg->mult_x < 0 || cfg->mult_y < 0) return ECC_ERR_INVALID;
    // (x*mult_x + y*mult_y) must not overflow int32 for u16 coordinates
    if ((int64_t)65535 * cfg->mult_x + (int64_t)65535 * cfg->mult_y > INT32_MAX) return ECC_ERR_INVALID;
    if (n == 0) return ECC_OK;
    const int64_t n_win = (n + cfg->window - 1) / cfg->window;
    if (n_win > INT32_MAX) return ECC_ERR_INVALID;
    const int n_chunks = (cfg->window + 4 * kThreads - 1) / (4 * kThreads);
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    // 16-B loads when every lane's quad is aligned (the instantiations keep one load form each)
    const bool quads = (cfg->window & 3) == 0 && (n & 3) == 0 && (reinterpret_cast<uintptr_t>(xy) & 15) == 0;
    auto kern = quads ? (n_chunks <= 4 ? downsample_hash_kernel<kThreads, 4, true> : downsample_hash_kernel<kThreads, 8, true>)
                      : (n_chunks <= 4 ? downsample_hash_kernel<kThreads, 4, false> : downsample_hash_kernel<kThreads, 8, false>);
    {
        ECC_TIMED(ctx, ecc::as_stream(stream), "downsample_hash_kernel");
        hipLaunchKernelGGL(kern, dim3((unsigned)n_win), dim3(kThreads), 0, ecc::as_stream(stream), xy,
                           n, cfg->window, n_chunks, cfg->x_max, cfg->y_max, cfg->mult_x, cfg->mult_y,
                           rep_xy, rep_idx, win_unique, win_repeated);
    }
    ECC_CHECK_LAUNCH(ctx, "downsample_hash_kernel");
    return ECC_OK;
}
