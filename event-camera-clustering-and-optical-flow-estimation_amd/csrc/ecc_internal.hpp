// Internal definitions shared by the HIP translation units of libecc (gfx950 / CDNA4).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/ecc.h"

#define ECC_API extern "C" __attribute__((visibility("default")))

struct EccKernelStat {
    double total_ms = 0.0;
    int64_t launches = 0;
};

struct EccTimingPair {
    const char *name;
    hipEvent_t a, b;
};

struct ecc_ctx {
    int device = 0;
    int n_cu = 256;  // compute units of the device (persistent-grid sizing)
    // per-kernel timing (ecc_ctx_set_timing)
    bool timing = false;
    std::vector<EccTimingPair> pending;
    std::vector<hipEvent_t> event_pool;
    std::map<std::string, EccKernelStat> stats;
    std::string last_error;
    // Scratch workspace, grown on demand (never inside a capture: call once eagerly first).
    void *ws = nullptr;
    size_t ws_bytes = 0;
    // Small pinned-free device words: [0] unsorted-time flag of the last fast_detect.
    int32_t *flags = nullptr;
};

namespace ecc {

// Records the HIP error on the context and returns ECC_ERR_HIP.
int hip_fail(ecc_ctx *ctx, hipError_t e, const char *what);

// Ensures the context workspace holds >= bytes (16-byte aligned carve base). Returns status.
int ws_reserve(ecc_ctx *ctx, size_t bytes);

inline hipStream_t as_stream(ecc_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Brackets one kernel launch with HIP events when the context's timing mode is on.
struct TimedLaunch {
    ecc_ctx *ctx;
    hipStream_t s;
    const char *name;
    hipEvent_t a = nullptr;
    TimedLaunch(ecc_ctx *c, hipStream_t st, const char *n);
    ~TimedLaunch();
};
#define ECC_TIMED(ctx, stream, name) ::ecc::TimedLaunch _ecc_tl((ctx), (stream), (name))

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// out[0..n] = exclusive scan of in[0..n) with out[n] = total (scratch: scan_scratch_bytes(n)).
size_t scan_scratch_bytes(int64_t n);
int exclusive_scan_i32_i64(ecc_ctx *ctx, const int32_t *in, int64_t n, int64_t *out, int64_t *scratch,
                           hipStream_t s);

// Frees the per-context corner-stage workspace (corners.hip); called by ecc_ctx_destroy.
void corner_state_release(const ecc_ctx *ctx);
// Frees the per-context NMS candidate buffer (nms.hip); called by ecc_ctx_destroy.
void nms_state_release(const ecc_ctx *ctx);
// Grid NMS in two steps (nms.hip), so that a producer of the per-slice candidate lists (the
// corner flag pass of ecc_fast_detect_nms) can replace nms_compact_kernel: the argument check of
// ecc_corner_nms; the per-context candidate buffer (n xy words at cand[s * S ...], counts
// n_cand[s]; both null when the grid form does not apply: a grid above 64 KiB of LDS); the
// greedy pass over the lists.
int nms_check_args(int64_t n, int32_t slice_events, int32_t width, int32_t height, int32_t box_size, int32_t cap);
int nms_candidates(ecc_ctx *ctx, int64_t n, int32_t slice_events, int32_t width, int32_t height, int32_t box_size,
                   uint32_t **cand, int32_t **n_cand);
int nms_greedy(ecc_ctx *ctx, const uint32_t *cand, const int32_t *n_cand, int64_t n, int32_t slice_events,
               int32_t width, int32_t height, int32_t box_size, int32_t cap, ecc_corner *out, int32_t *out_count,
               hipStream_t s);

// Launch-error check: kernel launches are asynchronous; this surfaces configuration errors.
#define ECC_CHECK_LAUNCH(ctx, what)                                  \
    do {                                                             \
        hipError_t _e = hipGetLastError();                           \
        if (_e != hipSuccess) return ::ecc::hip_fail(ctx, _e, what); \
    } while (0)

#define ECC_CHECK_HIP(ctx, call, what)                               \
    do {                                                             \
        hipError_t _e = (call);                                      \
        if (_e != hipSuccess) return ::ecc::hip_fail(ctx, _e, what); \
    } while (0)

// Packed xy helpers (x | y << 16).
__host__ __device__ inline int xy_x(uint32_t v) { return (int)(v & 0xffffu); }
__host__ __device__ inline int xy_y(uint32_t v) { return (int)(v >> 16); }

// Raw buffer view of [p, p + bytes) (stride 0, gfx9 resource word 3): loads at or past `bytes`
// return 0 by the hardware range check, so a wave can issue all its loads over a ragged range
// unconditionally (a load under a per-lane condition waits for every earlier one).
// The view must be wave-uniform (a divergent resource becomes a waterfall loop per load), so its
// words go through readfirstlane: callers pass uniform values, the compiler need not prove it.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_view(const void *p, uint32_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint64_t ua = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(ua), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ uint32_t buffer_load_u32(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff = 0) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0);
}
__device__ __forceinline__ void buffer_store_u32(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff = 0) {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)voff, (int)soff, 0);
}
__device__ __forceinline__ int64_t buffer_load_i64(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff = 0) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0);
    return (int64_t)(((uint64_t)v[1] << 32) | v[0]);
}
__device__ __forceinline__ uint4 buffer_load_u128(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff = 0) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// Inclusive prefix sum over the 64 lanes of a wave with DPP moves (no LDS round trip): row_shr
// 1/2/4/8 scans each row of 16 (bound_ctrl fills zeros at the row start), then row_bcast:15
// adds row 0's total into row 1 and row 2's into row 3, and row_bcast:31 adds rows 0-1's
// total into rows 2-3.  All 64 lanes must be active.
__device__ __forceinline__ int wave_incl_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
    return x;
}

// Wave reductions by DPP moves (VALU only: the __shfl_xor butterflies are LDS permutes, which
// competed with the kernels' own LDS traffic — the arc kernel's scans and minimum were a fifth of
// its LDS instructions).  Row rotations 8/4/2/1 leave every lane its row's result, row_bcast:15
// folds rows 0 -> 1 and 2 -> 3, row_bcast:31 folds rows 0-1 into 2-3, so lane 63 holds the
// wave's result, which is returned to every lane (readlane: wave-uniform).  Rows a broadcast
// step does not write keep `identity`'s contribution.  All 64 lanes must be active.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t identity, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)identity, (int)v, kCtrl, kRowMask, 0xf, false);
}
template <class Op>
__device__ __forceinline__ uint32_t wave_reduce_u32(uint32_t v, uint32_t identity, Op op) {
    v = op(v, dpp_u32<0x128, 0xf>(identity, v));  // row_ror:8
    v = op(v, dpp_u32<0x124, 0xf>(identity, v));  // row_ror:4
    v = op(v, dpp_u32<0x122, 0xf>(identity, v));  // row_ror:2
    v = op(v, dpp_u32<0x121, 0xf>(identity, v));  // row_ror:1
    v = op(v, dpp_u32<0x142, 0xa>(identity, v));  // row_bcast:15 into rows 1, 3
    v = op(v, dpp_u32<0x143, 0xc>(identity, v));  // row_bcast:31 into rows 2, 3
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int wave_min_i32(int v) {
    return (int)wave_reduce_u32((uint32_t)v, 0x7fffffffu, [](uint32_t a, uint32_t b) { return (uint32_t)min((int)a, (int)b); });
}
__device__ __forceinline__ int wave_max_i32(int v) {
    return (int)wave_reduce_u32((uint32_t)v, 0x80000000u, [](uint32_t a, uint32_t b) { return (uint32_t)max((int)a, (int)b); });
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    return wave_reduce_u32(v, 0u, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
}
__device__ __forceinline__ int wave_sum_i32(int v) {
    return (int)wave_reduce_u32((uint32_t)v, 0u, [](uint32_t a, uint32_t b) { return a + b; });
}
template <int kCtrl, int kRowMask>
__device__ __forceinline__ int64_t dpp_i64(int64_t identity, int64_t v) {
    const uint32_t lo = dpp_u32<kCtrl, kRowMask>((uint32_t)identity, (uint32_t)v);
    const uint32_t hi = dpp_u32<kCtrl, kRowMask>((uint32_t)((uint64_t)identity >> 32), (uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <class Op>
__device__ __forceinline__ int64_t wave_reduce_i64(int64_t v, int64_t identity, Op op) {
    v = op(v, dpp_i64<0x128, 0xf>(identity, v));
    v = op(v, dpp_i64<0x124, 0xf>(identity, v));
    v = op(v, dpp_i64<0x122, 0xf>(identity, v));
    v = op(v, dpp_i64<0x121, 0xf>(identity, v));
    v = op(v, dpp_i64<0x142, 0xa>(identity, v));
    v = op(v, dpp_i64<0x143, 0xc>(identity, v));
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, 63);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)v >> 32), 63);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
    return wave_reduce_i64(v, INT64_MAX, [](int64_t a, int64_t b) { return a < b ? a : b; });
}
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
    return wave_reduce_i64(v, INT64_MIN, [](int64_t a, int64_t b) { return a > b ? a : b; });
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
    return wave_reduce_i64(v, 0, [](int64_t a, int64_t b) { return a + b; });
}
// Inclusive prefix sum of an int64 over the wave (wave_incl_scan's pattern on both halves).
__device__ __forceinline__ int64_t wave_incl_scan_i64(int64_t x) {
    x += dpp_i64<0x111, 0xf>(0, x);
    x += dpp_i64<0x112, 0xf>(0, x);
    x += dpp_i64<0x114, 0xf>(0, x);
    x += dpp_i64<0x118, 0xf>(0, x);
    x += dpp_i64<0x142, 0xa>(0, x);
    x += dpp_i64<0x143, 0xc>(0, x);
    return x;
}
// The value of a wave-uniform lane index (readlane: scalar, no LDS permute).
__device__ __forceinline__ int lane_value(int v, int lane_idx) { return __builtin_amdgcn_readlane(v, lane_idx); }
__device__ __forceinline__ int64_t lane_value64(int64_t v, int lane_idx) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, lane_idx);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)v >> 32), lane_idx);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Correctly rounded fp32 square root.  On gfx950 `__fsqrt_rn` may lower to the bare
// v_sqrt_f32 (<= 1 ulp), which breaks bit-exactness against IEEE sqrtf on the host.  This is
// the hardware approximation followed by the exact one-ulp correction with FMA residuals
// (x - r'*r for the two neighbours r' of r), with scaling for tiny inputs.
__device__ __forceinline__ float sqrt_rn(float x) {
    const bool tiny = x < 0x1p-96f;
    const float xs = tiny ? x * 0x1p+32f : x;
    float r = __builtin_amdgcn_sqrtf(xs);
    const float rm = __int_as_float(__float_as_int(r) - 1);
    const float rp = __int_as_float(__float_as_int(r) + 1);
    const float em = __builtin_fmaf(-rm, r, xs);
    const float ep = __builtin_fmaf(-rp, r, xs);
    r = (em <= 0.0f) ? rm : r;
    r = (ep > 0.0f) ? rp : r;
    r = tiny ? r * 0x1p-16f : r;
    // +-0, +inf and NaN: IEEE results
    return (xs == 0.0f || !(xs < __builtin_inff())) ? __builtin_amdgcn_sqrtf(x) : r;
}

// Wave64 helpers (gfx950: wavefront = 64 lanes).
__device__ inline int lane_id() { return (int)__lane_id(); }

}  // namespace ecc
