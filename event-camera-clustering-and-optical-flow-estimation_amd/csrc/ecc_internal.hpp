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
