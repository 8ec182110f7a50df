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
//   mask[q]    : u32 bitmask of the group's slices that touched q   (atomicOr)
//   M[j][q]    : max t at q within slice j of the group              (atomicMax, int64)
//   B[q]       : SAE before the group (the caller's `sae` buffer, updated in place)
// so V(q,s) = M[j*][q] with j* = highest set bit of mask[q] & ((2 << j) - 1), else B[q]
// (timestamps are non-decreasing, so max == last writer; a device check enforces it).
// Two ping-pong buffer sets let one launch build group g while folding group g-1 into B, and
// the next launch test group g while resetting group g-1's entries (sparse, per event), so
// the buffers are clean between calls without full-image memsets:
//   K_build(g):  build(g) + fold(g-1)          K_test(g): arc(g) + clean(g-1)
// => 2 launches per 32 slices (524288 events) instead of 2 per slice.
//
// Arc test: the reference loop "exists i,s: T[c(i)]>=T[c(i-1)], T[c(i+s-1)]>=T[c(i+s)], and
// every T outside the streak < min(streak)" reduces to "the s largest values are strictly
// greater than the rest and occupy a contiguous arc" (the two >= conditions are implied).
// With cnt[j] = #{k : T[k] > T[j]}, the top-s set is {j : cnt[j] < s}; it is strictly
// separated iff its size is s.  This branch-free form is exact; tests/test_gpu_parity.py
// checks it against the literal loop in oracle/oracle.cpp.
// Algorithmic bytes: 12 B/event in (xy + t) + 1 B/event out (corner flag).
#include "ecc_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr int kGroup = 32;  // slices per group (mask bits)
constexpr int64_t kEmptyT = INT64_MIN;

struct CornerGeom {
    int W, H, S, margin, border_mode, first_detect;
    int64_t n, n_slices;
};

struct GroupBufs {
    uint32_t *mask;  // [H*W]
    int64_t *M;      // [kGroup][H*W]
};

__constant__ int8_t c3dy[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
__constant__ int8_t c3dx[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
__constant__ int8_t c4dy[20] = {0, 1, 2, 3, 4, 4, 4, 3, 2, 1, 0, -1, -2, -3, -4, -4, -4, -3, -2, -1};
__constant__ int8_t c4dx[20] = {4, 4, 3, 2, 1, 0, -1, -2, -3, -4, -4, -4, -3, -2, -1, 0, 1, 2, 3, 4};

__device__ __forceinline__ bool is_border(int x, int y, const CornerGeom &g) {
    return x < g.margin || x >= g.W - g.margin || y < g.margin || y >= g.H - g.margin;
}

// Build group `grp` (events of its slices) into buffer set `cur`; fold group grp-1 (buffer
// set `prv`) into B.  One thread per event slot of a group.
__global__ void __launch_bounds__(kThreads)
sae_build_kernel(const uint32_t *__restrict__ xy, const int64_t *__restrict__ t, CornerGeom g,
                 int64_t grp, GroupBufs cur, GroupBufs prv, int64_t *__restrict__ B,
                 int32_t *__restrict__ first_border, int32_t *__restrict__ err) {
    const int64_t slot = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const int64_t grp_events = (int64_t)kGroup * g.S;
    const int64_t HW = (int64_t)g.H * g.W;
    // build(grp)
    {
        const int64_t e = grp * grp_events + slot;
        if (e < g.n) {
            const uint32_t v = xy[e];
            const int64_t te = t[e];
            if (e > 0 && t[e - 1] > te) *err = 1;
            const int x = ecc::xy_x(v), y = ecc::xy_y(v);
            const int64_t s = e / g.S;
            const int j = (int)(s - grp * kGroup);
            if (x < g.W && y < g.H) {
                const int64_t q = (int64_t)y * g.W + x;
                atomicOr(&cur.mask[q], 1u << j);
                atomicMax(reinterpret_cast<long long *>(&cur.M[(int64_t)j * HW + q]), (long long)te);
            }
            if (g.border_mode == 1 && is_border(x, y, g))
                atomicMin(&first_border[s], (int32_t)(e - s * g.S));
        }
    }
    // fold(grp - 1): the last writer of each pixel of the previous group updates B
    if (grp > 0) {
        const int64_t e = (grp - 1) * grp_events + slot;
        if (e < g.n) {
            const uint32_t v = xy[e];
            const int x = ecc::xy_x(v), y = ecc::xy_y(v);
            if (x < g.W && y < g.H) {
                const int64_t q = (int64_t)y * g.W + x;
                const int j = (int)(e / g.S - (grp - 1) * kGroup);
                const uint32_t mk = prv.mask[q];
                if (31 - __clz(mk) == j) {
                    const int64_t te = t[e];
                    if (prv.M[(int64_t)j * HW + q] == te) B[q] = te;
                }
            }
        }
    }
}

// V(q, j): SAE value at pixel q as seen by slice j of the current group.
__device__ __forceinline__ int64_t sae_at(int64_t q, uint32_t below, const GroupBufs &cur,
                                          const int64_t *__restrict__ B, int64_t HW) {
    const uint32_t mk = cur.mask[q] & below;
    if (mk) return cur.M[(int64_t)(31 - __clz(mk)) * HW + q];
    return B[q];
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

// Arc test for group `grp` (buffer set cur) + sparse reset of group grp-1 (buffer set prv).
__global__ void __launch_bounds__(kThreads)
arc_test_kernel(const uint32_t *__restrict__ xy, const int64_t *__restrict__ t, CornerGeom g,
                int64_t grp, GroupBufs cur, GroupBufs prv, const int64_t *__restrict__ B,
                const int32_t *__restrict__ first_border, uint8_t *__restrict__ flags) {
    const int64_t slot = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const int64_t grp_events = (int64_t)kGroup * g.S;
    const int64_t HW = (int64_t)g.H * g.W;
    {
        const int64_t e = grp * grp_events + slot;
        if (e < g.n) {
            const uint32_t v = xy[e];
            const int x = ecc::xy_x(v), y = ecc::xy_y(v);
            const int64_t s = e / g.S;
            const int j = (int)(s - grp * kGroup);
            bool test = s >= g.first_detect && !is_border(x, y, g);
            if (test && g.border_mode == 1) test = (e - s * g.S) < first_border[s];
            uint8_t corner = 0;
            if (test) {
                const uint32_t below = (j == 31) ? 0xffffffffu : ((2u << j) - 1u);
                const int64_t q0 = (int64_t)y * g.W + x;
                int64_t v3[16];
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    v3[k] = sae_at(q0 + (int64_t)c3dy[k] * g.W + c3dx[k], below, cur, B, HW);
                if (arc_streak<16, 3, 6>(v3)) {
                    int64_t v4[20];
#pragma unroll
                    for (int k = 0; k < 20; ++k)
                        v4[k] = sae_at(q0 + (int64_t)c4dy[k] * g.W + c4dx[k], below, cur, B, HW);
                    corner = arc_streak<20, 4, 8>(v4) ? 1 : 0;
                }
            }
            flags[e] = corner;
        }
    }
    if (grp > 0) {
        const int64_t e = (grp - 1) * grp_events + slot;
        if (e < g.n) {
            const uint32_t v = xy[e];
            const int x = ecc::xy_x(v), y = ecc::xy_y(v);
            if (x < g.W && y < g.H) {
                const int64_t q = (int64_t)y * g.W + x;
                const int j = (int)(e / g.S - (grp - 1) * kGroup);
                prv.mask[q] = 0u;
                prv.M[(int64_t)j * HW + q] = kEmptyT;
            }
        }
    }
}

// Final fold / final reset of the last group (separate launches: fold reads what reset writes).
__global__ void __launch_bounds__(kThreads)
sae_tail_kernel(const uint32_t *__restrict__ xy, const int64_t *__restrict__ t, CornerGeom g,
                int64_t grp, GroupBufs buf, int64_t *__restrict__ B, int reset) {
    const int64_t slot = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const int64_t e = grp * (int64_t)kGroup * g.S + slot;
    if (e >= g.n) return;
    const int64_t HW = (int64_t)g.H * g.W;
    const uint32_t v = xy[e];
    const int x = ecc::xy_x(v), y = ecc::xy_y(v);
    if (x >= g.W || y >= g.H) return;
    const int64_t q = (int64_t)y * g.W + x;
    const int j = (int)(e / g.S - grp * kGroup);
    if (!reset) {
        const uint32_t mk = buf.mask[q];
        if (31 - __clz(mk) == j) {
            const int64_t te = t[e];
            if (buf.M[(int64_t)j * HW + q] == te) B[q] = te;
        }
    } else {
        buf.mask[q] = 0u;
        buf.M[(int64_t)j * HW + q] = kEmptyT;
    }
}

__global__ void fill_i64_kernel(int64_t *__restrict__ p, int64_t n, int64_t v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
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

// Dedicated, always-clean group buffers: [2][mask HW u32] + [2][G][HW] int64 (+ first_border).
struct CornerState {
    int W = 0, H = 0;
    void *mem = nullptr;
    size_t bytes = 0;
    GroupBufs set[2];
    int32_t *first_border = nullptr;
    int64_t fb_cap = 0;
};

CornerState *state_of(ecc_ctx *ctx);

}  // namespace

// one CornerState per context (kept outside ecc_ctx to keep the header light)
#include <map>
#include <mutex>
static std::mutex g_state_mu;
static std::map<const ecc_ctx *, CornerState *> g_states;

namespace {
CornerState *state_of(ecc_ctx *ctx) {
    std::lock_guard<std::mutex> lk(g_state_mu);
    auto it = g_states.find(ctx);
    if (it != g_states.end()) return it->second;
    auto *s = new CornerState();
    g_states[ctx] = s;
    return s;
}

int corner_state_reserve(ecc_ctx *ctx, CornerState *st, int W, int H, int64_t n_slices,
                         hipStream_t s) {
    if (st->W != W || st->H != H || !st->mem) {
        if (st->mem) {
            ECC_CHECK_HIP(ctx, hipDeviceSynchronize(), "sync(corner state)");
            hipFree(st->mem);
            st->mem = nullptr;
        }
        const size_t HW = (size_t)W * H;
        const size_t mask_b = ecc::align_up(HW * 4, 256);
        const size_t m_b = ecc::align_up(HW * 8 * kGroup, 256);
        const size_t bytes = 2 * mask_b + 2 * m_b;
        hipError_t e = hipMalloc(&st->mem, bytes);
        if (e != hipSuccess) { st->mem = nullptr; ecc::hip_fail(ctx, e, "hipMalloc(corner state)"); return ECC_ERR_NOMEM; }
        char *p = static_cast<char *>(st->mem);
        for (int b = 0; b < 2; ++b) {
            st->set[b].mask = reinterpret_cast<uint32_t *>(p + b * mask_b);
            st->set[b].M = reinterpret_cast<int64_t *>(p + 2 * mask_b + b * m_b);
        }
        ECC_CHECK_HIP(ctx, hipMemsetAsync(p, 0, 2 * mask_b, s), "memset(masks)");
        {
            ECC_TIMED(ctx, s, "fill_i64_kernel");
            hipLaunchKernelGGL(fill_i64_kernel, dim3(2048), dim3(256), 0, s,
                               reinterpret_cast<int64_t *>(p + 2 * mask_b), (int64_t)(2 * m_b / 8), kEmptyT);
        }
        ECC_CHECK_LAUNCH(ctx, "fill(M)");
        st->W = W;
        st->H = H;
        st->bytes = bytes;
    }
    if (n_slices > st->fb_cap) {
        if (st->first_border) {
            ECC_CHECK_HIP(ctx, hipDeviceSynchronize(), "sync(first_border)");
            hipFree(st->first_border);
        }
        st->fb_cap = ecc::align_up((size_t)n_slices, 4096);
        hipError_t e = hipMalloc(&st->first_border, st->fb_cap * 4);
        if (e != hipSuccess) { st->first_border = nullptr; st->fb_cap = 0; return ECC_ERR_NOMEM; }
    }
    return ECC_OK;
}
}  // namespace

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
    if (cfg->slice_events < 1 || (cfg->border_mode != 0 && cfg->border_mode != 1))
        return ECC_ERR_INVALID;
    hipStream_t s = ecc::as_stream(stream);
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    ECC_CHECK_HIP(ctx, hipMemsetAsync(ctx->flags, 0, 4, s), "memset(err flag)");
    if (n == 0) return ECC_OK;
    CornerGeom g{cfg->width, cfg->height, cfg->slice_events, cfg->margin, cfg->border_mode,
                 cfg->first_detect_slice, n, (n + cfg->slice_events - 1) / cfg->slice_events};
    CornerState *st = state_of(ctx);
    int rc = corner_state_reserve(ctx, st, g.W, g.H, g.n_slices, s);
    if (rc) return rc;
    if (g.border_mode == 1)
        ECC_CHECK_HIP(ctx, hipMemsetAsync(st->first_border, 0x7f, g.n_slices * 4, s), "memset(fb)");
    const int64_t grp_events = (int64_t)kGroup * g.S;
    const int64_t n_groups = (n + grp_events - 1) / grp_events;
    const int64_t blocks64 = (std::min<int64_t>(grp_events, n) + kThreads - 1) / kThreads;
    if (blocks64 > INT32_MAX) return ECC_ERR_INVALID;
    const dim3 grid((unsigned)blocks64);
    for (int64_t gi = 0; gi < n_groups; ++gi) {
        const GroupBufs cur = st->set[gi & 1], prv = st->set[(gi + 1) & 1];
        {
            ECC_TIMED(ctx, s, "sae_build_kernel");
            hipLaunchKernelGGL(sae_build_kernel, grid, dim3(kThreads), 0, s, xy, t, g, gi, cur, prv,
                               sae, st->first_border, ctx->flags);
        }
        {
            ECC_TIMED(ctx, s, "arc_test_kernel");
            hipLaunchKernelGGL(arc_test_kernel, grid, dim3(kThreads), 0, s, xy, t, g, gi, cur, prv,
                               (const int64_t *)sae, (const int32_t *)st->first_border, corner_flags);
        }
    }
    const int64_t last = n_groups - 1;
    {
        ECC_TIMED(ctx, s, "sae_tail_kernel");
        hipLaunchKernelGGL(sae_tail_kernel, grid, dim3(kThreads), 0, s, xy, t, g, last,
                           st->set[last & 1], sae, 0);
    }
    {
        ECC_TIMED(ctx, s, "sae_tail_kernel");
        hipLaunchKernelGGL(sae_tail_kernel, grid, dim3(kThreads), 0, s, xy, t, g, last,
                           st->set[last & 1], sae, 1);
    }
    ECC_CHECK_LAUNCH(ctx, "fast_detect");
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
