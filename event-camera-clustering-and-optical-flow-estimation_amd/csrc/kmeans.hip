// k-means over 2-D event points.
//
// Reference: KM/assign_to_centers.cl — assign_to_centers (:1-34: nearest of 8 centres by
// length((cx-x, cy-y, 0)), strict `<` from threshold 50, uchar 255 = none),
// assign_data_cluster (:36-119: atomic scatter into 8 bins of 2048), reduction_scalar
// (:121-140: 1024-wide tree sums), and the host loop KM/assign_to_centers2.c:184-548
// (buffers re-created every pass, blocking reads, goto restart).
//
// MI355X design ("fixed" mode, Appendix A Q7-Q10):
//   * one fused kernel per iteration: 16-B loads of 4 packed-u16 points per lane, centroids in
//     LDS (broadcast reads), assignment, and per-wave LDS accumulators updated with 64-bit LDS
//     atomics — no scatter pass, no bins, no host round trip;
//   * partial sums are INTEGERS (pixel coordinates): count<<40 | sum_x and sum_y per cluster,
//     flushed with one 64-bit global atomic per (WG, cluster, field) — exact, so the result is
//     independent of reduction order and bit-identical to the fp64 oracle;
//   * a 1-wave update kernel computes c = (float)(sum/n) in fp64, the max shift, and a
//     device-side `done` flag that makes the remaining queued iterations no-ops (no host
//     sync per iteration).
// Assignment arithmetic (canonical, shared with oracle/oracle.cpp assign_one): fp32
// d2 = dx*dx + dy*dy (no FMA contraction), correctly rounded sqrt (ecc::sqrt_rn), the
// reference's first-minimum rule; sqrt only where d2 improves (see assign_point).
// Algorithmic bytes: 4 B/point/iteration (packed u16 xy) + 1 B/point for the final labels.
#include "ecc_internal.hpp"

#ifndef ECC_KM_LUT_WG_PER_CU
#define ECC_KM_LUT_WG_PER_CU 5
#endif
#ifndef ECC_KM_LAB_WG_PER_CU
#define ECC_KM_LAB_WG_PER_CU 6
#endif
#ifndef ECC_KM_LUT_UNROLL
#define ECC_KM_LUT_UNROLL 4
#endif
#ifndef ECC_KM_MFMA_BLOCKS
#define ECC_KM_MFMA_BLOCKS 1  // matrix engine: 64-pair blocks per trip
#endif
#ifndef ECC_KM_MFMA_WAVES
#define ECC_KM_MFMA_WAVES 4  // matrix engine 3: waves/SIMD the register budget is held to
#endif
#ifndef ECC_KM_ACC_SUB
#define ECC_KM_ACC_SUB 4
#endif

#include <cmath>

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kMaxK = 64;
constexpr int kMaxGrid = 2048;
constexpr int kMaxGridPts = 4096;  // label-image point passes
constexpr int kFastMaxK = 32;
constexpr int kImgSide = 2048;  // label image side (see kmeans_step_kernel)
constexpr int kFlushBatches = 2;  // packed u64 slot fields stay exact for < 512 points

struct KmState {
    int32_t done;
    int32_t iters;
};

// assign_to_centers (KM/assign_to_centers.cl:10-27): the FIRST centre whose fp32 distance
// sqrtf(dx*dx + dy*dy) is strictly below the running best (initially the threshold).  The
// sqrt is only evaluated when d2 drops below the pruning bound pb (a centre with d2 >= pb has
// sqrt >= the current best, so it can never be strictly closer) — about ln(k)+1 square roots
// per point instead of k, with exactly the reference's selection.
__device__ __forceinline__ uint32_t assign_point(float px, float py, const float2 *__restrict__ c,
                                                 int k, float thr) {
    uint32_t best = 255u;
    float best_s = thr, pb = __builtin_inff();
    for (int i = 0; i < k; ++i) {
        const float2 ci = c[i];
        const float dx = __fsub_rn(ci.x, px), dy = __fsub_rn(ci.y, py);
        const float d2 = __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy));
        if (d2 < pb) {
            pb = d2;
            const float s = ecc::sqrt_rn(d2);
            if (s < best_s) { best_s = s; best = (uint32_t)i; }
        }
    }
    return best;
}

// Segment geometry: segment s holds cnt(s) points at base s*stride.
struct Segs {
    const int32_t *counts;  // nullable
    int64_t n_segs, stride, n_dense;
    __device__ __forceinline__ int64_t count(int64_t s) const {
        if (counts) return counts[s];
        const int64_t r = n_dense - s * stride;
        return r < stride ? r : stride;
    }
};

template <bool kAccumulate>
__global__ void __launch_bounds__(kThreads)
kmeans_xy16_kernel(const uint32_t *__restrict__ xy, Segs segs, const float *__restrict__ cent,
                   int k, float thr, unsigned long long *__restrict__ acc,
                   const KmState *__restrict__ st, uint8_t *__restrict__ labels) {
    if (kAccumulate && st->done) return;
    __shared__ float2 c_lds[kMaxK];
    __shared__ unsigned long long a_xc[kWaves][kMaxK];
    __shared__ unsigned long long a_y[kWaves][kMaxK];
    const int tid = threadIdx.x, wave = tid >> 6;
    if (tid < k) c_lds[tid] = make_float2(cent[2 * tid], cent[2 * tid + 1]);
    if (kAccumulate) {
        for (int i = tid; i < kWaves * kMaxK; i += kThreads) {
            (&a_xc[0][0])[i] = 0ull;
            (&a_y[0][0])[i] = 0ull;
        }
    }
    __syncthreads();
    const bool vec_ok = (segs.stride & 3) == 0;
    for (int64_t s = blockIdx.x; s < segs.n_segs; s += gridDim.x) {
        const int64_t cnt = segs.count(s);
        const int64_t base = s * segs.stride;
        for (int64_t j = 4 * tid; j < cnt; j += 4 * kThreads) {
            uint32_t v[4];
            if (vec_ok && j + 3 < cnt) {
                const uint4 q = *reinterpret_cast<const uint4 *>(xy + base + j);
                v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = (j + e < cnt) ? xy[base + j + e] : 0u;
            }
            uint32_t lab[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const bool ok = j + e < cnt;
                const int x = ecc::xy_x(v[e]), y = ecc::xy_y(v[e]);
                lab[e] = ok ? assign_point((float)x, (float)y, c_lds, k, thr) : 255u;
                if (kAccumulate && lab[e] != 255u) {
                    atomicAdd(&a_xc[wave][lab[e]], (1ull << 40) | (unsigned long long)x);
                    atomicAdd(&a_y[wave][lab[e]], (unsigned long long)y);
                }
            }
            if (labels) {
                if (j + 3 < cnt && ((base + j) & 3) == 0) {
                    const uint32_t pk = lab[0] | (lab[1] << 8) | (lab[2] << 16) | (lab[3] << 24);
                    *reinterpret_cast<uint32_t *>(labels + base + j) = pk;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (j + e < cnt) labels[base + j + e] = (uint8_t)lab[e];
                }
            }
        }
    }
    if (kAccumulate) {
        __syncthreads();
        if (tid < k) {
            unsigned long long xc = 0, ys = 0;
#pragma unroll
            for (int w = 0; w < kWaves; ++w) { xc += a_xc[w][tid]; ys += a_y[w][tid]; }
            const unsigned long long n_pts = xc >> 40;
            if (n_pts) {
                atomicAdd(&acc[3 * tid + 0], n_pts);
                atomicAdd(&acc[3 * tid + 1], xc & ((1ull << 40) - 1));
                atomicAdd(&acc[3 * tid + 2], ys);
            }
        }
    }
}

// ---- fast path for k <= 32: compile-time K, centroids in scalar registers -----------------
// Exact argmin without a square root per centre: sqrt_rn is monotone, so the reference's
// choice (first centre with the smallest sqrt_rn(d2), if below thr) is the first index of the
// smallest d2 — unless an EARLIER centre has a larger d2 that rounds to the same square root.
// That needs d2_i / d2_min <= ((1 + 2^-24) / (1 - 2^-24))^2 < 1 + 2^-22; the single pass
// keeps m_prev = min d2 over the indices before the winner and takes the exact
// sqrt-per-centre loop (assign_point's rule) only when m_prev <= m * (1 + 2^-20).
template <int K>
__device__ __forceinline__ uint32_t assign_fast(float px, float py, const float (&cx)[K],
                                                const float (&cy)[K], float thr) {
    float m = __builtin_inff(), m_prev = __builtin_inff();
    int ia = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const float dx = __fsub_rn(cx[i], px), dy = __fsub_rn(cy[i], py);
        const float d2 = __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy));
        const bool lt = d2 < m;
        m_prev = lt ? m : m_prev;
        ia = lt ? i : ia;
        m = lt ? d2 : m;
    }
    if (__builtin_expect(m_prev <= __fmul_rn(m, 1.0f + 0x1p-20f), 0)) {
        uint32_t best = 255u;
        float best_s = thr;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const float dx = __fsub_rn(cx[i], px), dy = __fsub_rn(cy[i], py);
            const float s = ecc::sqrt_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)));
            if (s < best_s) { best_s = s; best = (uint32_t)i; }
        }
        return best;
    }
    return ecc::sqrt_rn(m) < thr ? (uint32_t)ia : 255u;
}

// The f32 engine's screen on the packed fp32 ALU (v_pk_add/mul/fma_f32), two centres per op.
// d2' = fma(dx, dx, dy*dy) (dx, dy exact as the reference's) is within 2 ulps of the reference's
// d2 = dx*dx + dy*dy; keys (bits(d2') & ~31) | i order the centres by 32-ulp bucket, then index,
// and one v_min + one v_med3 per centre keep the smallest two keys.  When the second-best key
// lies two or more buckets above the best (>= 33 ulps, i.e. > 2^-19 relative, beyond both the
// d2' error and assign_fast's 2^-20 square-root tie band), the best index is the reference's
// unique choice: the first centre with the smallest sqrt_rn(d2).  Its exact d2 then meets the
// threshold as d2 < thr2 (thr2 = the first float whose correctly rounded sqrt is >= thr, found
// by bisection on the host: sqrt_rn is monotone).  Closer calls, inf and NaN take assign_fast.
typedef float f32x2 __attribute__((ext_vector_type(2)));

// median of three: with a <= b the two smallest of {a, b, c} are min(a, c) and med3(a, b, c).
// The min/max idiom is not matched to v_med3_u32 for register operands, hence the asm.
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// One point against the centres two at a time: the packed operands are a centre PAIR (two
// consecutive scalar registers, no copies) and the point broadcast, so the screen costs
// 2 packed + 3 scalar (v_and_or, v_min, v_med3) instructions per centre and point.
template <int K>
__device__ __forceinline__ void screen_point(float px, float py, const float (&cx)[K], const float (&cy)[K],
                                             uint32_t &k1, uint32_t &k2) {
    const f32x2 pxx = {px, px}, pyy = {py, py};
    k1 = 0xffffffffu;
    k2 = 0xffffffffu;
#pragma unroll
    for (int i = 0; i < K; i += 2) {
        const f32x2 dx = (f32x2){cx[i], cx[i + 1]} - pxx, dy = (f32x2){cy[i], cy[i + 1]} - pyy;
        const f32x2 d2 = __builtin_elementwise_fma(dx, dx, dy * dy);
        const uint32_t ka = (__float_as_uint(d2.x) & ~31u) | (uint32_t)i;
        const uint32_t kb = (__float_as_uint(d2.y) & ~31u) | (uint32_t)(i + 1);
        k2 = umed3(k1, k2, ka);
        k1 = min(k1, ka);
        k2 = umed3(k1, k2, kb);
        k1 = min(k1, kb);
    }
}

template <int K>
__device__ __forceinline__ uint32_t finish_point(float px, float py, uint32_t k1, uint32_t k2,
                                                 const float (&cx)[K], const float (&cy)[K],
                                                 const float2 *__restrict__ s_c, float thr, float thr2) {
    constexpr uint32_t kInfBucket = 0x7F800000u >> 5;
    if (__builtin_expect((k1 >> 5) < kInfBucket && (k2 >> 5) > (k1 >> 5) + 1u, 1)) {
        const float2 c = s_c[k1 & 31u];
        const float dx = __fsub_rn(c.x, px), dy = __fsub_rn(c.y, py);
        return __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)) < thr2 ? (k1 & 31u) : 255u;
    }
    return assign_fast<K>(px, py, cx, cy, thr);
}

template <int K>
__device__ __forceinline__ void assign_pair(float2 p0, float2 p1, const float (&cx)[K], const float (&cy)[K],
                                            const float2 *__restrict__ s_c, float thr, float thr2, uint32_t &l0,
                                            uint32_t &l1) {
    // the two points' screens interleaved centre pair by centre pair: two independent min/med3
    // chains per step (one point's chain alone leaves the VALU waiting on its own results)
    uint32_t a1 = 0xffffffffu, a2 = 0xffffffffu, b1 = 0xffffffffu, b2 = 0xffffffffu;
    {
        const f32x2 pxa = {p0.x, p0.x}, pya = {p0.y, p0.y}, pxb = {p1.x, p1.x}, pyb = {p1.y, p1.y};
#pragma unroll
        for (int i = 0; i < K; i += 2) {
            const f32x2 ccx = {cx[i], cx[i + 1]}, ccy = {cy[i], cy[i + 1]};
            const f32x2 dxa = ccx - pxa, dya = ccy - pya, dxb = ccx - pxb, dyb = ccy - pyb;
            const f32x2 da = __builtin_elementwise_fma(dxa, dxa, dya * dya);
            const f32x2 db = __builtin_elementwise_fma(dxb, dxb, dyb * dyb);
            const uint32_t ka0 = (__float_as_uint(da.x) & ~31u) | (uint32_t)i;
            const uint32_t kb0 = (__float_as_uint(db.x) & ~31u) | (uint32_t)i;
            const uint32_t ka1 = (__float_as_uint(da.y) & ~31u) | (uint32_t)(i + 1);
            const uint32_t kb1 = (__float_as_uint(db.y) & ~31u) | (uint32_t)(i + 1);
            a2 = umed3(a1, a2, ka0);
            b2 = umed3(b1, b2, kb0);
            a1 = min(a1, ka0);
            b1 = min(b1, kb0);
            a2 = umed3(a1, a2, ka1);
            b2 = umed3(b1, b2, kb1);
            a1 = min(a1, ka1);
            b1 = min(b1, kb1);
        }
    }
    l0 = finish_point<K>(p0.x, p0.y, a1, a2, cx, cy, s_c, thr, thr2);
    l1 = finish_point<K>(p1.x, p1.y, b1, b2, cx, cy, s_c, thr, thr2);
}

// assign_fast's arithmetic, step for step, with the centres read from LDS inside a rolled loop
// (the asm barrier keeps the compiler from hoisting them into registers).  Used by the
// label-image passes for points outside the image only; tests/test_gpu_parity.py covers both
// the outside points and the near-tie rule.
template <int K>
__device__ __forceinline__ uint32_t assign_lds(float px, float py, const float *s_cx, const float *s_cy, float thr) {
    float m = __builtin_inff(), m_prev = __builtin_inff();
    int ia = 0;
#pragma unroll 1
    for (int i = 0; i < K; ++i) {
        asm volatile("" ::: "memory");
        const float dx = __fsub_rn(s_cx[i], px), dy = __fsub_rn(s_cy[i], py);
        const float d2 = __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy));
        const bool lt = d2 < m;
        m_prev = lt ? m : m_prev;
        ia = lt ? i : ia;
        m = lt ? d2 : m;
    }
    if (m_prev <= __fmul_rn(m, 1.0f + 0x1p-20f)) {
        uint32_t best = 255u;
        float best_s = thr;
#pragma unroll 1
        for (int i = 0; i < K; ++i) {
            asm volatile("" ::: "memory");
            const float dx = __fsub_rn(s_cx[i], px), dy = __fsub_rn(s_cy[i], py);
            const float s = ecc::sqrt_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)));
            if (s < best_s) { best_s = s; best = (uint32_t)i; }
        }
        return best;
    }
    return ecc::sqrt_rn(m) < thr ? (uint32_t)ia : 255u;
}

__device__ __forceinline__ uint64_t lanes_below_mask(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

__device__ __forceinline__ float uniform_f32(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}


// Replicated accumulators: the per-WG flush goes to replica blockIdx % n_copies, which spreads
// the same-address global atomics; the update kernel sums the replicas.
constexpr int kAccStride = 3 * kMaxK;
constexpr int kAccCopies = 16;  // replicas: 256 pixel-pass WGs -> 16 atomics per address

// One Lloyd pass (kAccumulate) or the final labelling.  Accumulation: every point adds
// (1 << 52) | (x << 26) | y to its cluster's u64 slot of its WAVE in LDS with one no-return
// ds_add_u64 (64 lanes spread over <= K addresses).  The packed fields are exact while a slot
// receives < 512 points of < 2^16 per coordinate, so each wave unpacks its slots into u64 lane
// totals (lane c = cluster c) every kFlushBatches = 2 batches of 256 points.  One global u64
// atomic per (WG, cluster, field) at the end, spread over n_copies accumulator replicas.
// (Fusing the update into the last-arriving workgroup was measured slower: the device-scope
// release every workgroup needs before arriving costs more than the separate 1-wave launch.)
template <int K, bool kAccumulate>
__global__ void __launch_bounds__(kThreads)
kmeans_fast_kernel(const uint32_t *__restrict__ xy, Segs segs, const float *__restrict__ cent, int k, float thr,
                   unsigned long long *acc, int n_copies, const KmState *st, uint8_t *__restrict__ labels) {
    if (kAccumulate && st->done) return;
    __shared__ unsigned long long slot[kWaves][K];
    __shared__ unsigned long long w_acc[3][K];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    // the centroids live in scalar registers
    float cx[K], cy[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        cx[i] = uniform_f32(i < k ? cent[2 * i] : __builtin_inff());
        cy[i] = uniform_f32(i < k ? cent[2 * i + 1] : __builtin_inff());
    }
    if (kAccumulate) {
        for (int i = tid; i < 3 * K; i += kThreads) (&w_acc[0][0])[i] = 0ull;
        if (lane < K) slot[wave][lane] = 0ull;
        __syncthreads();
    }
    unsigned long long tn = 0, tx = 0, ty = 0;  // lane c: wave totals of cluster c
    int batches = 0;
    auto flush = [&]() {  // the wave's own slots: LDS ops of one wave complete in order
        if (lane < K) {
            const unsigned long long w = slot[wave][lane];
            slot[wave][lane] = 0ull;
            tn += w >> 52;
            tx += (w >> 26) & ((1ull << 26) - 1);
            ty += w & ((1ull << 26) - 1);
        }
    };
    for (int64_t s = blockIdx.x; s < segs.n_segs; s += gridDim.x) {
        const int64_t cnt = segs.count(s);
        const int64_t base = s * segs.stride;
        // Two 4-point batches per lane per trip: both loads and all eight label gathers are in
        // flight before the first LDS add, halving the dependent load -> gather -> add rounds.
        // the segment through a buffer view rounded up to 16 B (inside the allocation's last 16-B
        // block; points past cnt are masked): unconditional 16-B loads (4-B alignment suffices)
        const __amdgpu_buffer_rsrc_t vs = ecc::buffer_view(xy + base, (uint32_t)((cnt * 4 + 15) & ~15ll));
        for (int64_t j0 = 0; j0 < cnt; j0 += 8 * kThreads) {  // uniform trip count per WG
            uint32_t v[8], lab[8];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const uint4 q = ecc::buffer_load_u128(vs, (uint32_t)tid * 16u, (uint32_t)(j0 + u * 4 * kThreads) * 4u);
                v[4 * u] = q.x; v[4 * u + 1] = q.y; v[4 * u + 2] = q.z; v[4 * u + 3] = q.w;
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int64_t j = j0 + u * 4 * kThreads + 4 * tid;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t w = v[4 * u + e];
                    const uint32_t x = (uint32_t)ecc::xy_x(w), y = (uint32_t)ecc::xy_y(w);
                    uint32_t l;
                    if (j + e >= cnt) l = 255u;
                    else l = assign_fast<K>((float)x, (float)y, cx, cy, thr);
                    lab[4 * u + e] = l;
                }
            }
            if (kAccumulate) {
                // Runs of equal labels are summed in registers first: neighbouring events mostly share
                // a cluster, and LDS atomics from many lanes to one slot serialise.
                uint32_t cl = lab[0];
                unsigned long long run = 0ull;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const unsigned long long pk = (1ull << 52) | ((unsigned long long)ecc::xy_x(v[e]) << 26) |
                                                  (unsigned long long)ecc::xy_y(v[e]);
                    if (lab[e] != cl) {
                        if (cl < (uint32_t)K) atomicAdd(&slot[wave][cl], run);
                        cl = lab[e];
                        run = 0ull;
                    }
                    run += pk;
                }
                if (cl < (uint32_t)K) atomicAdd(&slot[wave][cl], run);
                batches += 2;
                if (batches >= kFlushBatches) {
                    flush();
                    batches = 0;
                }
            }
            if (labels) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int64_t j = j0 + u * 4 * kThreads + 4 * tid;
                    if (j + 3 < cnt && ((base + j) & 3) == 0) {
                        const uint32_t pk = lab[4 * u] | (lab[4 * u + 1] << 8) | (lab[4 * u + 2] << 16) |
                                            (lab[4 * u + 3] << 24);
                        *reinterpret_cast<uint32_t *>(labels + base + j) = pk;
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (j + e < cnt) labels[base + j + e] = (uint8_t)lab[4 * u + e];
                    }
                }
            }
        }
    }
    if (!kAccumulate) return;
    flush();
    if (lane < K && tn) {
        atomicAdd(&w_acc[0][lane], tn);
        atomicAdd(&w_acc[1][lane], tx);
        atomicAdd(&w_acc[2][lane], ty);
    }
    __syncthreads();
    if (tid < 3 * k) {
        const int f = tid / k, c = tid - f * k;
        const unsigned long long sum = w_acc[f][c];
        if (sum) atomicAdd(&acc[(int)(blockIdx.x % n_copies) * kAccStride + 3 * c + f], sum);
    }
}

// Final labels from the label image: one workgroup per segment, 16 points per lane, so a
// segment of up to 4096 points is ONE trip — its four 16-B loads, sixteen image gathers and four
// packed stores each in flight together (kmeans_fast_kernel's two-batch trips took two dependent
// load -> gather -> store rounds per bench segment of ~3150 points).  The loads are issued
// before the segment count arrives: a lane reads within the segment's stride (always readable),
// and only the stores are masked by the count.  Labels equal assign_fast's on the same points.
constexpr int kLabPer = 16;
template <int K>
__global__ void __launch_bounds__(kThreads)
kmeans_img_labels_kernel(const uint32_t *__restrict__ xy, Segs segs, const float *__restrict__ cent, int k,
                         float thr, const uint8_t *__restrict__ img, const uint32_t *__restrict__ img_wh,
                         uint8_t *__restrict__ labels) {
    __shared__ float s_cx[K], s_cy[K];
    const int tid = threadIdx.x;
    if (tid < K) {
        s_cx[tid] = tid < k ? cent[2 * tid] : __builtin_inff();
        s_cy[tid] = tid < k ? cent[2 * tid + 1] : __builtin_inff();
    }
    __syncthreads();
    const uint32_t img_w = img_wh[0], img_h = img_wh[1];
    for (int64_t s = blockIdx.x; s < segs.n_segs; s += gridDim.x) {
        const int64_t base = s * segs.stride;
        // readable extent: the whole stride (the next segment starts after it), except in the
        // last segment, whose buffer may end at its count
        const int64_t cnt = segs.count(s);
        const int64_t lim = s + 1 < segs.n_segs ? segs.stride : cnt;
        const __amdgpu_buffer_rsrc_t vs = ecc::buffer_view(xy + base, (uint32_t)((lim * 4 + 15) & ~15ll));
        for (int64_t j0 = 0; j0 < cnt; j0 += kLabPer * kThreads) {
            uint32_t v[kLabPer], lab[kLabPer];
#pragma unroll
            for (int u = 0; u < kLabPer / 4; ++u) {  // unconditional 16-B loads (see kmeans_fast_kernel)
                const uint4 q = ecc::buffer_load_u128(vs, (uint32_t)tid * 16u, (uint32_t)(j0 + u * 4 * kThreads) * 4u);
                v[4 * u] = q.x; v[4 * u + 1] = q.y; v[4 * u + 2] = q.z; v[4 * u + 3] = q.w;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < kLabPer / 4; ++u) {
                const int64_t j = j0 + u * 4 * kThreads + 4 * tid;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t w = v[4 * u + e];
                    const uint32_t x = (uint32_t)ecc::xy_x(w), y = (uint32_t)ecc::xy_y(w);
                    uint32_t l = 255u;
                    if (j + e < cnt) {
                        if (__builtin_expect(x < img_w && y < img_h, 1)) l = img[y * kImgSide + x];
                        else l = assign_lds<K>((float)x, (float)y, s_cx, s_cy, thr);
                    }
                    lab[4 * u + e] = l;
                }
            }
#pragma unroll
            for (int u = 0; u < kLabPer / 4; ++u) {
                const int64_t j = j0 + u * 4 * kThreads + 4 * tid;
                if (j + 3 < cnt && ((base + j) & 3) == 0) {
                    const uint32_t pk = lab[4 * u] | (lab[4 * u + 1] << 8) | (lab[4 * u + 2] << 16) |
                                        (lab[4 * u + 3] << 24);
                    *reinterpret_cast<uint32_t *>(labels + base + j) = pk;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (j + e < cnt) labels[base + j + e] = (uint8_t)lab[4 * u + e];
                }
            }
        }
    }
}

// The same labels with the label image staged in LDS (frames up to kLabLdsBytes, e.g. the
// 90 KB of 346x260): the image gathers of kmeans_img_labels_kernel hit a different cache line per
// lane, so its 7.7 M gathers were bound by the texture units' one-line-per-cycle tag lookups, not
// by HBM.  One 1024-lane workgroup per CU copies the image once from L2, then takes four segments
// per trip (256 lanes x 16 points each), loads issued before the counts arrive as above.
constexpr int kLabLdsThreads = 1024;
constexpr int kLabLdsBytes = 96 * 1024;
template <int K>
__global__ void __launch_bounds__(kLabLdsThreads)
kmeans_lds_labels_kernel(const uint32_t *__restrict__ xy, Segs segs, const float *__restrict__ cent, int k,
                         float thr, const uint8_t *__restrict__ img, const uint32_t *__restrict__ img_wh,
                         uint8_t *__restrict__ labels) {
    extern __shared__ uint8_t s_img[];  // [img_h][img_w], compact
    __shared__ float s_cx[K], s_cy[K];
    const int tid = threadIdx.x, sub = tid >> 8, t = tid & 255;
    if (tid < K) {
        s_cx[tid] = tid < k ? cent[2 * tid] : __builtin_inff();
        s_cy[tid] = tid < k ? cent[2 * tid + 1] : __builtin_inff();
    }
    const uint32_t img_w = img_wh[0], img_h = img_wh[1];
    // rows copied as words (row pitch img_w rounded up to 4), eight loads in flight per lane
    const uint32_t wq = (img_w + 3) >> 2, pitch = 4 * wq, n_words = wq * img_h;
    for (uint32_t i0 = 0; i0 < n_words; i0 += 8 * kLabLdsThreads) {
        uint32_t wv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {  // clamped word: unconditional loads, all eight in flight
            const uint32_t i0u = i0 + u * kLabLdsThreads + tid, i = i0u < n_words ? i0u : n_words - 1, r = i / wq;
            wv[u] = *reinterpret_cast<const uint32_t *>(img + r * kImgSide + 4 * (i - r * wq));
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t i = i0 + u * kLabLdsThreads + tid;
            if (i < n_words) reinterpret_cast<uint32_t *>(s_img)[i] = wv[u];
        }
    }
    __syncthreads();
    for (int64_t s0 = 4 * (int64_t)blockIdx.x; s0 < segs.n_segs; s0 += 4 * (int64_t)gridDim.x) {
        const int64_t s = s0 + sub;
        if (s >= segs.n_segs) continue;  // no barrier below
        const int64_t base = s * segs.stride;
        const int64_t cnt = segs.count(s);
        const int64_t lim = s + 1 < segs.n_segs ? segs.stride : cnt;
        // the segment through a buffer view rounded up to 16 B (inside the allocation's last 16-B
        // block; points past cnt are masked): one unconditional 16-B load per quad
        const __amdgpu_buffer_rsrc_t vs = ecc::buffer_view(xy + base, (uint32_t)((lim * 4 + 15) & ~15ll));
        for (int64_t j0 = 0; j0 < cnt; j0 += kLabPer * 256) {
            uint32_t v[kLabPer], lab[kLabPer];
#pragma unroll
            for (int u = 0; u < kLabPer / 4; ++u) {  // (16-B buffer loads need only 4-B alignment)
                const uint4 q = ecc::buffer_load_u128(vs, (uint32_t)t * 16u, (uint32_t)(j0 + u * 4 * 256) * 4u);
                v[4 * u] = q.x; v[4 * u + 1] = q.y; v[4 * u + 2] = q.z; v[4 * u + 3] = q.w;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < kLabPer / 4; ++u) {
                const int64_t j = j0 + u * 4 * 256 + 4 * t;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t w = v[4 * u + e];
                    const uint32_t x = (uint32_t)ecc::xy_x(w), y = (uint32_t)ecc::xy_y(w);
                    uint32_t l = 255u;
                    if (j + e < cnt) {
                        if (__builtin_expect(x < img_w && y < img_h, 1)) l = s_img[y * pitch + x];
                        else l = assign_lds<K>((float)x, (float)y, s_cx, s_cy, thr);
                    }
                    lab[4 * u + e] = l;
                }
            }
#pragma unroll
            for (int u = 0; u < kLabPer / 4; ++u) {
                const int64_t j = j0 + u * 4 * 256 + 4 * t;
                if (j + 3 < cnt && ((base + j) & 3) == 0) {
                    const uint32_t pk = lab[4 * u] | (lab[4 * u + 1] << 8) | (lab[4 * u + 2] << 16) |
                                        (lab[4 * u + 3] << 24);
                    *reinterpret_cast<uint32_t *>(labels + base + j) = pk;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (j + e < cnt) labels[base + j + e] = (uint8_t)lab[4 * u + e];
                }
            }
        }
    }
}

// float-input variant (reference data layout: interleaved float x,y): fp64 LDS + global
// atomics (order-dependent only at the 1e-16 relative level).
template <bool kAccumulate>
__global__ void __launch_bounds__(kThreads)
kmeans_f32_kernel(const float *__restrict__ xy, int64_t n, const float *__restrict__ cent, int k,
                  float thr, double *__restrict__ acc, const KmState *__restrict__ st,
                  uint8_t *__restrict__ labels) {
    if (kAccumulate && st->done) return;
    __shared__ float2 c_lds[kMaxK];
    __shared__ double a_s[kMaxK * 3];
    const int tid = threadIdx.x;
    if (tid < k) c_lds[tid] = make_float2(cent[2 * tid], cent[2 * tid + 1]);
    if (kAccumulate)
        for (int i = tid; i < kMaxK * 3; i += kThreads) a_s[i] = 0.0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * kThreads + tid; i < n; i += (int64_t)gridDim.x * kThreads) {
        const float2 p = reinterpret_cast<const float2 *>(xy)[i];
        const uint32_t lab = assign_point(p.x, p.y, c_lds, k, thr);
        if (labels) labels[i] = (uint8_t)lab;
        if (kAccumulate && lab != 255u) {
            atomicAdd(&a_s[3 * lab + 0], 1.0);
            atomicAdd(&a_s[3 * lab + 1], (double)p.x);
            atomicAdd(&a_s[3 * lab + 2], (double)p.y);
        }
    }
    if (kAccumulate) {
        __syncthreads();
        if (tid < 3 * k && a_s[tid] != 0.0) atomicAdd(&acc[tid], a_s[tid]);
    }
}

// ---- float points, k <= 32 (BASELINE config C3): two assignment engines, one accumulation ---------
// Vector engine: assign_fast<K> with the centres in scalar registers (exact, ~9 VALU per centre).
// Matrix engine: the distance part on the matrix cores.  v_mfma_f32_4x4x1f32 runs 16 blocks of
// 4x4x1; with block b = lanes 4b..4b+3, A_b[i] = -2 cx_{4g+i} (lane 4b+i) and B_b[j] = px of
// lane 4b+j, D_b[i][j] (lane 4b+j, register i) = C + A_b[i] B_b[j]: so two MFMAs per group g of
// four centres give every lane s_i = |c_i|^2 - 2 c_i.p for ITS OWN point (an fma chain, one
// rounding per step).  The argmin over s equals the argmin over d^2 = s + |p|^2 up to rounding:
// with E bounding the error of every s (E = 2^-21 (max|c|^2 + 2 max|cx| |px| + 2 max|cy| |py|),
// >= 4x the worst case of the three roundings), a gap between the best and second-best s above
// 2E + 2^-19 (|s_best| + |p|^2 + E) proves the best index is the unique d^2 minimum with no
// earlier centre inside assign_fast's square-root tie band; the winner's exact d^2 then decides
// the threshold.  Any closer call (and NaN input) takes the exact vector path.
// The argument assumes only that each of the three roundings of s is bounded — not the order in
// which the matrix core sums the products, nor how it treats subnormals: a relative bound does
// not hold for subnormal or flushed results, so E also carries an absolute term (kAbsRound)
// above three flushes to zero of a result below the smallest normal (3 x 2^-126).  Points whose
// gaps are that small (coordinates around 1e-19 and below) always take the exact path.
// Accumulation (both engines): per wave LDS slots, u32 count and fp64 sums (ds_add_f64: exact for
// integer-valued coordinates, 1e-16 relative otherwise); per workgroup one fp64 global atomic per
// (cluster, field) into one of n_copies replicas that the update kernel sums.
typedef float floatx4_t __attribute__((ext_vector_type(4)));
constexpr float kAbsRound = 0x1p-124f;  // > 3 x 2^-126: the absolute part of E (see above)

template <int K>
__device__ __forceinline__ uint32_t assign_mfma(float px, float py, const float (&ax)[K / 4], const float (&ay)[K / 4],
                                                const float (&c2)[K], float emul_c2, float emul_x, float emul_y,
                                                const float2 *__restrict__ s_c, const float (&cx)[K],
                                                const float (&cy)[K], float thr, float thr2) {
    floatx4_t d[K / 4];
#pragma unroll
    for (int g = 0; g < K / 4; ++g) {
        d[g] = floatx4_t{c2[4 * g], c2[4 * g + 1], c2[4 * g + 2], c2[4 * g + 3]};
        d[g] = __builtin_amdgcn_mfma_f32_4x4x1f32(ax[g], px, d[g], 0, 0, 0);
        d[g] = __builtin_amdgcn_mfma_f32_4x4x1f32(ay[g], py, d[g], 0, 0, 0);
    }
    float b = __builtin_inff(), b2 = __builtin_inff();
    int bi = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const float v = d[i / 4][i % 4];
        const bool lt = v < b;
        b2 = lt ? b : fminf(b2, v);
        bi = lt ? i : bi;
        b = lt ? v : b;
    }
    const float E = 0x1p-21f * (emul_c2 + 2.0f * (emul_x * fabsf(px) + emul_y * fabsf(py))) + kAbsRound;
    const float P = px * px + py * py;
    const float margin = 2.0f * E + 0x1p-19f * (fabsf(b) + P + E);
    if (__builtin_expect(!(b2 - b > margin), 0)) return assign_fast<K>(px, py, cx, cy, thr);  // close call / NaN
    const float2 c = s_c[bi];
    const float dx = __fsub_rn(c.x, px), dy = __fsub_rn(c.y, py);
    return __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)) < thr2 ? (uint32_t)bi : 255u;  // sqrt_rn(d2) < thr
}

// Matrix engine, streaming form (k <= 16, 16-B aligned points): v_mfma_f32_32x32x2f32, a 32 x 32
// x 2 product per instruction (4x the work of the 4x4x1 form above at twice its cycles).  A = 32
// centre rows (k index 0: -2 cx, 1: -2 cy), row i holding centre (i & 3) | (i >> 3) << 2, so that
// D register r of EVERY lane is centre r (rows (r&3) + 8 (r>>2) + 4 (lane>>5)); B = 32 point
// columns (lanes 0-31: x, lanes 32-63: y of point lane & 31); C = |c_r|^2.  D is the same k-ordered
// fma chain as assign_mfma's two 4x4x1 steps, fma(-2cy, py, fma(-2cx, px, |c|^2)).  Both halves of
// the wave see the same 32 columns, so each pair of instructions (even and odd points of 32 pairs)
// leaves lanes 0-31 the even points' 16 values and lanes 32-63 the odd points'.
typedef float floatx16_t __attribute__((ext_vector_type(16)));

// The argmin of one point from its 16 MFMA values s_r = |c_r|^2 - 2 c_r.p: the smallest s, and the
// one index whose s lies below s + margin' (margin' = 1.0625 x assign_mfma's margin, which covers
// the rounding of the sum, so every other s exceeds the winner by more than the margin).  More
// than one such index (a close call, a tie), none (NaN input) or an infinite margin takes the exact
// vector path; so does a non-finite point.  Same proof as assign_mfma.
template <int K>
__device__ __forceinline__ uint32_t pick_mfma(const float (&v)[K], float px, float py, float emul_c2, float emul_x,
                                              float emul_y, const float2 *__restrict__ s_c, const float (&cx)[K],
                                              const float (&cy)[K], float thr, float thr2) {
    float b = v[0];
#pragma unroll
    for (int i = 1; i < K; ++i) b = fminf(b, v[i]);
    const float E = 0x1p-21f * (emul_c2 + 2.0f * (emul_x * fabsf(px) + emul_y * fabsf(py))) + kAbsRound;
    const float P = px * px + py * py;
    const float margin = 2.0f * E + 0x1p-19f * (fabsf(b) + P + E);
    const float lim = b + 1.0625f * margin;
    int cnt = 0, bi = 0;
#pragma unroll
    for (int i = K - 1; i >= 0; --i) {
        const bool in = v[i] < lim;
        cnt += in ? 1 : 0;
        bi = in ? i : bi;
    }
    if (__builtin_expect(!(cnt == 1 && lim < __builtin_inff()), 0)) return assign_fast<K>(px, py, cx, cy, thr);
    const float2 c = s_c[bi];
    const float dx = __fsub_rn(c.x, px), dy = __fsub_rn(c.y, py);
    return __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)) < thr2 ? (uint32_t)bi : 255u;  // sqrt_rn(d2) < thr
}

constexpr int kF32Unroll = 4;  // 64-point blocks per wave per trip (loads in flight together)

template <int K, bool kMfma, bool kAccumulate>
__global__ void __launch_bounds__(kThreads)
kmeans_f32_fast_kernel(const float2 *__restrict__ xy, int64_t n, const float *__restrict__ cent, int k, float thr,
                       float thr2, double *__restrict__ acc, int n_copies, const KmState *__restrict__ st,
                       uint8_t *__restrict__ labels) {
    if (kAccumulate && st->done) return;
    __shared__ uint32_t s_n[kWaves][K];
    __shared__ double s_sx[kWaves][K], s_sy[kWaves][K];
    __shared__ float2 s_c[K];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    float cx[K], cy[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        cx[i] = uniform_f32(i < k ? cent[2 * i] : __builtin_inff());
        cy[i] = uniform_f32(i < k ? cent[2 * i + 1] : __builtin_inff());
    }
    // matrix-engine operands: A rows (lane & 3 = row i of every 4x4 block), |c|^2 per register
    float ax[K / 4], ay[K / 4], c2[K];
    float em_c2 = 0.f, em_x = 0.f, em_y = 0.f;
    if constexpr (kMfma) {
#pragma unroll
        for (int g = 0; g < K / 4; ++g) {
            const int i = 4 * g + (lane & 3);
            const float vx = i < k ? cent[2 * i] : 0.f, vy = i < k ? cent[2 * i + 1] : 0.f;
            ax[g] = -2.0f * vx;
            ay[g] = -2.0f * vy;
        }
#pragma unroll
        for (int i = 0; i < K; ++i) {
            c2[i] = i < k ? __fadd_rn(__fmul_rn(cx[i], cx[i]), __fmul_rn(cy[i], cy[i])) : __builtin_inff();
            if (i < k) {
                em_c2 = fmaxf(em_c2, c2[i]);
                em_x = fmaxf(em_x, fabsf(cx[i]));
                em_y = fmaxf(em_y, fabsf(cy[i]));
            }
        }
    }
    if (tid < K) s_c[tid] = make_float2(tid < k ? cent[2 * tid] : __builtin_inff(), tid < k ? cent[2 * tid + 1] : __builtin_inff());
    if (kAccumulate && lane < K) {
        s_n[wave][lane] = 0u;
        s_sx[wave][lane] = 0.0;
        s_sy[wave][lane] = 0.0;
    }
    __syncthreads();
    const int64_t nblk = (n + 63) / 64;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    for (int64_t b0 = (int64_t)blockIdx.x * kWaves + wave; b0 < nblk; b0 += stride * kF32Unroll) {
        float2 q[kF32Unroll];
#pragma unroll
        for (int u = 0; u < kF32Unroll; ++u) {  // clamped, unconditional: all loads in flight at once
            const int64_t p = (b0 + u * stride) * 64 + lane;
            q[u] = xy[p < n ? p : n - 1];
        }
#pragma unroll
        for (int u = 0; u < kF32Unroll; u += 2) {
            if (b0 + u * stride >= nblk) break;  // wave-uniform
            uint32_t lab[2];
            if constexpr (kMfma) {
                lab[0] = assign_mfma<K>(q[u].x, q[u].y, ax, ay, c2, em_c2, em_x, em_y, s_c, cx, cy, thr, thr2);
                lab[1] = assign_mfma<K>(q[u + 1].x, q[u + 1].y, ax, ay, c2, em_c2, em_x, em_y, s_c, cx, cy, thr, thr2);
            } else {
                assign_pair<K>(q[u], q[u + 1], cx, cy, s_c, thr, thr2, lab[0], lab[1]);
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int64_t blk = b0 + (u + h) * stride;
                if (blk >= nblk) break;  // wave-uniform
                const int64_t p = blk * 64 + lane;
                const uint32_t l = p < n ? lab[h] : 255u;
                if (labels && p < n) labels[p] = (uint8_t)l;
                if (kAccumulate && l < (uint32_t)K) {
                    atomicAdd(&s_n[wave][l], 1u);
                    atomicAdd(&s_sx[wave][l], (double)q[u + h].x);
                    atomicAdd(&s_sy[wave][l], (double)q[u + h].y);
                }
            }
        }
    }
    if (!kAccumulate) return;
    __syncthreads();
    if (tid < 3 * k) {
        const int f = tid / k, c = tid - f * k;
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) v += f == 0 ? (double)s_n[w][c] : (f == 1 ? s_sx[w][c] : s_sy[w][c]);
        if (v != 0.0) atomicAdd(&acc[(int)(blockIdx.x % n_copies) * kAccStride + 3 * c + f], v);
    }
}

// ---- candidate table for the vector engine (k <= 32, 16-B aligned points) ---------------------
// Each Lloyd pass labels every point by the first centre of smallest sqrt_rn(d2); with k = 16
// that is ~105 VALU per point in the screen above, and the pass is VALU-bound (r03j counters:
// 84 M VALU wave-instructions for 50 M points, 71 % busy).  Here a 64 x 64 grid of square cells
// over the points' bounding box holds, per cell and pass, the centres that can win ANYWHERE in
// the cell (computed in fp64 by the update kernel right after the centres move):
//   candidate i  <=>  dmin2_i(cell) <= min_j dmax2_j(cell) * (1 + 2^-12) + 1e-30,
// the cell grown by cs * 2^-12 on each side (covers the fp32 cell-index rounding, < cs * 2^-16).
// A non-candidate's fp32 d2 then exceeds the winner's by more than 2^-13 relative, beyond the
// fp32 rounding of d2 (< 2^-21) and assign_fast's 2^-20 square-root tie band: it can neither win
// nor make the tie test fire, so testing the (at most 3) candidates in ascending index with
// assign_fast's own steps gives assign_fast's label.  A cell whose every point lies beyond the
// threshold (dmin2 > thr2 (1 + 2^-12) for all centres) names a NaN sentinel centre three times
// (d2 NaN: no tie, label 255); more than 3 candidates name an infinite one (d2 = inf: the tie
// test fires).  A point outside the grid (or NaN) and a tie-band hit take assign_fast's steps over
// all centres.  The bounding box comes from a 64 K-point sample (points outside it are only
// slower, never wrong).  An entry holds the three candidates' BYTE offsets into the kernels' LDS
// centre table (10 bits each), so the lookup needs no shifts.
constexpr int kLutSide = 64;
constexpr int kLutCells = kLutSide * kLutSide;
constexpr int kLutBlocks = kLutCells / kThreads;
constexpr int kBoxBlocks = 64, kBoxPerThread = 4;
constexpr int kLutInf = kFastMaxK, kLutNan = kFastMaxK + 1;  // sentinel slots of the centre table
// Candidate slots the assignment tests per point.  With pairwise domination (lut_entry) about 1 %
// of the cells near the centres keep 3 candidates: their points go through the wave's fallback
// queue, which is cheaper than a third distance for every point.
constexpr int kLutSlots = 2;
__host__ __device__ constexpr uint32_t lut_pack(uint32_t a, uint32_t b, uint32_t c) {
    return (a * 8u) | (b * 8u) << 10 | (c * 8u) << 20;
}
constexpr uint32_t kLutFull = lut_pack(kLutInf, kLutInf, kLutInf);
constexpr uint32_t kLutFar = lut_pack(kLutNan, kLutNan, kLutNan);

struct LutGeom {
    float x0, y0, inv_cs, fgx, fgy, cs;
    int32_t gx, gy, ok, pad[7];
};
static_assert(sizeof(LutGeom) == 64, "LutGeom is one 64-B record");

// float -> u32 with the same order (so u32 atomic max gives float max; max of ~u gives the min)
__device__ __forceinline__ uint32_t ordered_u32(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float from_ordered(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// box[4 b + 0..3] = workgroup b's max ord(x), max ~ord(x), max ord(y), max ~ord(y) over its finite
// sampled points (0 = none); kmeans_update_lut_kernel reduces the kBoxBlocks records.  (One u32
// atomic max per wave into a single record measured 15 us: 1024 same-address atomics.)
__global__ void __launch_bounds__(kThreads)
kmeans_bbox_sample_kernel(const float2 *__restrict__ xy, int64_t n, uint32_t *__restrict__ box) {
    constexpr int64_t kSamples = (int64_t)kBoxBlocks * kThreads * kBoxPerThread;
    __shared__ uint32_t s_r[kThreads / 64][4];
    const int64_t step = n > kSamples ? n / kSamples : 1;
    const int tid = threadIdx.x;
    float2 p[kBoxPerThread + 1];
#pragma unroll
    for (int u = 0; u < kBoxPerThread; ++u) {
        const int64_t j = (((int64_t)blockIdx.x * kThreads + tid) * kBoxPerThread + u) * step;
        p[u] = xy[j < n ? j : n - 1];
    }
    p[kBoxPerThread] = xy[n - 1];  // the last point too
    uint32_t r[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int u = 0; u <= kBoxPerThread; ++u) {
        if (__builtin_isfinite(p[u].x) && __builtin_isfinite(p[u].y)) {
            const uint32_t ox = ordered_u32(p[u].x), oy = ordered_u32(p[u].y);
            r[0] = max(r[0], ox);
            r[1] = max(r[1], ~ox);
            r[2] = max(r[2], oy);
            r[3] = max(r[3], ~oy);
        }
    }
#pragma unroll
    for (int f = 0; f < 4; ++f) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) r[f] = max(r[f], (uint32_t)__shfl_xor((int)r[f], o));
    }
    if ((tid & 63) == 0)
        for (int f = 0; f < 4; ++f) s_r[tid >> 6][f] = r[f];
    __syncthreads();
    if (tid < 4) {
        uint32_t v = 0u;
        for (int w = 0; w < kThreads / 64; ++w) v = max(v, s_r[w][tid]);
        box[4 * blockIdx.x + tid] = v;
    }
}

// The grid over the sampled box (deterministic: every launch derives the same record).
__device__ inline LutGeom lut_geometry(const uint32_t (&box)[4]) {
    LutGeom g{};
    g.ok = 0;
    if (box[0] == 0u) return g;
    const float xmax = from_ordered(box[0]), xmin = from_ordered(~box[1]);
    const float ymax = from_ordered(box[2]), ymin = from_ordered(~box[3]);
    const double mag = fmax(fmax(fabs((double)xmin), fabs((double)xmax)), fmax(fabs((double)ymin), fabs((double)ymax)));
    if (!(mag < 1e18)) return g;  // keeps every candidate's fp32 d2 finite
    const double w = (double)xmax - xmin, h = (double)ymax - ymin;
    double cs = fmax(w, h) / kLutSide * (1.0 + 0x1p-10);
    cs = fmax(cs, fmax(mag * 0x1p-20, 1e-12));
    g.cs = (float)cs;
    g.inv_cs = __fdiv_rn(1.0f, g.cs);
    g.gx = min(kLutSide, (int)(w / (double)g.cs) + 1);
    g.gy = min(kLutSide, (int)(h / (double)g.cs) + 1);
    g.x0 = xmin;
    g.y0 = ymin;
    g.fgx = (float)g.gx;
    g.fgy = (float)g.gy;
    g.ok = 1;
    return g;
}

// One cell's entry: the candidates (ascending, padded with the last) as lut_pack offsets,
// kLutFar when no point of the cell can be within the threshold, kLutFull past 3 candidates.
__device__ inline uint32_t lut_entry(int ix, int iy, const LutGeom &g, const float2 *__restrict__ s_c, int k,
                                     float thr2) {
    const double cs = g.cs, e = cs * 0x1p-12;
    const double x0 = (double)g.x0 + ix * cs - e, x1 = (double)g.x0 + (ix + 1) * cs + e;
    const double y0 = (double)g.y0 + iy * cs - e, y1 = (double)g.y0 + (iy + 1) * cs + e;
    auto dmin2 = [&](float2 c) {
        const double dx = fmax(fmax(x0 - c.x, c.x - x1), 0.0), dy = fmax(fmax(y0 - c.y, c.y - y1), 0.0);
        return dx * dx + dy * dy;
    };
    double best = __builtin_inf(), near = __builtin_inf();
    for (int i = 0; i < k; ++i) {
        const float2 c = s_c[i];
        const double dx = fmax(fabs(c.x - x0), fabs(c.x - x1)), dy = fmax(fabs(c.y - y0), fabs(c.y - y1));
        best = fmin(best, dx * dx + dy * dy);
        near = fmin(near, dmin2(c));
    }
    // every point beyond the threshold: 255 whatever the candidates (far from all centres, many
    // of them are nearly equidistant, so such cells would otherwise overflow)
    if (near > (double)thr2 * (1.0 + 0x1p-12) + 1e-30) return kLutFar;
    const double bound = best * (1.0 + 0x1p-12) + 1e-30;
    constexpr int kPre = 4;
    int pre[kPre] = {0, 0, 0, 0};
    int np = 0;
    for (int i = 0; i < k; ++i) {
        if (dmin2(s_c[i]) <= bound) {
            pre[np < kPre ? np : kPre - 1] = np < kPre ? i : pre[kPre - 1];
            ++np;
        }
    }
    if (np == 0 || np > kPre) return kLutFull;  // (none: non-finite centres) -> all centres
    // Pairwise domination (the bound above is per centre): i cannot win in the cell if some other
    // candidate j has d_i^2 > (1 + 2^-12) d_j^2 + 1e-30 at every point of it.  d_i^2 - (1+eps) d_j^2
    // is concave in the point (its quadratic part is -eps |p|^2), so its minimum over the cell is
    // at a corner: four evaluations decide.  A pruned centre then stays 2^-13 above the winner, as
    // the per-centre bound guarantees.  This leaves 1-2 candidates in nearly every cell (the bound
    // alone left 4+ near Voronoi vertices).  Fixed-size, fully unrolled (register arrays).
    double dc[kPre][4];
#pragma unroll
    for (int a = 0; a < kPre; ++a) {
        const float2 c = s_c[pre[a]];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const double dx = c.x - ((q & 1) ? x1 : x0), dy = c.y - ((q & 2) ? y1 : y0);
            dc[a][q] = dx * dx + dy * dy;
        }
    }
    uint32_t keep = (1u << np) - 1u;
#pragma unroll
    for (int a = 0; a < kPre; ++a) {
#pragma unroll
        for (int b = 0; b < kPre; ++b) {
            if (a == b) continue;
            bool dom = a < np && b < np;
#pragma unroll
            for (int q = 0; q < 4; ++q) dom = dom && (dc[a][q] - (1.0 + 0x1p-12) * dc[b][q] > 1e-30);
            keep &= dom ? ~(1u << a) : ~0u;
        }
    }
    uint32_t cand[3] = {0u, 0u, 0u};
    int cnt = 0;
#pragma unroll
    for (int a = 0; a < kPre; ++a) {
        if (keep >> a & 1u) {
            if (cnt < 3) cand[cnt] = (uint32_t)pre[a];
            ++cnt;
        }
    }
    if (cnt == 0 || cnt > kLutSlots) return kLutFull;
    if (cnt < 2) cand[1] = cand[0];
    return lut_pack(cand[0], cand[1], cand[1]);
}

// Centroid update fused with the candidate table.  kLutBlocks workgroups each sum the replicas
// (the same fp64 arithmetic as kmeans_update_kernel), keep the new centres in LDS and build 256
// cells; workgroup 0 writes the centres and the state.  Accumulators ping-pong between two sets:
// this launch reads acc_rd and zeroes acc_zero (read by the previous update), so no workgroup
// zeroes what another still reads.  iter < 0: table for the current centres only (before pass 0;
// also writes the grid record).  st->done holds iter + 1 of the converging update, so workgroups
// of that same launch still build its table.
__global__ void __launch_bounds__(kThreads)
kmeans_update_lut_kernel(const double *__restrict__ acc_rd, double *__restrict__ acc_zero, int n_copies,
                         float *__restrict__ cent, int k, float tol, KmState *__restrict__ st, int iter,
                         const uint32_t *__restrict__ box, LutGeom *__restrict__ geom, uint32_t *__restrict__ lut,
                         float thr2) {
    if (iter >= 0) {
        const int d = __builtin_amdgcn_readfirstlane(st->done);
        if (d != 0 && d <= iter) return;
    }
    __shared__ float2 s_c[kFastMaxK];
    __shared__ LutGeom s_g;
    const int tid = threadIdx.x;
    if (tid >= 64 && tid < 128) {  // wave 1: the grid record (reduced from the samples before pass 0)
        if (iter < 0) {
            const int l = tid - 64;
            uint32_t r[4];
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                r[f] = l < kBoxBlocks ? box[4 * l + f] : 0u;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) r[f] = max(r[f], (uint32_t)__shfl_xor((int)r[f], o));
            }
            if (l == 0) {
                s_g = lut_geometry(r);
                if (blockIdx.x == 0) *geom = s_g;
            }
        } else if (tid == 64) {
            s_g = *geom;
        }
    }
    if (iter >= 0) {
        const int z = blockIdx.x * kThreads + tid;
        if (z < n_copies * kAccStride) acc_zero[z] = 0.0;
    }
    if (tid < 64) {  // wave 0: centres (k <= 32 lanes) and, in workgroup 0, the state
        float shift = 0.f;
        if (tid < k) {
            const float ox = cent[2 * tid], oy = cent[2 * tid + 1];
            float nx = ox, ny = oy;
            if (iter >= 0) {
                double a[3] = {0.0, 0.0, 0.0}, v[kAccCopies][3];
#pragma unroll
                for (int r = 0; r < kAccCopies; ++r)
#pragma unroll
                    for (int f = 0; f < 3; ++f) v[r][f] = r < n_copies ? acc_rd[r * kAccStride + 3 * tid + f] : 0.0;
#pragma unroll
                for (int r = 0; r < kAccCopies; ++r)
#pragma unroll
                    for (int f = 0; f < 3; ++f) a[f] += v[r][f];
                if (a[0] > 0.0) {
                    nx = (float)(a[1] / a[0]);
                    ny = (float)(a[2] / a[0]);
                    shift = fmaxf(fabsf(nx - ox), fabsf(ny - oy));
                    if (blockIdx.x == 0) {
                        cent[2 * tid] = nx;
                        cent[2 * tid + 1] = ny;
                    }
                }
            }
            s_c[tid] = make_float2(nx, ny);
        }
        if (iter >= 0 && blockIdx.x == 0) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) shift = fmaxf(shift, __shfl_xor(shift, o));
            if (tid == 0) {
                st->iters += 1;
                if (tol >= 0.f && shift <= tol) st->done = iter + 1;
            }
        }
    }
    __syncthreads();
    const LutGeom g = s_g;
    if (!g.ok) return;
    const int c = blockIdx.x * kThreads + tid;
    if (c < g.gx * g.gy) lut[c] = lut_entry(c % g.gx, c / g.gx, g, s_c, k, thr2);
}

// What the assignment kernels need of the grid record.
struct LutView {
    float x0, y0, inv_cs, fgx_m, fgy_m;  // fgx_m: the largest float below the column count
    int32_t gx4;                          // row stride of the table in bytes
};

// assign_fast's steps with the centres read from LDS (the table kernels keep no centres in
// registers; this is their rare fallback)
template <int K>
__device__ __forceinline__ uint32_t assign_lds2(float px, float py, const float2 *__restrict__ s_c, float thr) {
    float m = __builtin_inff(), m_prev = __builtin_inff();
    int ia = 0;
#pragma unroll 4
    for (int i = 0; i < K; ++i) {
        const float2 c = s_c[i];
        const float dx = __fsub_rn(c.x, px), dy = __fsub_rn(c.y, py);
        const float d2 = __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy));
        const bool lt = d2 < m;
        m_prev = lt ? m : m_prev;
        ia = lt ? i : ia;
        m = lt ? d2 : m;
    }
    if (m_prev <= __fmul_rn(m, 1.0f + 0x1p-20f)) {
        uint32_t best = 255u;
        float best_s = thr;
        for (int i = 0; i < K; ++i) {
            const float2 c = s_c[i];
            const float dx = __fsub_rn(c.x, px), dy = __fsub_rn(c.y, py);
            const float sd = ecc::sqrt_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)));
            if (sd < best_s) { best_s = sd; best = (uint32_t)i; }
        }
        return best;
    }
    return ecc::sqrt_rn(m) < thr ? (uint32_t)ia : 255u;
}

// One point through the table: assign_fast's steps over the cell's kLutSlots candidates.  full =
// the caller must take the steps over all centres (outside the grid, > 3 candidates, or a
// tie-band hit).  ~33 VALU per point: med3 clamps the cell coordinates and tells inside from
// outside in one compare, the entry's byte offsets address the centre table directly, and the
// first candidate seeds the running minimum (a real candidate's d2 is finite; the sentinels' inf /
// NaN propagate as described above).
__device__ __forceinline__ uint32_t lut_point(float px, float py, const LutView &g, const uint32_t *__restrict__ s_lut,
                                              const float2 *__restrict__ s_c, float thr2, bool &full) {
    const float tx = __fmul_rn(__fsub_rn(px, g.x0), g.inv_cs), ty = __fmul_rn(__fsub_rn(py, g.y0), g.inv_cs);
    const float cxf = __builtin_amdgcn_fmed3f(tx, 0.f, g.fgx_m), cyf = __builtin_amdgcn_fmed3f(ty, 0.f, g.fgy_m);
    const bool inside = (cxf == tx) & (cyf == ty);  // false for NaN
    const uint32_t a = __umul24((uint32_t)(int)cyf, (uint32_t)g.gx4) + ((uint32_t)(int)cxf << 2);
    const uint32_t e = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(s_lut) + a);
    const uint32_t o0 = e & 0x3ffu, o1 = (e >> 10) & 0x3ffu;
    const char *cb = reinterpret_cast<const char *>(s_c);
    const float2 c0 = *reinterpret_cast<const float2 *>(cb + o0);
    const float2 c1 = *reinterpret_cast<const float2 *>(cb + o1);
    auto d2 = [&](float2 c) {
        const float dx = __fsub_rn(c.x, px), dy = __fsub_rn(c.y, py);
        return __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy));
    };
    float m = d2(c0), m_prev = __builtin_inff();
    uint32_t ia = o0;
    {
        const float d = d2(c1);
        const bool lt = d < m;
        m_prev = lt ? m : m_prev;
        ia = lt ? o1 : ia;
        m = lt ? d : m;
    }
    full = !inside | (m_prev <= __fmul_rn(m, 1.0f + 0x1p-20f));
    return m < thr2 ? ia >> 3 : 255u;
}

// Vector engine, streaming form: a lane takes two consecutive points per 16-B load (the pair the
// packed screen tests together), kPairUnroll such loads per trip, and the NEXT trip's loads are
// issued before this trip's tests, so a wave keeps 2 x kPairUnroll x 16 B in flight across its
// compute (the one-trip form waited on its loads every trip: bound by bytes in flight, ~2.2 TB/s).
// The pair's two labels go out as one 2-byte store.  Needs 16-B aligned points (and labels 2-B
// aligned); an odd last point is taken by lane 0 of workgroup 0.
constexpr int kPairUnroll = 4;

template <int K, bool kAccumulate, bool kLut, bool kMfma = false>
__global__ void __launch_bounds__(kThreads, kMfma ? ECC_KM_MFMA_WAVES : 1)
kmeans_f32_pair_kernel(const float4 *__restrict__ xy4, int64_t n, const float *__restrict__ cent, int k, float thr,
                       float thr2, double *__restrict__ acc, int n_copies, const KmState *__restrict__ st,
                       uint8_t *__restrict__ labels, const LutGeom *__restrict__ geom,
                       const uint32_t *__restrict__ lut) {
    if (kAccumulate && st->done) return;
    // accumulator slots per wave, kSub copies (lane % kSub) to spread same-address LDS atomics
    constexpr int kSub = ECC_KM_ACC_SUB;
    __shared__ uint32_t s_n[kWaves * kSub][K];
    __shared__ double s_sx[kWaves * kSub][K], s_sy[kWaves * kSub][K];
    __shared__ float2 s_c[kLut ? kFastMaxK + 2 : K];  // + the table's inf and NaN sentinels
    __shared__ __attribute__((aligned(16))) uint32_t s_lut[kLut ? kLutCells : 4];
    __shared__ float4 s_q[kWaves][kLut ? 128 : 1];  // fallback queues: < 64 + 64 entries
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    // The grid record as scalars (a struct copy of the 64-B record went to the stack).  Without a
    // grid (non-finite or huge box) every point is outside: fgx = 0, one cell, assign_lds2.
    LutView g{};
    if constexpr (kLut) {
        const bool ok = geom->ok != 0;
        g.x0 = geom->x0;
        g.y0 = geom->y0;
        g.inv_cs = geom->inv_cs;
        if (!ok) g.inv_cs = __builtin_nanf("");  // no grid: every point is outside (NaN compares false)
        g.fgx_m = ok ? __uint_as_float(__float_as_uint(geom->fgx) - 1u) : 0.f;  // fgx >= 1
        g.fgy_m = ok ? __uint_as_float(__float_as_uint(geom->fgy) - 1u) : 0.f;
        g.gx4 = ok ? 4 * geom->gx : 4;
        if (tid == kLutInf) s_c[kLutInf] = make_float2(__builtin_inff(), __builtin_inff());
        if (tid == kLutNan) s_c[kLutNan] = make_float2(__builtin_nanf(""), __builtin_nanf(""));
        // the table into LDS: all of a lane's 16-B loads in flight at once (a strided word loop
        // paid one L2 round trip per word, at the start of every workgroup)
        const __amdgpu_buffer_rsrc_t v = ecc::buffer_view(lut, ok ? (uint32_t)(geom->gx * geom->gy) * 4u : 0u);
        uint4 q[kLutCells / (4 * kThreads)];
#pragma unroll
        for (int u = 0; u < kLutCells / (4 * kThreads); ++u)
            q[u] = ecc::buffer_load_u128(v, (uint32_t)tid * 16u, (uint32_t)(u * kThreads * 16));
#pragma unroll
        for (int u = 0; u < kLutCells / (4 * kThreads); ++u)
            reinterpret_cast<uint4 *>(s_lut)[u * kThreads + tid] = q[u];
        if (!ok && tid == 0) s_lut[0] = kLutFull;
    }
    float cx[K], cy[K];  // the screen's centres in scalar registers (not with the table)
    if constexpr (!kLut) {
#pragma unroll
        for (int i = 0; i < K; ++i) {
            cx[i] = uniform_f32(i < k ? cent[2 * i] : __builtin_inff());
            cy[i] = uniform_f32(i < k ? cent[2 * i + 1] : __builtin_inff());
        }
    }
    // matrix-engine operands (kMfma): this lane's A element, |c_r|^2 as the C input, error scales
    float a_ev = 0.f, a_od = 0.f, em_c2 = 0.f, em_x = 0.f, em_y = 0.f;
    floatx16_t c2v{};
    if constexpr (kMfma) {
        static_assert(K == 16, "the 32x32x2 layout maps D register r to centre r < 16");
        const int i = lane & 31, c = (i & 3) | ((i >> 3) << 2);
        const float a_op = c < k ? -2.0f * cent[2 * c + (lane >> 5)] : 0.f;
        // rows (i & 4) == 0 are lanes 0-31's D rows, the others lanes 32-63's: the even points'
        // instruction fills the first, the odd points' (chained on its output) the second
        a_ev = (i & 4) ? 0.f : a_op;
        a_od = (i & 4) ? a_op : 0.f;
#pragma unroll
        for (int r = 0; r < K; ++r) {
            c2v[r] = r < k ? __fadd_rn(__fmul_rn(cx[r], cx[r]), __fmul_rn(cy[r], cy[r])) : __builtin_inff();
            if (r < k) {
                em_c2 = fmaxf(em_c2, c2v[r]);
                em_x = fmaxf(em_x, fabsf(cx[r]));
                em_y = fmaxf(em_y, fabsf(cy[r]));
            }
        }
    }
    if (tid < K) s_c[tid] = make_float2(tid < k ? cent[2 * tid] : __builtin_inff(), tid < k ? cent[2 * tid + 1] : __builtin_inff());
    if (kAccumulate && lane < K) {
        for (int b = 0; b < kSub; ++b) {
            s_n[wave * kSub + b][lane] = 0u;
            s_sx[wave * kSub + b][lane] = 0.0;
            s_sy[wave * kSub + b][lane] = 0.0;
        }
    }
    const int slot = wave * kSub + lane % kSub;
    __syncthreads();
    auto account = [&](float2 q, uint32_t l) __attribute__((always_inline)) {
        if (kAccumulate && l < (uint32_t)K) {
            atomicAdd(&s_n[slot][l], 1u);
            atomicAdd(&s_sx[slot][l], (double)q.x);
            atomicAdd(&s_sy[slot][l], (double)q.y);
        }
    };
    const int64_t npair = n / 2;
    const int64_t nblk = (npair + 63) / 64;  // 64 pairs per wave block
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    // table path: loads per trip (8 measured slower than 4: 117 vs 110 us per accumulate pass)
    // matrix engine: each lane loads the pairs of lanes (lane & 31) and (lane & 31) + 32 of a block
    // (the two column sets of its two instruction pairs; the duplicate addresses coalesce)
    constexpr int kBlk = kMfma ? ECC_KM_MFMA_BLOCKS : (kLut ? ECC_KM_LUT_UNROLL : kPairUnroll);  // blocks per trip
    constexpr int kU = kMfma ? 2 * kBlk : kBlk;  // 16-B loads per lane per trip
    const int64_t span = stride * kBlk;
    // a trip's loads through a buffer view based at its first pair: unconditional (0 past the
    // last pair), one VGPR of lane offset for all of them, the u part in the scalar offset
    auto load = [&](int64_t b0, float4 (&q)[kU]) __attribute__((always_inline)) {
        const int64_t first = b0 * 64 < npair ? b0 * 64 : npair;
        const int64_t rem = (npair - first) * 16;
        const __amdgpu_buffer_rsrc_t v = ecc::buffer_view(xy4 + first, rem < 0xffffffffll ? (uint32_t)rem : 0xffffffffu);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint32_t lo = kMfma ? (uint32_t)(lane & 31) * 16u + (uint32_t)(u & 1) * 512u : (uint32_t)lane * 16u;
            const uint4 w = ecc::buffer_load_u128(v, lo, (uint32_t)((kMfma ? u >> 1 : u) * stride * 64 * 16));
            q[u] = make_float4(__uint_as_float(w.x), __uint_as_float(w.y), __uint_as_float(w.z), __uint_as_float(w.w));
        }
    };
    // Fallback queue of this wave (table path): points the table cannot decide (outside the grid,
    // > kLutSlots candidates, a tie-band hit) are appended with their index and labelled 64 at a
    // time by assign_lds2 with every lane busy, instead of one divergent round per trip.  The
    // queue is wave-private LDS; a wave's LDS operations execute in order, so only the compiler
    // is fenced.  A queued point's byte label is stored after the trip's 2-byte store of its pair.
    uint32_t qn = 0;  // wave-uniform fill
    auto drain = [&](uint32_t cnt) __attribute__((always_inline)) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint32_t i = qn - cnt + (uint32_t)lane;
        if ((uint32_t)lane < cnt) {
            const float4 e = s_q[wave][i];
            const float2 q2 = make_float2(e.x, e.y);
            const uint32_t l = assign_lds2<K>(q2.x, q2.y, s_c, thr);
            const int64_t idx = (int64_t)__float_as_uint(e.z) | ((int64_t)__float_as_uint(e.w) << 32);
            if (labels) labels[idx] = (uint8_t)l;
            account(q2, l);
        }
        qn -= cnt;
        __builtin_amdgcn_wave_barrier();
    };
    auto enqueue = [&](float2 p0, float2 p1, int64_t pp, bool f0, bool f1) __attribute__((always_inline)) {
        if constexpr (kLut) {
            const uint64_t m0 = __ballot(f0), m1 = __ballot(f1);
            if ((m0 | m1) == 0ull) return;  // uniform
            const uint32_t n0 = (uint32_t)__popcll(m0);
            const uint64_t below = lanes_below_mask(lane);
            auto put = [&](uint32_t slot, float2 pt, int64_t idx) {
                s_q[wave][slot] = make_float4(pt.x, pt.y, __uint_as_float((uint32_t)idx),
                                              __uint_as_float((uint32_t)((uint64_t)idx >> 32)));
            };
            // one half at a time with a drain check between: the queue never holds 128 entries
            if (f0) put(qn + (uint32_t)__popcll(m0 & below), p0, 2 * pp);
            qn += n0;
            if (qn >= 64u) drain(64u);
            if (f1) put(qn + (uint32_t)__popcll(m1 & below), p1, 2 * pp + 1);
            qn += (uint32_t)__popcll(m1);
            if (qn >= 64u) drain(64u);
        }
    };
    auto test = [&](int64_t b0, const float4 (&q)[kU]) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < kBlk; ++u) {
            const int64_t blk = b0 + u * stride;
            if (blk >= nblk) break;  // wave-uniform
            if constexpr (kMfma) {
                // set h = the pairs 32h..32h+31 of the block, in both halves of the wave
                const bool low = lane < 32;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int src = (lane & 31) + 32 * h;
                    const float4 qs = q[2 * u + h];
                    const float sx = qs.x, sy = qs.y, sz = qs.z, sw = qs.w;
                    // even points into lanes 0-31's rows (lanes 32-63 keep C), then the odd points
                    // into lanes 32-63's rows with the first result as C (lanes 0-31 add fma(0, b)
                    // terms: unchanged, or NaN for a non-finite odd point -> the exact path)
                    const floatx16_t de = __builtin_amdgcn_mfma_f32_32x32x2f32(a_ev, low ? sx : sy, c2v, 0, 0, 0);
                    const floatx16_t dd = __builtin_amdgcn_mfma_f32_32x32x2f32(a_od, low ? sz : sw, de, 0, 0, 0);
                    float v[K];
#pragma unroll
                    for (int r = 0; r < K; ++r) v[r] = dd[r];
                    const float px = low ? sx : sz, py = low ? sy : sw;  // lanes 0-31: even, 32-63: odd point
                    const uint32_t l = pick_mfma<K>(v, px, py, em_c2, em_x, em_y, s_c, cx, cy, thr, thr2);
                    const int64_t pq = blk * 64 + src;
                    if (pq < npair) {
                        if (labels) labels[2 * pq + (low ? 0 : 1)] = (uint8_t)l;
                        account(make_float2(px, py), l);
                    }
                }
                continue;
            }
            const int64_t pp = blk * 64 + lane;
            const float2 p0 = make_float2(q[u].x, q[u].y), p1 = make_float2(q[u].z, q[u].w);
            uint32_t l0, l1;
            bool f0 = false, f1 = false;
            if constexpr (kLut) {
                l0 = lut_point(p0.x, p0.y, g, s_lut, s_c, thr2, f0);
                l1 = lut_point(p1.x, p1.y, g, s_lut, s_c, thr2, f1);
                f0 = f0 && pp < npair;
                f1 = f1 && pp < npair;
            } else {
                assign_pair<K>(p0, p1, cx, cy, s_c, thr, thr2, l0, l1);
            }
            if (pp < npair) {
                if (labels) reinterpret_cast<uint16_t *>(labels)[pp] = (uint16_t)(l0 | l1 << 8);
                if (!f0) account(p0, l0);
                if (!f1) account(p1, l1);
            }
            // after the pair's store: a drain rewrites the queued points' bytes
            if constexpr (kLut) enqueue(p0, p1, pp, f0, f1);
        }
    };
    // Two buffers in ping-pong with unconditional (clamped) loads: no register copies between
    // trips and no branch around the loads, so the wait before each trip's tests covers only
    // that trip's own loads while the other buffer's are in flight.
    float4 qa[kU], qb[kU];
    int64_t b0 = (int64_t)blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(wave);  // uniform: scalar descriptors
    if (npair > 0 && b0 < nblk) {
        load(b0, qa);
        for (;;) {
            load(b0 + span, qb);
            test(b0, qa);
            b0 += span;
            if (b0 >= nblk) break;  // wave-uniform
            load(b0 + span, qa);
            test(b0, qb);
            b0 += span;
            if (b0 >= nblk) break;
        }
    }
    if constexpr (kLut) {
        if (qn) drain(qn);
    }
    if ((n & 1) && blockIdx.x == 0 && tid == 0) {  // the odd last point
        const float2 q = reinterpret_cast<const float2 *>(xy4)[n - 1];
        uint32_t l;
        if constexpr (kLut) l = assign_lds2<K>(q.x, q.y, s_c, thr);
        else l = assign_fast<K>(q.x, q.y, cx, cy, thr);
        if (labels) labels[n - 1] = (uint8_t)l;
        account(q, l);
    }
    if (!kAccumulate) return;
    __syncthreads();
    if (tid < 3 * k) {
        const int f = tid / k, c = tid - f * k;
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < kWaves * kSub; ++w) v += f == 0 ? (double)s_n[w][c] : (f == 1 ? s_sx[w][c] : s_sy[w][c]);
        if (v != 0.0) atomicAdd(&acc[(int)(blockIdx.x % n_copies) * kAccStride + 3 * c + f], v);
    }
}

// Host: the smallest float s >= 0 with sqrtf(s) >= thr (sqrtf correctly rounded, like sqrt_rn;
// monotone), so that sqrt_rn(d2) < thr <=> d2 < thr2.  Bisection over the bit patterns.
inline float sqrt_threshold(float thr) {
    if (!(thr > 0.f)) return 0.f;           // nothing is below (NaN threshold: nothing either)
    if (std::isinf(thr)) return __builtin_inff();
    uint32_t lo = 0u, hi = 0x7F800000u;      // sqrt(+0) < thr; sqrt(+inf) = inf >= thr
    while (hi - lo > 1u) {
        const uint32_t mid = lo + (hi - lo) / 2;
        float f;
        std::memcpy(&f, &mid, 4);
        (std::sqrt(f) < thr ? lo : hi) = mid;
    }
    float r;
    std::memcpy(&r, &hi, 4);
    return r;
}

template <bool kAccumulate>
bool launch_f32_fast(int k, int method, dim3 grid, hipStream_t s, const float *xy, int64_t n, const float *cent,
                     float thr, double *acc, int n_copies, const KmState *st, uint8_t *labels,
                     const LutGeom *geom = nullptr, const uint32_t *lut = nullptr) {
    const float thr2 = sqrt_threshold(thr);
    if (k > kFastMaxK) return false;
    const float2 *p = reinterpret_cast<const float2 *>(xy);
#define ECC_F32_LAUNCH(KK, MF)                                                                               \
    hipLaunchKernelGGL((kmeans_f32_fast_kernel<KK, MF, kAccumulate>), grid, dim3(kThreads), 0, s, p, n, cent, k, \
                       thr, thr2, acc, n_copies, st, labels)
    const bool pairs_ok = (reinterpret_cast<uintptr_t>(xy) & 15) == 0 && (reinterpret_cast<uintptr_t>(labels) & 1) == 0;
    if (method == 3 && k <= 16 && pairs_ok) {  // matrix engine, 32x32x2 streaming form
        hipLaunchKernelGGL((kmeans_f32_pair_kernel<16, kAccumulate, false, true>), grid, dim3(kThreads), 0, s,
                           reinterpret_cast<const float4 *>(xy), n, cent, k, thr, thr2, acc, n_copies, st, labels,
                           geom, lut);
    } else if (method >= 2) {  // matrix engine, 4x4x1 form (also engine 3's k > 16 / unaligned case)
        if (k <= 16) ECC_F32_LAUNCH(16, true);
        else ECC_F32_LAUNCH(32, true);
    } else if ((reinterpret_cast<uintptr_t>(xy) & 15) == 0 && (reinterpret_cast<uintptr_t>(labels) & 1) == 0) {  // 16-B loads of point pairs
        const float4 *p4 = reinterpret_cast<const float4 *>(xy);
#define ECC_PAIR_LAUNCH(KK, LUT)                                                                                 \
    hipLaunchKernelGGL((kmeans_f32_pair_kernel<KK, kAccumulate, LUT>), grid, dim3(kThreads), 0, s, p4, n, cent, k, \
                       thr, thr2, acc, n_copies, st, labels, geom, lut)
        if (geom) {
            if (k <= 16) ECC_PAIR_LAUNCH(16, true);
            else ECC_PAIR_LAUNCH(32, true);
        } else {
            if (k <= 16) ECC_PAIR_LAUNCH(16, false);
            else ECC_PAIR_LAUNCH(32, false);
        }
#undef ECC_PAIR_LAUNCH
    } else {
        if (k <= 16) ECC_F32_LAUNCH(16, false);
        else ECC_F32_LAUNCH(32, false);
    }
#undef ECC_F32_LAUNCH
    return true;
}

// Centroid update, one wave: c = (float)(sum / n) (fp64), shift = max |new - old|.
// Sums n_copies replicas of acc (stride kAccStride) and zeroes them.
template <typename AccT>
__global__ void __launch_bounds__(64)
kmeans_update_kernel(AccT *__restrict__ acc, int n_copies, float *__restrict__ cent, int k, float tol,
                     KmState *__restrict__ st) {
    if (st->done) return;
    const int lane = threadIdx.x;
    float shift = 0.f;
    if (lane < k) {
        AccT a[3] = {0, 0, 0};
        AccT v[kAccCopies][3];  // every replica's loads in flight together
#pragma unroll
        for (int r = 0; r < kAccCopies; ++r)
#pragma unroll
            for (int f = 0; f < 3; ++f) v[r][f] = r < n_copies ? acc[r * kAccStride + 3 * lane + f] : (AccT)0;
#pragma unroll
        for (int r = 0; r < kAccCopies; ++r)
#pragma unroll
            for (int f = 0; f < 3; ++f) {
                a[f] += v[r][f];
                if (r < n_copies) acc[r * kAccStride + 3 * lane + f] = 0;
            }
        const double n_pts = (double)a[0];
        if (n_pts > 0.0) {
            const float nx = (float)((double)a[1] / n_pts);
            const float ny = (float)((double)a[2] / n_pts);
            shift = fmaxf(fabsf(nx - cent[2 * lane]), fabsf(ny - cent[2 * lane + 1]));
            cent[2 * lane] = nx;
            cent[2 * lane + 1] = ny;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) shift = fmaxf(shift, __shfl_xor(shift, o));
    if (lane == 0) {
        st->iters += 1;
        if (tol >= 0.f && shift <= tol) st->done = 1;
    }
}

// ---- label image (k <= 32) -------------------------------------------------------------------
// The assignment depends on a point's (x, y) only, and event representatives sit on a sensor
// grid (the bench: 7.7 M points on 346x260 pixels, ~85 per pixel).  Each pass therefore first
// labels every pixel of the points' bounding box once (assign_fast, the same function), and the
// accumulation pass reads a point's label from that image instead of testing k centres.  Points
// outside the kImgSide x kImgSide area are assigned directly.

__global__ void __launch_bounds__(kThreads)
kmeans_extent_kernel(const uint32_t *__restrict__ xy, Segs segs, uint32_t *__restrict__ ext) {
    uint32_t mx = 0, my = 0;
    bool any = false;
    for (int64_t s = blockIdx.x; s < segs.n_segs; s += gridDim.x) {
        const int64_t cnt = segs.count(s), base = s * segs.stride;
        for (int64_t j = threadIdx.x; j < cnt; j += kThreads) {
            const uint32_t v = xy[base + j], x = v & 0xffffu, y = v >> 16;
            if (x < kImgSide && y < kImgSide) {
                mx = max(mx, x);
                my = max(my, y);
                any = true;
            }
        }
    }
    // per-WG maxima into ext[2 * blockIdx] (no atomics: same-address device atomics serialise)
    __shared__ uint32_t wmx[kThreads / 64], wmy[kThreads / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
        my = max(my, (uint32_t)__shfl_xor((int)my, o));
    }
    const bool wany = __any(any);
    if ((threadIdx.x & 63) == 0) {
        wmx[threadIdx.x >> 6] = wany ? mx + 1 : 0u;
        wmy[threadIdx.x >> 6] = wany ? my + 1 : 0u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t a = 0, b = 0;
        for (int w = 0; w < kThreads / 64; ++w) { a = max(a, wmx[w]); b = max(b, wmy[w]); }
        ext[2 * blockIdx.x] = a;
        ext[2 * blockIdx.x + 1] = b;
    }
}

// Per-pixel point counts: the assignment depends on a point's pixel only, so a Lloyd pass can
// visit each occupied pixel once with its multiplicity n, adding (n, n*x, n*y) — the same
// integer sums as adding every point.  Counts are compact over the bounding box (w x h from the
// extent kernel): cnt[y * w + x].  No global atomics (they execute at the memory side): workgroup
// (chunk c, part m) counts the points of its part falling in pixel chunk c into LDS and stores
// the chunk densely into partial[m]; kmeans_count_sum_kernel adds the parts.  Part 0's
// workgroups of chunk 0 also list the points outside the kImgSide^2 image.
constexpr int kHistThreads = 1024;
#ifndef ECC_KM_HIST_CHUNK
#define ECC_KM_HIST_CHUNK 32768
#endif
constexpr int kHistChunk = ECC_KM_HIST_CHUNK;  // pixels per LDS chunk (128 KiB)
constexpr int64_t kHistBudget = 16 << 20;  // partial-count entries (64 MiB): parts used = budget / cells

__host__ __device__ inline int parts_used(int parts, int64_t cells) {
    const int64_t p = cells > 0 ? kHistBudget / cells : parts;
    return (int)(p < 1 ? 1 : (p < parts ? p : parts));
}
constexpr int kHistUnroll = 4;
constexpr int kHistSegs = 4;
#ifndef ECC_KM_PIX_GRID
#define ECC_KM_PIX_GRID 128
#endif
// pixel-pass workgroups: on the k-means chain alone 256 were fastest (64: 102 us per ten passes
// against 82), but that chain runs beside the corner chain and has slack; 128 (87 us) leaves the
// corner chain more room: two-stream step 0.636 -> 0.630 ms
constexpr int kPixGrid = ECC_KM_PIX_GRID;

__device__ __forceinline__ void reduce_extent(const uint32_t *__restrict__ ext, int n_ext, uint32_t *s_red,
                                              uint32_t &w, uint32_t &h) {
    uint32_t p = 0, q = 0;
    for (int i = threadIdx.x; i < n_ext; i += blockDim.x) { p = max(p, ext[2 * i]); q = max(q, ext[2 * i + 1]); }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        p = max(p, (uint32_t)__shfl_xor((int)p, o));
        q = max(q, (uint32_t)__shfl_xor((int)q, o));
    }
    if ((threadIdx.x & 63) == 0) {
        s_red[2 * (threadIdx.x >> 6)] = p;
        s_red[2 * (threadIdx.x >> 6) + 1] = q;
    }
    __syncthreads();
    w = 0;
    h = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) { w = max(w, s_red[2 * i]); h = max(h, s_red[2 * i + 1]); }
}

// 1-D grid, XCD-aware: workgroup b runs on XCD b % 8; the kCountSlots chunk workgroups of one
// part (point range) share b % 8 and are dispatched back to back, so the second and third reads of
// the part's points hit that XCD's L2 instead of HBM.
// The slot count is the frame's chunk count when the caller gives the frame (3 at 346x260, so
// no workgroup of a fourth slot idles), else 4; parts fill the 256 CUs: 8 * (32 / slots).
constexpr int kCountSlots = 4;
#ifndef ECC_KM_COUNT_MUL
#define ECC_KM_COUNT_MUL 8
#endif
#ifndef ECC_KM_LAB_GRID
#define ECC_KM_LAB_GRID 256
#endif

__host__ __device__ inline int count_grid(int parts, int slots) { return 8 * ((parts + 7) / 8) * slots; }

inline void count_layout(int64_t n_segs, int64_t cells, int &parts, int &slots) {
    const int64_t ch = (cells + kHistChunk - 1) / kHistChunk;
    slots = cells > 0 ? (int)(ch < 1 ? 1 : (ch < kCountSlots ? ch : kCountSlots)) : kCountSlots;
    parts = (int)std::min<int64_t>(ECC_KM_COUNT_MUL * (32 / slots), std::max<int64_t>(n_segs, 1));
}

__global__ void __launch_bounds__(kHistThreads)
kmeans_count_kernel(const uint32_t *__restrict__ xy, Segs segs, const uint32_t *__restrict__ ext, int n_ext,
                    int parts, int slots, uint32_t *__restrict__ partial, uint32_t *__restrict__ wh,
                    uint32_t *__restrict__ outside, uint32_t *__restrict__ n_outside, uint32_t fixed_w,
                    uint32_t fixed_h, int32_t *__restrict__ err) {
    extern __shared__ uint32_t hist[];  // [kHistChunk]
    __shared__ uint32_t s_red[2 * kHistThreads / 64];
    const int xcd = (int)(blockIdx.x % 8), i8 = (int)(blockIdx.x / 8);
    const int m = (i8 / slots) * 8 + xcd, slot = i8 % slots, tid = threadIdx.x;
    // frame: fixed_w > 0 = the caller's frame; points outside it are an error (err != null: the
    // multi-GPU count images) or go to the outside list; otherwise the bounding box of the points
    // inside the kImgSide^2 image
    const bool fixed = fixed_w > 0;
    uint32_t w = fixed_w, h = fixed_h;
    if (!fixed) reduce_extent(ext, n_ext, s_red, w, h);
    const uint32_t lim_x = fixed ? w : kImgSide, lim_y = fixed ? h : kImgSide;
    const int64_t cells = (int64_t)w * h;
    if (blockIdx.x == 0 && tid == 0) {
        wh[0] = w;
        wh[1] = h;
    }
    parts = parts_used(parts, cells);
    if (m >= parts) return;
    const int64_t s0 = segs.n_segs * m / parts, s1 = segs.n_segs * (m + 1) / parts;
    const int64_t n_chunks = (cells + kHistChunk - 1) / kHistChunk;
    for (int64_t c = slot; c < (n_chunks > 0 ? n_chunks : 1); c += slots) {
        const int64_t lo = c * kHistChunk;
        const int n_loc = (int)((cells - lo) < kHistChunk ? (cells - lo) : kHistChunk);
        for (int i = tid; i < kHistChunk; i += kHistThreads) hist[i] = 0u;
        __syncthreads();
        // kHistSegs segments per trip, kHistUnroll x 1024 points of each: 16 independent loads per
        // lane in flight (a bench segment holds ~3150 points, so one segment per trip left the
        // trips latency-bound: 30 dependent trips per part)
        for (int64_t sg = s0; sg < s1; sg += kHistSegs) {
            int64_t cnt[kHistSegs], base[kHistSegs], cmax = 0;
            int32_t cl[kHistSegs];  // the counts' loads together (clamped segment, no branch between)
            if (segs.counts) {
#pragma unroll
                for (int i = 0; i < kHistSegs; ++i) cl[i] = segs.counts[sg + i < s1 ? sg + i : s1 - 1];
            } else {
#pragma unroll
                for (int i = 0; i < kHistSegs; ++i) cl[i] = (int32_t)segs.count(sg + i);
            }
#pragma unroll
            for (int i = 0; i < kHistSegs; ++i) {
                cnt[i] = sg + i < s1 ? cl[i] : 0;
                base[i] = (sg + i) * segs.stride;
                cmax = cnt[i] > cmax ? cnt[i] : cmax;
            }
            // per segment a buffer view (0 past its count): the 16 loads are unconditional, so all
            // of them are in flight together (a load under a per-lane condition waited for the last)
            __amdgpu_buffer_rsrc_t vs[kHistSegs];
#pragma unroll
            for (int i = 0; i < kHistSegs; ++i) vs[i] = ecc::buffer_view(xy + base[i], (uint32_t)cnt[i] * 4u);
            for (int64_t j0 = 0; j0 < cmax; j0 += kHistUnroll * kHistThreads) {
                uint32_t v[kHistSegs][kHistUnroll];
#pragma unroll
                for (int i = 0; i < kHistSegs; ++i)
#pragma unroll
                    for (int u = 0; u < kHistUnroll; ++u)
                        v[i][u] = ecc::buffer_load_u32(vs[i], (uint32_t)tid * 4u, (uint32_t)(j0 + u * kHistThreads) * 4u);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < kHistSegs; ++i)
#pragma unroll
                    for (int u = 0; u < kHistUnroll; ++u) {
                        if (j0 + u * kHistThreads + tid >= cnt[i]) continue;
                        const uint32_t x = v[i][u] & 0xffffu, y = v[i][u] >> 16;
                        if (x < lim_x && y < lim_y) {
                            const int64_t idx = (int64_t)y * w + x - lo;
                            if (idx >= 0 && idx < n_loc) atomicAdd(&hist[idx], 1u);
                        } else if (c == 0) {
                            if (err) *err = 1;
                            else outside[atomicAdd(n_outside, 1u)] = v[i][u];
                        }
                    }
            }
        }
        __syncthreads();
        uint32_t *out = partial + (int64_t)m * cells + lo;
        for (int i = tid; i < n_loc; i += kHistThreads) out[i] = hist[i];
        __syncthreads();
    }
}

__global__ void __launch_bounds__(kThreads)
kmeans_count_sum_kernel(const uint32_t *__restrict__ partial, int parts, const uint32_t *__restrict__ wh,
                        uint32_t *__restrict__ cnt) {
    const int64_t cells = (int64_t)wh[0] * wh[1];
    parts = parts_used(parts, cells);
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < cells; i += (int64_t)gridDim.x * kThreads) {
        uint32_t t = 0;
        int m = 0;
        for (; m + 8 <= parts; m += 8) {  // eight independent loads in flight
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = partial[(int64_t)(m + u) * cells + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) t += v[u];
        }
        for (; m < parts; ++m) t += partial[(int64_t)m * cells + i];
        cnt[i] = t;
    }
}

// One kmeans_step_kernel per Lloyd pass replaces "update, then label image": every workgroup
// re-derives the centroid update from the previous pass's accumulator replicas (a few hundred
// L2 reads), so no second launch and no grid-wide hand-off is needed.  Buffers alternate by pass:
// pass it accumulates into acc[it & 1] and labels with C_it, stored in cb[it & 1].  step(it)
// reads acc[(it-1) & 1] and cb[(it-1) & 1], so WG 0 alone may write cb[it & 1], the caller's
// centroids and the state, and zero acc[it & 1] (last read by step(it-1)).  The update
// arithmetic is kmeans_update_kernel's, in the same order.
struct StepArgs {
    const unsigned long long *acc_in;  // pass it-1's replicas (nullptr: no update in this step)
    unsigned long long *acc_zero;      // pass it's replicas, zeroed by WG 0
    const float *c_prev;               // C_{it-1} (or C_0 when acc_in is null)
    float *c_next;                     // cb[it & 1]
    float *cent;                       // the caller's centroids (final result)
    int n_copies, k;
    float thr, tol;
    bool final_pass;                   // after the last pass: update, then label image if wanted
    bool want_image;
};

// kPix: instead of a label image, the pass itself — (n, n*x, n*y) of every occupied pixel (cnt)
// and (1, x, y) of every outside point, into acc_out; WG 0 zeroes acc_zero, the replicas the
// NEXT pass accumulates into (three sets rotate: read by this pass's update, written, zeroed).
struct PixArgs {
    const uint32_t *cnt, *outside, *n_outside;
    unsigned long long *acc_out;
    const uint32_t *wh;  // bounding box (w, h), or null: reduce the per-WG extents
};

template <int K, bool kPix>
__global__ void __launch_bounds__(kThreads)
kmeans_step_kernel(StepArgs a, const uint32_t *__restrict__ ext, int n_ext, uint8_t *__restrict__ img,
                   KmState *st, PixArgs px) {
    // tol < 0 never sets done (fixed pass count): no dependent read of the state before the update
    const bool done_in = a.tol >= 0.f && st->done != 0;
    if (done_in && !a.final_pass) return;
    const int tid = threadIdx.x;
    __shared__ uint32_t s_wh[2][kThreads];
    __shared__ unsigned long long s_sum[3][K];
    __shared__ float s_c[2][K];
    __shared__ int s_done;
    const bool update = a.acc_in && !done_in;
    const float *c_src = done_in ? a.cent : a.c_prev;  // converged earlier: the caller's array is final
    if (update) {
        if (tid < 3 * a.k) {
            const int c = tid / 3, f = tid - 3 * c;
            unsigned long long t[kAccCopies], v = 0;  // all replicas' loads in flight together
#pragma unroll
            for (int r = 0; r < kAccCopies; ++r) t[r] = r < a.n_copies ? a.acc_in[r * kAccStride + 3 * c + f] : 0ull;
#pragma unroll
            for (int r = 0; r < kAccCopies; ++r) v += t[r];
            s_sum[f][c] = v;
        }
        if (blockIdx.x == 0)
            for (int i = tid; i < a.n_copies * kAccStride; i += kThreads) a.acc_zero[i] = 0ull;
        __syncthreads();
        if (tid < 64) {
            float shift = 0.f;
            if (tid < a.k) {
                const float ox = c_src[2 * tid], oy = c_src[2 * tid + 1];
                float nx = ox, ny = oy;
                const double n_pts = (double)s_sum[0][tid];
                if (n_pts > 0.0) {
                    nx = (float)((double)s_sum[1][tid] / n_pts);
                    ny = (float)((double)s_sum[2][tid] / n_pts);
                    shift = fmaxf(fabsf(nx - ox), fabsf(ny - oy));
                }
                s_c[0][tid] = nx;
                s_c[1][tid] = ny;
                if (blockIdx.x == 0) {
                    a.c_next[2 * tid] = nx;
                    a.c_next[2 * tid + 1] = ny;
                    a.cent[2 * tid] = nx;
                    a.cent[2 * tid + 1] = ny;
                }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) shift = fmaxf(shift, __shfl_xor(shift, o));
            if (tid == 0) {
                const int done = (a.tol >= 0.f && shift <= a.tol) ? 1 : 0;
                s_done = done;
                if (blockIdx.x == 0) {
                    st->iters += 1;
                    st->done = done;
                }
            }
        }
    } else {
        if (tid < a.k) {
            s_c[0][tid] = c_src[2 * tid];
            s_c[1][tid] = c_src[2 * tid + 1];
            if (blockIdx.x == 0 && !done_in) {
                a.c_next[2 * tid] = s_c[0][tid];
                a.c_next[2 * tid + 1] = s_c[1][tid];
            }
        }
        if (tid == 0) s_done = done_in ? 1 : 0;
    }
    if (px.wh) {  // bounding box stored by kmeans_count_kernel
        if (tid == 0) {
            s_wh[0][0] = px.wh[0];
            s_wh[1][0] = px.wh[1];
        }
        __syncthreads();
    } else {  // bounding box = max over the extent kernel's per-WG maxima
        uint32_t p = 0, q = 0;
        for (int i = tid; i < n_ext; i += kThreads) { p = max(p, ext[2 * i]); q = max(q, ext[2 * i + 1]); }
        s_wh[0][tid] = p;
        s_wh[1][tid] = q;
        __syncthreads();
        for (int o = kThreads / 2; o > 0; o >>= 1) {
            if (tid < o) {
                s_wh[0][tid] = max(s_wh[0][tid], s_wh[0][tid + o]);
                s_wh[1][tid] = max(s_wh[1][tid], s_wh[1][tid + o]);
            }
            __syncthreads();
        }
    }
    // a pass that converged runs no further accumulation: its image is only needed for labels
    if (a.final_pass ? !a.want_image : s_done != 0) return;
    float cx[K], cy[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        cx[i] = uniform_f32(i < a.k ? s_c[0][i] : __builtin_inff());
        cy[i] = uniform_f32(i < a.k ? s_c[1][i] : __builtin_inff());
    }
    const uint32_t w = s_wh[0][0], h = s_wh[1][0];
    const int64_t cells = (int64_t)w * h;
    if constexpr (!kPix) {
        for (uint32_t c = blockIdx.x * kThreads + tid; c < (uint32_t)cells; c += gridDim.x * kThreads) {
            const uint32_t y = c / w, x = c - y * w;  // cells <= kImgSide^2: 32-bit index
            img[(int64_t)y * kImgSide + x] = (uint8_t)assign_fast<K>((float)x, (float)y, cx, cy, a.thr);
        }
    } else {
        __shared__ unsigned long long w_acc[3][K];
        for (int i = tid; i < 3 * K; i += kThreads) (&w_acc[0][0])[i] = 0ull;
        __syncthreads();
        for (uint32_t c = blockIdx.x * kThreads + tid; c < (uint32_t)cells; c += gridDim.x * kThreads) {
            const uint32_t y = c / w, x = c - y * w;  // cells <= kImgSide^2: 32-bit index
            const uint32_t n = px.cnt[c];
            if (!n) continue;
            const uint32_t l = assign_fast<K>((float)x, (float)y, cx, cy, a.thr);
            if (l >= (uint32_t)K) continue;
            atomicAdd(&w_acc[0][l], (unsigned long long)n);
            atomicAdd(&w_acc[1][l], (unsigned long long)n * x);
            atomicAdd(&w_acc[2][l], (unsigned long long)n * y);
        }
        const uint32_t n_out = *px.n_outside;  // (cnt is compact: cnt[y * w + x])
        for (uint32_t i = blockIdx.x * kThreads + tid; i < n_out; i += gridDim.x * kThreads) {
            const uint32_t v = px.outside[i], x = v & 0xffffu, y = v >> 16;
            const uint32_t l = assign_fast<K>((float)x, (float)y, cx, cy, a.thr);
            if (l >= (uint32_t)K) continue;
            atomicAdd(&w_acc[0][l], 1ull);
            atomicAdd(&w_acc[1][l], (unsigned long long)x);
            atomicAdd(&w_acc[2][l], (unsigned long long)y);
        }
        __syncthreads();
        if (tid < 3 * a.k) {
            const int f = tid / a.k, c = tid - f * a.k;
            const unsigned long long sum = w_acc[f][c];
            if (sum) atomicAdd(&px.acc_out[(int)(blockIdx.x % a.n_copies) * kAccStride + 3 * c + f], sum);
        }
    }
}

template <int K, bool kPix>
void launch_step(dim3 grid, hipStream_t s, const StepArgs &a, const uint32_t *ext, int n_ext, uint8_t *img,
                 KmState *st, const PixArgs &px) {
    hipLaunchKernelGGL((kmeans_step_kernel<K, kPix>), grid, dim3(kThreads), 0, s, a, ext, n_ext, img, st, px);
}

// Launch helpers for the fast path (k <= kFastMaxK); false when k needs the generic kernel.
template <bool kAccumulate>
bool launch_fast(int k, dim3 grid, hipStream_t s, const uint32_t *xy, const Segs &segs, const float *cent,
                 float thr, unsigned long long *acc, int n_copies, const KmState *st, uint8_t *labels) {
    if (k > kFastMaxK) return false;
    if (k <= 16)
        hipLaunchKernelGGL((kmeans_fast_kernel<16, kAccumulate>), grid, dim3(kThreads), 0, s, xy, segs, cent, k, thr,
                           acc, n_copies, st, labels);
    else
        hipLaunchKernelGGL((kmeans_fast_kernel<32, kAccumulate>), grid, dim3(kThreads), 0, s, xy, segs, cent, k, thr,
                           acc, n_copies, st, labels);
    return true;
}

int grid_for(int64_t units) {
    int64_t g = units < kMaxGrid ? units : kMaxGrid;
    return g < 1 ? 1 : (int)g;
}

}  // namespace

ECC_API void ecc_kmeans_cfg_default(ecc_kmeans_cfg *cfg) {
    if (!cfg) return;
    cfg->k = 16;            // BASELINE.json C3 (the reference hard-codes 8, assign_to_centers.cl:14)
    cfg->max_iters = 20;
    cfg->threshold = 50.f;  // assign_to_centers.cl:11
    cfg->tol = 1e-3f;
}

static int kmeans_check(const ecc_ctx *ctx, const ecc_kmeans_cfg *cfg, const float *centroids) {
    if (!ctx || !cfg || !centroids) return ECC_ERR_INVALID;
    if (cfg->k < 1 || cfg->k > kMaxK || cfg->max_iters < 0) return ECC_ERR_INVALID;
    return ECC_OK;
}

static int kmeans_run_xy16_impl(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                                const int32_t *seg_counts, int32_t frame_w, int32_t frame_h,
                                const ecc_kmeans_cfg *cfg, float *centroids, uint8_t *labels,
                                int32_t *iters_out, ecc_stream_t stream) {
    int rc = kmeans_check(ctx, cfg, centroids);
    if (rc) return rc;
    if (n_segs < 0 || seg_stride < 1) return ECC_ERR_INVALID;
    if (frame_w < 0 || frame_h < 0 || frame_w > kImgSide || frame_h > kImgSide || (frame_w == 0) != (frame_h == 0))
        return ECC_ERR_INVALID;
    Segs segs{seg_counts, n_segs, seg_stride, n_segs * seg_stride};
    if (!seg_counts) {
        // dense array of n_segs*seg_stride points: re-cut into 16384-point segments
        const int64_t n = n_segs * seg_stride;
        segs.stride = 16384;
        segs.n_segs = (n + segs.stride - 1) / segs.stride;
        segs.n_dense = n;
    }
    if (segs.n_segs > 0 && !xy) return ECC_ERR_INVALID;
    // per-WG packed counts must stay < 2^24 points (sum_x < 2^40)
    const int grid = grid_for(segs.n_segs);
    if (segs.n_segs * segs.stride / grid >= (1ll << 24)) return ECC_ERR_INVALID;
    // workspace: three sets of kAccCopies accumulator replicas (rotating by pass; the generic path
    // uses copy 0 of set 0), the state, the centroid history cb[2], the per-WG extents, the label
    // image, the per-pixel counts and the outside-point list
    constexpr size_t kAccBytes = (size_t)kAccCopies * kAccStride * 8;
    const size_t off_st = 3 * kAccBytes;
    const size_t off_cb = off_st + 64;
    const size_t off_ext = ecc::align_up(off_cb + 2 * 2 * kMaxK * sizeof(float), 256);
    const size_t off_img = ecc::align_up(off_ext + (size_t)grid * 8, 256);
    const size_t off_cnt = ecc::align_up(off_img + (size_t)kImgSide * kImgSide, 256);
    const size_t off_part = off_cnt + (size_t)kImgSide * kImgSide * 4;
    int parts, slots;
    count_layout(segs.n_segs, (int64_t)frame_w * frame_h, parts, slots);
    const size_t off_out = off_part + (size_t)kHistBudget * 4;
    const int64_t n_pts_max = segs.n_segs * segs.stride;
    rc = ecc::ws_reserve(ctx, off_out + 256 + (size_t)n_pts_max * 4);
    if (rc) return rc;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    char *ws = static_cast<char *>(ctx->ws);
    unsigned long long *accb[3] = {reinterpret_cast<unsigned long long *>(ws),
                                   reinterpret_cast<unsigned long long *>(ws + kAccBytes),
                                   reinterpret_cast<unsigned long long *>(ws + 2 * kAccBytes)};
    auto *st = reinterpret_cast<KmState *>(ws + off_st);
    float *cb[2] = {reinterpret_cast<float *>(ws + off_cb), reinterpret_cast<float *>(ws + off_cb) + 2 * kMaxK};
    auto *ext = reinterpret_cast<uint32_t *>(ws + off_ext);
    auto *img = reinterpret_cast<uint8_t *>(ws + off_img);
    auto *cnt = reinterpret_cast<uint32_t *>(ws + off_cnt);
    auto *partial = reinterpret_cast<uint32_t *>(ws + off_part);
    auto *n_out = reinterpret_cast<uint32_t *>(ws + off_out);
    auto *wh = n_out + 1;
    auto *outside = reinterpret_cast<uint32_t *>(ws + off_out + 256);
    ECC_CHECK_HIP(ctx, hipMemsetAsync(ws, 0, off_st + 64, s), "memset(kmeans acc)");
    if (segs.n_segs == 0) {
        if (iters_out)
            ECC_CHECK_HIP(ctx, hipMemcpyAsync(iters_out, &st->iters, 4, hipMemcpyDeviceToDevice, s), "copy iters");
        return ECC_OK;
    }
    if (cfg->k > kFastMaxK) {  // generic kernel: assign per point, separate update launch
        for (int it = 0; it < cfg->max_iters; ++it) {
            {
                ECC_TIMED(ctx, s, "kmeans_xy16_kernel");
                hipLaunchKernelGGL(kmeans_xy16_kernel<true>, dim3(grid), dim3(kThreads), 0, s, xy, segs, centroids,
                                   cfg->k, cfg->threshold, accb[0], st, (uint8_t *)nullptr);
            }
            {
                ECC_TIMED(ctx, s, "kmeans_update_kernel");
                hipLaunchKernelGGL(kmeans_update_kernel<unsigned long long>, dim3(1), dim3(64), 0, s, accb[0], 1,
                                   centroids, cfg->k, cfg->tol, st);
            }
        }
        ECC_CHECK_LAUNCH(ctx, "kmeans_xy16 iteration");
        if (labels) {
            ECC_TIMED(ctx, s, "kmeans_xy16_labels");
            hipLaunchKernelGGL(kmeans_xy16_kernel<false>, dim3(grid), dim3(kThreads), 0, s, xy, segs, centroids,
                               cfg->k, cfg->threshold, accb[0], st, labels);
            ECC_CHECK_LAUNCH(ctx, "kmeans_xy16 labels");
        }
    } else {
        // per-pixel passes: the points are counted per pixel once, every Lloyd pass is ONE launch
        // over the occupied pixels of the bounding box (+ the outside list); labels come from the
        // final label image
        const int grid_pts = (int)std::min<int64_t>(segs.n_segs, kMaxGridPts);
        ECC_CHECK_HIP(ctx, hipMemsetAsync(n_out, 0, 4, s), "memset(kmeans outside)");
        if (frame_w == 0) {  // no frame given: the points' bounding box
            ECC_TIMED(ctx, s, "kmeans_extent_kernel");
            hipLaunchKernelGGL(kmeans_extent_kernel, dim3(grid), dim3(kThreads), 0, s, xy, segs, ext);
        }
        {
            ECC_TIMED(ctx, s, "kmeans_count_kernel");
            static bool lds_ok = false;
            if (!lds_ok) {
                ECC_CHECK_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void *>(&kmeans_count_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, kHistChunk * 4),
                              "kmeans_count LDS");
                lds_ok = true;
            }
            hipLaunchKernelGGL(kmeans_count_kernel, dim3(count_grid(parts, slots)), dim3(kHistThreads), kHistChunk * 4,
                               s, xy, segs, ext, grid, parts, slots, partial, wh, outside, n_out, (uint32_t)frame_w,
                               (uint32_t)frame_h, (int32_t *)nullptr);
        }
        {
            ECC_TIMED(ctx, s, "kmeans_count_sum_kernel");
            hipLaunchKernelGGL(kmeans_count_sum_kernel, dim3(1024), dim3(kThreads), 0, s, partial, parts, wh, cnt);
        }
        auto step = [&](int it, bool final_pass) {
            StepArgs a{};
            a.acc_in = it ? accb[(it - 1) % 3] : nullptr;
            a.acc_zero = accb[(it + 1) % 3];
            a.c_prev = it ? cb[(it - 1) & 1] : centroids;
            a.c_next = cb[it & 1];
            a.cent = centroids;
            a.n_copies = kAccCopies;
            a.k = cfg->k;
            a.thr = cfg->threshold;
            a.tol = cfg->tol;
            a.final_pass = final_pass;
            a.want_image = labels != nullptr;
            const PixArgs px{cnt, outside, n_out, accb[it % 3], wh};
            if (final_pass) {
                ECC_TIMED(ctx, s, "kmeans_step_kernel");
                if (cfg->k <= 16) launch_step<16, false>(dim3(512), s, a, ext, grid, img, st, px);
                else launch_step<32, false>(dim3(512), s, a, ext, grid, img, st, px);
            } else {
                ECC_TIMED(ctx, s, "kmeans_pixel_pass");
                if (cfg->k <= 16) launch_step<16, true>(dim3(kPixGrid), s, a, ext, grid, img, st, px);
                else launch_step<32, true>(dim3(kPixGrid), s, a, ext, grid, img, st, px);
            }
        };
        for (int it = 0; it < cfg->max_iters; ++it) step(it, false);
        if (cfg->max_iters > 0 || labels) step(cfg->max_iters, true);  // last update (+ image for labels)
        ECC_CHECK_LAUNCH(ctx, "kmeans_xy16 iteration");
        if (labels) {
            ECC_TIMED(ctx, s, "kmeans_xy16_labels");
            const int64_t frame_px = (int64_t)frame_w * frame_h;
            const int64_t frame_lds = (int64_t)ecc::align_up((size_t)frame_w, 4) * frame_h;
            if (frame_px > 0 && frame_lds <= kLabLdsBytes) {  // the frame's label image fits in LDS
                const int lds = (int)frame_lds;
                const dim3 g((unsigned)std::min<int64_t>((segs.n_segs + 3) / 4, ECC_KM_LAB_GRID));
                static bool lab_lds_ok = false;
                if (!lab_lds_ok) {
                    ECC_CHECK_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void *>(&kmeans_lds_labels_kernel<16>),
                                                           hipFuncAttributeMaxDynamicSharedMemorySize, kLabLdsBytes),
                                  "kmeans labels LDS");
                    ECC_CHECK_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void *>(&kmeans_lds_labels_kernel<32>),
                                                           hipFuncAttributeMaxDynamicSharedMemorySize, kLabLdsBytes),
                                  "kmeans labels LDS");
                    lab_lds_ok = true;
                }
                if (cfg->k <= 16)
                    hipLaunchKernelGGL(kmeans_lds_labels_kernel<16>, g, dim3(kLabLdsThreads), lds, s, xy, segs,
                                       centroids, cfg->k, cfg->threshold, img, wh, labels);
                else
                    hipLaunchKernelGGL(kmeans_lds_labels_kernel<32>, g, dim3(kLabLdsThreads), lds, s, xy, segs,
                                       centroids, cfg->k, cfg->threshold, img, wh, labels);
            } else if (cfg->k <= 16)
                hipLaunchKernelGGL(kmeans_img_labels_kernel<16>, dim3(grid_pts), dim3(kThreads), 0, s, xy, segs,
                                   centroids, cfg->k, cfg->threshold, img, wh, labels);
            else
                hipLaunchKernelGGL(kmeans_img_labels_kernel<32>, dim3(grid_pts), dim3(kThreads), 0, s, xy, segs,
                                   centroids, cfg->k, cfg->threshold, img, wh, labels);
            ECC_CHECK_LAUNCH(ctx, "kmeans_xy16 labels");
        }
    }
    if (iters_out)
        ECC_CHECK_HIP(ctx, hipMemcpyAsync(iters_out, &st->iters, 4, hipMemcpyDeviceToDevice, s),
                      "copy iters");
    return ECC_OK;
}

static int kmeans_run_f32_impl(ecc_ctx *ctx, const float *xy, int64_t n_points, const ecc_kmeans_cfg *cfg,
                               int method, float *centroids, uint8_t *labels, int32_t *iters_out, ecc_stream_t stream) {
    int rc = kmeans_check(ctx, cfg, centroids);
    if (rc) return rc;
    if (n_points < 0 || (n_points > 0 && !xy) || method < 0 || method > 3) return ECC_ERR_INVALID;
    if (method != 0 && cfg->k > kFastMaxK) return ECC_ERR_INVALID;  // the engines take k <= 32
    if ((reinterpret_cast<uintptr_t>(xy) & 7) != 0) return ECC_ERR_INVALID;  // float2 loads
    const bool fast = cfg->k <= kFastMaxK;
    const int n_copies = fast ? kAccCopies : 1;
    const int eng = method == 0 ? 1 : method;  // auto = the vector engine (measured faster)
    // the vector engine's pair kernel (16-B aligned points) runs on the candidate table
    const bool use_lut = fast && eng == 1 && n_points > 0 && (reinterpret_cast<uintptr_t>(xy) & 15) == 0;
    const size_t acc_bytes = (size_t)n_copies * kAccStride * 8;
    // workspace: accumulator set 0 | set 1 (the table path ping-pongs) | state | box | grid | table
    const size_t st_off = 2 * acc_bytes, box_off = st_off + 64, geom_off = box_off + 16 * kBoxBlocks, lut_off = geom_off + 64;
    const size_t ws_bytes = lut_off + (size_t)kLutCells * 4;
    rc = ecc::ws_reserve(ctx, ws_bytes);
    if (rc) return rc;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    char *ws = reinterpret_cast<char *>(ctx->ws);
    auto *acc = reinterpret_cast<double *>(ws);
    auto *st = reinterpret_cast<KmState *>(ws + st_off);
    auto *box = reinterpret_cast<uint32_t *>(ws + box_off);
    auto *geom = reinterpret_cast<LutGeom *>(ws + geom_off);
    auto *lut = reinterpret_cast<uint32_t *>(ws + lut_off);
    ECC_CHECK_HIP(ctx, hipMemsetAsync(ctx->ws, 0, box_off, s), "memset(kmeans acc)");
    const char *name = eng == 3 ? "kmeans_f32_mfma32_kernel" : eng == 2 ? "kmeans_f32_mfma_kernel" : "kmeans_f32_vec_kernel";
    const int grid = fast ? (int)std::max<int64_t>(1, std::min<int64_t>((n_points + 255) / 256, 4096))
                          : grid_for((n_points + kThreads - 1) / kThreads);
    const float thr2 = sqrt_threshold(cfg->threshold);
    if (use_lut) {
        {
            ECC_TIMED(ctx, s, "kmeans_bbox_sample_kernel");
            hipLaunchKernelGGL(kmeans_bbox_sample_kernel, dim3(kBoxBlocks), dim3(kThreads), 0, s,
                               reinterpret_cast<const float2 *>(xy), n_points, box);
        }
        {
            ECC_TIMED(ctx, s, "kmeans_update_lut_kernel");
            hipLaunchKernelGGL(kmeans_update_lut_kernel, dim3(kLutBlocks), dim3(kThreads), 0, s, acc, acc, n_copies,
                               centroids, cfg->k, cfg->tol, st, -1, box, geom, lut, thr2);
        }
        // one round of resident workgroups, as many per CU as registers and LDS allow (a
        // latency-bound stream: the labels pass took 104 us at four per CU, 93 at five): the
        // accumulate pass 5 (k <= 16: 86 VGPRs, 30 KB) or 4 (k <= 32: 35 KB of slots and table),
        // the labels pass 6 (80 VGPRs, 25 KB)
        auto rgrid = [&](int per_cu) {
            return (int)std::max<int64_t>(1, std::min<int64_t>((n_points + 255) / 256, (int64_t)per_cu * ctx->n_cu));
        };
        const int lgrid = rgrid(cfg->k <= 16 ? ECC_KM_LUT_WG_PER_CU : 4);
        const int lgrid_lab = rgrid(ECC_KM_LAB_WG_PER_CU);
        for (int it = 0; it < cfg->max_iters; ++it) {
            double *acc_it = acc + (size_t)(it & 1) * n_copies * kAccStride;
            double *acc_next = acc + (size_t)((it + 1) & 1) * n_copies * kAccStride;
            {
                ECC_TIMED(ctx, s, name);
                launch_f32_fast<true>(cfg->k, eng, dim3(lgrid), s, xy, n_points, centroids, cfg->threshold, acc_it,
                                      n_copies, st, nullptr, geom, lut);
            }
            {
                ECC_TIMED(ctx, s, "kmeans_update_lut_kernel");
                hipLaunchKernelGGL(kmeans_update_lut_kernel, dim3(kLutBlocks), dim3(kThreads), 0, s, acc_it,
                                   acc_next, n_copies, centroids, cfg->k, cfg->tol, st, it, box, geom, lut, thr2);
            }
        }
        ECC_CHECK_LAUNCH(ctx, "kmeans_f32 iteration");
        if (labels) {
            {
                ECC_TIMED(ctx, s, "kmeans_f32_labels");
                const bool lab_ok = (reinterpret_cast<uintptr_t>(labels) & 1) == 0;
                launch_f32_fast<false>(cfg->k, eng, dim3(lab_ok ? lgrid_lab : grid), s, xy, n_points, centroids, cfg->threshold, nullptr,
                                       1, st, labels, lab_ok ? geom : nullptr, lut);
            }
            ECC_CHECK_LAUNCH(ctx, "kmeans_f32 labels");
        }
        if (iters_out)
            ECC_CHECK_HIP(ctx, hipMemcpyAsync(iters_out, &st->iters, 4, hipMemcpyDeviceToDevice, s), "copy iters");
        return ECC_OK;
    }
    for (int it = 0; it < cfg->max_iters && n_points > 0; ++it) {
        {
            ECC_TIMED(ctx, s, fast ? name : "kmeans_f32_kernel");
            if (!launch_f32_fast<true>(cfg->k, eng, dim3(grid), s, xy, n_points, centroids, cfg->threshold, acc,
                                       n_copies, st, nullptr))
                hipLaunchKernelGGL(kmeans_f32_kernel<true>, dim3(grid), dim3(kThreads), 0, s, xy, n_points,
                                   centroids, cfg->k, cfg->threshold, acc, st, (uint8_t *)nullptr);
        }
        {
            ECC_TIMED(ctx, s, "kmeans_update_kernel");
            hipLaunchKernelGGL(kmeans_update_kernel<double>, dim3(1), dim3(64), 0, s, acc, n_copies, centroids,
                               cfg->k, cfg->tol, st);
        }
    }
    ECC_CHECK_LAUNCH(ctx, "kmeans_f32 iteration");
    if (labels && n_points > 0) {
        {
            ECC_TIMED(ctx, s, "kmeans_f32_labels");
            if (!launch_f32_fast<false>(cfg->k, eng, dim3(grid), s, xy, n_points, centroids, cfg->threshold,
                                        nullptr, 1, st, labels))
                hipLaunchKernelGGL(kmeans_f32_kernel<false>, dim3(grid), dim3(kThreads), 0, s, xy, n_points,
                                   centroids, cfg->k, cfg->threshold, acc, st, labels);
        }
        ECC_CHECK_LAUNCH(ctx, "kmeans_f32 labels");
    }
    if (iters_out)
        ECC_CHECK_HIP(ctx, hipMemcpyAsync(iters_out, &st->iters, 4, hipMemcpyDeviceToDevice, s),
                      "copy iters");
    return ECC_OK;
}

ECC_API int ecc_kmeans_run_xy16(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                                const int32_t *seg_counts, const ecc_kmeans_cfg *cfg, float *centroids,
                                uint8_t *labels, int32_t *iters_out, ecc_stream_t stream) {
    return kmeans_run_xy16_impl(ctx, xy, n_segs, seg_stride, seg_counts, 0, 0, cfg, centroids, labels, iters_out,
                                stream);
}

ECC_API int ecc_kmeans_run_xy16_frame(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                                      const int32_t *seg_counts, int32_t frame_w, int32_t frame_h,
                                      const ecc_kmeans_cfg *cfg, float *centroids, uint8_t *labels,
                                      int32_t *iters_out, ecc_stream_t stream) {
    if (frame_w < 1 || frame_h < 1) return ECC_ERR_INVALID;
    return kmeans_run_xy16_impl(ctx, xy, n_segs, seg_stride, seg_counts, frame_w, frame_h, cfg, centroids, labels,
                                iters_out, stream);
}

ECC_API int ecc_kmeans_run_f32(ecc_ctx *ctx, const float *xy, int64_t n_points,
                               const ecc_kmeans_cfg *cfg, float *centroids, uint8_t *labels,
                               int32_t *iters_out, ecc_stream_t stream) {
    return kmeans_run_f32_impl(ctx, xy, n_points, cfg, 0, centroids, labels, iters_out, stream);
}

ECC_API int ecc_kmeans_run_f32_engine(ecc_ctx *ctx, const float *xy, int64_t n_points,
                                      const ecc_kmeans_cfg *cfg, int32_t engine, float *centroids,
                                      uint8_t *labels, int32_t *iters_out, ecc_stream_t stream) {
    return kmeans_run_f32_impl(ctx, xy, n_points, cfg, engine, centroids, labels, iters_out, stream);
}

ECC_API int ecc_kmeans_assign_f32(ecc_ctx *ctx, const float *xy, int64_t n_points,
                                  const float *centroids, int32_t k, float threshold,
                                  uint8_t *labels, ecc_stream_t stream) {
    if (!ctx || !centroids || !labels || k < 1 || k > kMaxK || n_points < 0) return ECC_ERR_INVALID;
    if (n_points == 0) return ECC_OK;
    if (!xy) return ECC_ERR_INVALID;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    const int grid = grid_for((n_points + kThreads - 1) / kThreads);
    {
        ECC_TIMED(ctx, ecc::as_stream(stream), "kmeans_f32_kernel");
        hipLaunchKernelGGL(kmeans_f32_kernel<false>, dim3(grid), dim3(kThreads), 0,
                           ecc::as_stream(stream), xy, n_points, centroids, k, threshold,
                           (double *)nullptr, (const KmState *)nullptr, labels);
    }
    ECC_CHECK_LAUNCH(ctx, "kmeans assign");
    return ECC_OK;
}

// ---- split form (multi-GPU: accumulate -> all-reduce(acc) -> update) ---------------------
static Segs make_segs(int64_t n_segs, int64_t seg_stride, const int32_t *seg_counts) {
    Segs segs{seg_counts, n_segs, seg_stride, n_segs * seg_stride};
    if (!seg_counts) {
        const int64_t n = n_segs * seg_stride;
        segs.stride = 16384;
        segs.n_segs = (n + segs.stride - 1) / segs.stride;
        segs.n_dense = n;
    }
    return segs;
}

ECC_API int ecc_kmeans_accumulate_xy16(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs,
                                       int64_t seg_stride, const int32_t *seg_counts,
                                       const float *centroids, int32_t k, float threshold,
                                       uint64_t *acc, const int32_t *state, ecc_stream_t stream) {
    if (!ctx || !centroids || !acc || !state || k < 1 || k > kMaxK || n_segs < 0 || seg_stride < 1)
        return ECC_ERR_INVALID;
    const Segs segs = make_segs(n_segs, seg_stride, seg_counts);
    if (segs.n_segs == 0) return ECC_OK;
    if (!xy) return ECC_ERR_INVALID;
    const int grid = grid_for(segs.n_segs);
    if (segs.n_segs * segs.stride / grid >= (1ll << 24)) return ECC_ERR_INVALID;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    {
        ECC_TIMED(ctx, s, "kmeans_xy16_kernel");
        auto *acc64 = reinterpret_cast<unsigned long long *>(acc);
        auto *km = reinterpret_cast<const KmState *>(state);
        if (!launch_fast<true>(k, dim3(grid), s, xy, segs, centroids, threshold, acc64, 1, km, nullptr))
            hipLaunchKernelGGL(kmeans_xy16_kernel<true>, dim3(grid), dim3(kThreads), 0, s, xy, segs,
                               centroids, k, threshold, acc64, km, (uint8_t *)nullptr);
    }
    ECC_CHECK_LAUNCH(ctx, "kmeans accumulate");
    return ECC_OK;
}

ECC_API int ecc_kmeans_update(ecc_ctx *ctx, uint64_t *acc, float *centroids, int32_t k, float tol,
                              int32_t *state, ecc_stream_t stream) {
    if (!ctx || !acc || !centroids || !state || k < 1 || k > kMaxK) return ECC_ERR_INVALID;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    {
        ECC_TIMED(ctx, s, "kmeans_update_kernel");
        hipLaunchKernelGGL(kmeans_update_kernel<unsigned long long>, dim3(1), dim3(64), 0, s,
                           reinterpret_cast<unsigned long long *>(acc), 1, centroids, k, tol,
                           reinterpret_cast<KmState *>(state));
    }
    ECC_CHECK_LAUNCH(ctx, "kmeans update");
    return ECC_OK;
}

ECC_API int ecc_kmeans_labels_xy16(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs,
                                   int64_t seg_stride, const int32_t *seg_counts,
                                   const float *centroids, int32_t k, float threshold,
                                   uint8_t *labels, ecc_stream_t stream) {
    if (!ctx || !centroids || !labels || k < 1 || k > kMaxK || n_segs < 0 || seg_stride < 1)
        return ECC_ERR_INVALID;
    const Segs segs = make_segs(n_segs, seg_stride, seg_counts);
    if (segs.n_segs == 0) return ECC_OK;
    if (!xy) return ECC_ERR_INVALID;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    {
        ECC_TIMED(ctx, s, "kmeans_xy16_labels");
        const dim3 grid(grid_for(segs.n_segs));
        if (!launch_fast<false>(k, grid, s, xy, segs, centroids, threshold, nullptr, 1, nullptr, labels))
            hipLaunchKernelGGL(kmeans_xy16_kernel<false>, grid, dim3(kThreads), 0, s, xy, segs, centroids, k,
                               threshold, (unsigned long long *)nullptr, (const KmState *)nullptr, labels);
    }
    ECC_CHECK_LAUNCH(ctx, "kmeans labels");
    return ECC_OK;
}

// ---- "ref_compat" k-means loop ----------------------------------------
// The reference's host loop KM/assign_to_centers2.c:184-548 over its three kernels, with its
// quirks: 8 centres; assign_to_centers (:10-27 of the .cl) labels a point, assign_data_cluster
// appends it to its cluster's bin of 2048 slots (x in [0, 2048), y in [2048, 4096) of the bin's
// 4096 floats; a point past the 2048th is counted but not stored); the bins are zeroed once
// (:133-137) and never cleared, so a bin keeps the previous passes' values past its count (Q8);
// reduction_scalar sums each 1024-float chunk as a pairwise tree; the update reads the chunk sums
// as ss[j], ss[j+1] (x) and ss[j+2], ss[j+3] (y) for j = 2c (:509-512, Q7), divides by the bin
// count (0: inf / NaN), and replaces coordinate j only while |new - old| — C's int abs of the
// float — exceeds the running maximum (:525-532, Q9); the loop restarts while that maximum is
// > 10 (:545-548).  The reference appends in atomic order; here a bin is filled in point-index
// order (oracle/oracle.cpp orc_kmeans_refcompat, pinned pass by pass against the reference kernels
// run on the box: tests/test_ref_opencl.py).  ONE workgroup: the 128 KB of bins live in LDS for
// the whole loop, the points are taken in 16 rounds of 1024 (a bin slot is the point's rank in
// its cluster by ballots and per-wave counts), and wave w sums chunks w and w + 16 with each lane
// holding the chunk's elements lane + 64 i (the tree's first four levels inside a lane, the last
// six by shuffles).
constexpr int kRcThreads = 1024;
constexpr int kRcPer = 16;                         // points per thread
constexpr int kRcMaxPts = kRcThreads * kRcPer;     // 16384 = 8 bins of 2048
constexpr int kRcBinFloats = 8 * 4096;

// C's int abs of a float (the reference's `abs` on float, :526-527): truncation to int; an
// out-of-range or NaN value converts to INT_MIN on the reference's x86-64 (cvttss2si), whose abs
// stays INT_MIN (the oracle's ref_int_abs)
__device__ __forceinline__ float ref_int_abs_dev(float d) {
    if (!(d > -2147483648.f && d < 2147483648.f)) return -2147483648.f;
    const int i = __float2int_rz(d);
    return __int2float_rn(i < 0 ? -i : i);
}

__global__ void __launch_bounds__(kRcThreads)
kmeans_refcompat_kernel(const float *__restrict__ xy, int n, float *__restrict__ cent16, int max_passes,
                        int32_t *__restrict__ passes_out, int32_t *__restrict__ bin_counts_out,
                        float *__restrict__ sums_out) {
    extern __shared__ float bins[];  // [8][4096]
    __shared__ float2 s_c[8];
    __shared__ float s_ss[32];
    __shared__ int s_wc[kRcThreads / 64][8];  // a round's cluster counts per wave
    __shared__ int s_run[8];                  // the pass's cluster counts so far (cluster_index)
    __shared__ int s_again;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int i = tid; i < kRcBinFloats; i += kRcThreads) bins[i] = 0.f;  // :133-137, once
    if (tid < 8) s_c[tid] = make_float2(cent16[2 * tid], cent16[2 * tid + 1]);
    int passes = 0;
    for (;;) {
        if (tid < 8) s_run[tid] = 0;
        __syncthreads();
        // assign_to_centers, then assign_data_cluster in point-index order: round u takes points
        // u * 1024 + thread, so a point's slot is its cluster's count over the earlier rounds,
        // the earlier waves of its round and the earlier lanes of its wave
        for (int u = 0; u < kRcPer; ++u) {
            const int g = u * kRcThreads + tid;
            float x = 0.f, y = 0.f;
            uint32_t c = 127u;
            if (g < n) {
                x = xy[2 * g];
                y = xy[2 * g + 1];
                const uint32_t a = assign_point(x, y, s_c, 8, 50.f);
                c = a == 255u ? 127u : a;  // (2c)/2 of the reference's label: 255/2 = 127, no bin
            }
            int rank = 0;
#pragma unroll
            for (int cc = 0; cc < 8; ++cc) {
                const uint64_t m = __ballot(c == (uint32_t)cc);
                if (c == (uint32_t)cc) rank = __popcll(m & lt);
                if (lane == 0) s_wc[wave][cc] = __popcll(m);
            }
            __syncthreads();
            if (c < 8u) {
                int idx = s_run[c] + rank;
                for (int w = 0; w < wave; ++w) idx += s_wc[w][c];
                if (idx < 2048) {  // counted but not stored past the bin (no check in the kernel)
                    bins[c * 4096 + idx] = x;
                    bins[c * 4096 + 2048 + idx] = y;
                }
            }
            __syncthreads();
            if (tid < 8) {
                int tot = 0;
#pragma unroll
                for (int w = 0; w < kRcThreads / 64; ++w) tot += s_wc[w][tid];
                s_run[tid] += tot;
            }
        }
        __syncthreads();
        // reduction_scalar: chunk sums, buf[l] += buf[l + s] for s = 512 .. 1
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int chunk = wave + 16 * h;
            float v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = bins[chunk * 1024 + lane + 64 * i];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = __fadd_rn(v[i], v[i + 8]);  // s = 512
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = __fadd_rn(v[i], v[i + 4]);  // 256
            v[0] = __fadd_rn(v[0], v[2]);                                   // 128
            v[1] = __fadd_rn(v[1], v[3]);
            v[0] = __fadd_rn(v[0], v[1]);                                   // 64
#pragma unroll
            for (int sft = 32; sft > 0; sft >>= 1) {                        // 32 .. 1
                const float o = __shfl_down(v[0], sft);
                if (lane < sft) v[0] = __fadd_rn(v[0], o);
            }
            if (lane == 0) s_ss[chunk] = v[0];
        }
        __syncthreads();
        if (tid == 0) {  // the update (:509-532) and the restart test (:545-548)
            float nc[16], c16[16];
#pragma unroll
            for (int j = 0; j < 16; j += 2) {
                const float cn = __int2float_rn(s_run[j / 2]);
                nc[j] = __fdiv_rn(__fadd_rn(s_ss[j], s_ss[j + 1]), cn);
                nc[j + 1] = __fdiv_rn(__fadd_rn(s_ss[j + 2], s_ss[j + 3]), cn);
                c16[j] = s_c[j / 2].x;
                c16[j + 1] = s_c[j / 2].y;
            }
            float error_max = 0.f;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const float a = ref_int_abs_dev(__fsub_rn(nc[j], c16[j]));
                if (a > error_max) {
                    error_max = a;
                    c16[j] = nc[j];
                }
            }
#pragma unroll
            for (int c = 0; c < 8; ++c) s_c[c] = make_float2(c16[2 * c], c16[2 * c + 1]);
            s_again = error_max > 10.f && passes + 1 < max_passes;
        }
        ++passes;
        __syncthreads();
        if (!s_again) break;  // uniform
    }
    if (tid < 8) {
        cent16[2 * tid] = s_c[tid].x;
        cent16[2 * tid + 1] = s_c[tid].y;
        if (bin_counts_out) bin_counts_out[tid] = s_run[tid];
    }
    if (sums_out && tid < 32) sums_out[tid] = s_ss[tid];
    if (passes_out && tid == 0) *passes_out = passes;
}

ECC_API int ecc_kmeans_refcompat_f32(ecc_ctx *ctx, const float *xy, int64_t n, float *centroids16, int32_t max_passes,
                                     int32_t *passes_out, int32_t *bin_counts_out, float *partial_sums_out,
                                     ecc_stream_t stream) {
    if (!ctx || !centroids16 || n < 0 || n > kRcMaxPts || max_passes < 1 || (n > 0 && !xy)) return ECC_ERR_INVALID;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    static bool lds_ok = false;
    if (!lds_ok) {
        ECC_CHECK_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void *>(&kmeans_refcompat_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, kRcBinFloats * 4),
                      "kmeans_refcompat LDS");
        lds_ok = true;
    }
    {
        ECC_TIMED(ctx, s, "kmeans_refcompat_kernel");
        hipLaunchKernelGGL(kmeans_refcompat_kernel, dim3(1), dim3(kRcThreads), kRcBinFloats * 4, s, xy, (int)n,
                           centroids16, max_passes, passes_out, bin_counts_out, partial_sums_out);
    }
    ECC_CHECK_LAUNCH(ctx, "kmeans_refcompat");
    return ECC_OK;
}

// ---- count images (multi-GPU k-means: one all-reduce of the counts instead of one per pass) ----
// A shard's representatives counted per pixel of a caller-given frame (counts[y * w + x], u32).
// Counts are additive over shards, and a Lloyd pass over a count image adds exactly the integer
// sums of the points it counts, so summing the shards' images once and running every pass
// locally gives each rank the single-GPU centroids.
constexpr int kKmFlagWord = 5;  // ctx->flags[5]: a point outside the count frame (3: evt, 4: dbscan)

__global__ void kmeans_set_wh_kernel(uint32_t *wh, uint32_t w, uint32_t h) {
    wh[0] = w;
    wh[1] = h;
}

ECC_API int ecc_kmeans_counts_xy16(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                                   const int32_t *seg_counts, int32_t frame_w, int32_t frame_h, uint32_t *counts,
                                   ecc_stream_t stream) {
    if (!ctx || !counts || n_segs < 0 || seg_stride < 1 || frame_w < 1 || frame_h < 1 || frame_w > 65536 ||
        frame_h > 65536)
        return ECC_ERR_INVALID;
    const Segs segs = make_segs(n_segs, seg_stride, seg_counts);
    const int64_t cells = (int64_t)frame_w * frame_h;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    ECC_CHECK_HIP(ctx, hipMemsetAsync(ctx->flags + kKmFlagWord, 0, 4, s), "memset(kmeans err)");
    if (segs.n_segs == 0) {
        ECC_CHECK_HIP(ctx, hipMemsetAsync(counts, 0, (size_t)cells * 4, s), "memset(counts)");
        return ECC_OK;
    }
    if (!xy) return ECC_ERR_INVALID;
    int parts, slots;
    count_layout(segs.n_segs, cells, parts, slots);
    const size_t off_part = 256;
    int rc = ecc::ws_reserve(ctx, off_part + (size_t)kHistBudget * 4);
    if (rc) return rc;
    char *ws = static_cast<char *>(ctx->ws);
    auto *wh = reinterpret_cast<uint32_t *>(ws);
    auto *partial = reinterpret_cast<uint32_t *>(ws + off_part);
    static bool lds_ok = false;
    if (!lds_ok) {
        ECC_CHECK_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void *>(&kmeans_count_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, kHistChunk * 4),
                      "kmeans_count LDS");
        lds_ok = true;
    }
    {
        ECC_TIMED(ctx, s, "kmeans_count_kernel");
        hipLaunchKernelGGL(kmeans_count_kernel, dim3(count_grid(parts, slots)), dim3(kHistThreads), kHistChunk * 4, s,
                           xy, segs, (const uint32_t *)nullptr, 0, parts, slots, partial, wh, (uint32_t *)nullptr, (uint32_t *)nullptr,
                           (uint32_t)frame_w, (uint32_t)frame_h, ctx->flags + kKmFlagWord);
    }
    {
        ECC_TIMED(ctx, s, "kmeans_count_sum_kernel");
        hipLaunchKernelGGL(kmeans_count_sum_kernel, dim3(1024), dim3(kThreads), 0, s, (const uint32_t *)partial, parts,
                           (const uint32_t *)wh, counts);
    }
    ECC_CHECK_LAUNCH(ctx, "kmeans counts");
    return ECC_OK;
}

ECC_API int ecc_kmeans_counts_status(ecc_ctx *ctx, ecc_stream_t stream) {
    if (!ctx) return ECC_ERR_INVALID;
    int32_t f = 0;
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(&f, ctx->flags + kKmFlagWord, 4, hipMemcpyDeviceToHost, ecc::as_stream(stream)),
                  "read kmeans flag");
    ECC_CHECK_HIP(ctx, hipStreamSynchronize(ecc::as_stream(stream)), "sync");
    return f ? ECC_ERR_INVALID : ECC_OK;
}

ECC_API int ecc_kmeans_run_counts(ecc_ctx *ctx, const uint32_t *counts, int32_t frame_w, int32_t frame_h,
                                  const ecc_kmeans_cfg *cfg, float *centroids, int32_t *iters_out,
                                  ecc_stream_t stream) {
    int rc = kmeans_check(ctx, cfg, centroids);
    if (rc) return rc;
    if (!counts || frame_w < 1 || frame_h < 1 || frame_w > 65536 || frame_h > 65536) return ECC_ERR_INVALID;
    if (cfg->k > kFastMaxK) return ECC_ERR_INVALID;  // pixel passes: k <= 32
    constexpr size_t kAccBytes = (size_t)kAccCopies * kAccStride * 8;
    const size_t off_st = 3 * kAccBytes;
    const size_t off_cb = off_st + 64;
    const size_t off_wh = ecc::align_up(off_cb + 2 * 2 * kMaxK * sizeof(float), 256);
    rc = ecc::ws_reserve(ctx, off_wh + 256);
    if (rc) return rc;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    char *ws = static_cast<char *>(ctx->ws);
    unsigned long long *accb[3] = {reinterpret_cast<unsigned long long *>(ws),
                                   reinterpret_cast<unsigned long long *>(ws + kAccBytes),
                                   reinterpret_cast<unsigned long long *>(ws + 2 * kAccBytes)};
    auto *st = reinterpret_cast<KmState *>(ws + off_st);
    float *cb[2] = {reinterpret_cast<float *>(ws + off_cb), reinterpret_cast<float *>(ws + off_cb) + 2 * kMaxK};
    auto *wh = reinterpret_cast<uint32_t *>(ws + off_wh);
    auto *n_out = wh + 2;
    ECC_CHECK_HIP(ctx, hipMemsetAsync(ws, 0, off_st + 64, s), "memset(kmeans acc)");
    ECC_CHECK_HIP(ctx, hipMemsetAsync(n_out, 0, 4, s), "memset(kmeans outside)");
    hipLaunchKernelGGL(kmeans_set_wh_kernel, dim3(1), dim3(1), 0, s, wh, (uint32_t)frame_w, (uint32_t)frame_h);
    auto step = [&](int it, bool final_pass) {
        StepArgs a{};
        a.acc_in = it ? accb[(it - 1) % 3] : nullptr;
        a.acc_zero = accb[(it + 1) % 3];
        a.c_prev = it ? cb[(it - 1) & 1] : centroids;
        a.c_next = cb[it & 1];
        a.cent = centroids;
        a.n_copies = kAccCopies;
        a.k = cfg->k;
        a.thr = cfg->threshold;
        a.tol = cfg->tol;
        a.final_pass = final_pass;
        a.want_image = false;
        const PixArgs px{counts, (const uint32_t *)n_out, n_out, accb[it % 3], wh};
        if (final_pass) {
            ECC_TIMED(ctx, s, "kmeans_step_kernel");
            if (cfg->k <= 16) launch_step<16, false>(dim3(1), s, a, nullptr, 0, nullptr, st, px);
            else launch_step<32, false>(dim3(1), s, a, nullptr, 0, nullptr, st, px);
        } else {
            ECC_TIMED(ctx, s, "kmeans_pixel_pass");
            if (cfg->k <= 16) launch_step<16, true>(dim3(kPixGrid), s, a, nullptr, 0, nullptr, st, px);
            else launch_step<32, true>(dim3(kPixGrid), s, a, nullptr, 0, nullptr, st, px);
        }
    };
    for (int it = 0; it < cfg->max_iters; ++it) step(it, false);
    if (cfg->max_iters > 0) step(cfg->max_iters, true);  // the last pass's update
    ECC_CHECK_LAUNCH(ctx, "kmeans run_counts");
    if (iters_out)
        ECC_CHECK_HIP(ctx, hipMemcpyAsync(iters_out, &st->iters, 4, hipMemcpyDeviceToDevice, s), "copy iters");
    return ECC_OK;
}
