// Greedy box NMS per slice.
//
// Reference: CornerFilter::filterCorners, FCT/…group_track.cpp:81-152 — a H×W u8 mask
// (cv::Mat::zeros per call), corners visited in detection order, a corner is kept iff no mask
// pixel inside its clipped box [x±7]×[y±7] is set, and a kept corner paints its box
// (cv::rectangle filled).  Called once per 16384-event slice (:832-837).
//
// MI355X design: one workgroup per slice, every slice of a batch in ONE launch.  The slice's
// corner flags (16 KiB) are read with 16-B loads and compacted in event order into LDS; the
// greedy pass then runs on one wave without any mask image: "box touches a painted pixel"
// == "box intersects the box of an earlier kept corner" (kept boxes are the painted set).
// Candidates are processed 64 at a time: each lane tests its candidate against the kept list
// (LDS broadcast reads), then the within-chunk order dependency is resolved on a 64x64
// overlap bitmask with scalar bit logic.  Output label = rank in the kept list (:140).
//
// Grid form (used whenever the grid fits LDS): two boxes [c±h] overlap iff their centres are
// within Chebyshev distance 2h (clipping to the image never separates two boxes whose centres
// lie inside it), so kept boxes are pairwise disjoint and a grid of (2h+1)-pixel cells holds at
// most ONE kept centre per cell.  "Overlaps an earlier kept box" is then 9 LDS probes.  A
// parallel compaction kernel (256 lanes per slice) first lists each slice's flagged events in
// event order; one wave per slice then takes them 64 at a time, and within a chunk the kept ones
// are found by a scalar loop over the surviving lanes (each kept lane's centre is broadcast and
// kills the later lanes it overlaps).  ~2 KiB of LDS per slice, so many slices run per CU.
#include "ecc_internal.hpp"

#include <map>
#include <mutex>

namespace {

constexpr int kThreads = 256;
constexpr int kMaxCand = 16384;  // LDS candidate list (64 KiB)
constexpr int kMaxKept = 8192;   // LDS kept list (boxes are disjoint => <= W*H/144)

struct Box { int16_t x0, x1, y0, y1; };

__device__ __forceinline__ Box make_box(uint32_t v, int half, int W, int H) {
    const int x = ecc::xy_x(v), y = ecc::xy_y(v);
    Box b;
    b.x0 = (int16_t)max(0, x - half);     // :114-117
    b.x1 = (int16_t)min(W - 1, x + half);
    b.y0 = (int16_t)max(0, y - half);
    b.y1 = (int16_t)min(H - 1, y + half);
    return b;
}

__device__ __forceinline__ bool overlap(const Box &a, const Box &b) {
    return a.x0 <= b.x1 && b.x0 <= a.x1 && a.y0 <= b.y1 && b.y0 <= a.y1;
}

__global__ void __launch_bounds__(kThreads)
nms_kernel(const uint32_t *__restrict__ xy, const uint8_t *__restrict__ flags, int64_t n, int S,
           int W, int H, int half, int cap, ecc_corner *__restrict__ out,
           int32_t *__restrict__ out_count, int32_t *__restrict__ err) {
    __shared__ uint32_t cand[kMaxCand];
    __shared__ Box kept[kMaxKept];
    __shared__ int wave_tot[kThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t s = blockIdx.x;
    const int64_t lo = s * (int64_t)S;
    const int64_t hi = (lo + S < n) ? lo + S : n;
    const int64_t len = hi - lo;

    // 1. compaction of flagged events in event order, in chunks of 256*16 events
    int n_cand = 0;
    for (int64_t c0 = 0; c0 < len; c0 += kThreads * 16) {
        const int64_t my0 = c0 + (int64_t)tid * 16;
        uint32_t bits = 0;
        if (my0 + 15 < len && ((lo + my0) & 15) == 0) {
            const uint4 q = *reinterpret_cast<const uint4 *>(flags + lo + my0);
            const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int k = 0; k < 16; ++k) bits |= (((w4[k >> 2] >> (8 * (k & 3))) & 0xffu) ? 1u : 0u) << k;
        } else {
            for (int k = 0; k < 16; ++k)
                if (my0 + k < len && flags[lo + my0 + k]) bits |= 1u << k;
        }
        const int cntv = __popc(bits);
        // wave inclusive scan of cntv
        const int incl = ecc::wave_incl_scan(cntv);  // DPP
        if (lane == 63) wave_tot[wave] = incl;
        __syncthreads();
        int off = n_cand + incl - cntv, tot = 0;
        for (int w = 0; w < kThreads / 64; ++w) {
            if (w < wave) off += wave_tot[w];
            tot += wave_tot[w];
        }
        while (bits) {
            const int k = __ffs(bits) - 1;
            bits &= bits - 1;
            if (off < kMaxCand) cand[off] = xy[lo + my0 + k];
            ++off;
        }
        n_cand += tot;
        __syncthreads();
    }
    if (n_cand > kMaxCand) n_cand = kMaxCand;  // cannot happen when S <= kMaxCand
    __syncthreads();
    // 2. greedy NMS on wave 0 (the other waves only keep the barriers uniform)
    int n_kept = 0;
    bool overflow = false;
    for (int c0 = 0; c0 < n_cand; c0 += 64) {
        if (wave == 0) {
            const int ci = c0 + lane;
            const bool valid = ci < n_cand;
            const uint32_t v = valid ? cand[ci] : 0u;
            const Box b = make_box(v, half, W, H);
            bool alive = valid;
            for (int k = 0; k < n_kept && alive; ++k)
                if (overlap(b, kept[k])) alive = false;
            // within-chunk dependency: ov = lanes j < lane whose box overlaps mine
            uint64_t ov = 0;
            for (int j = 0; j < 64; ++j) {
                const int x0 = __shfl((int)b.x0, j), x1 = __shfl((int)b.x1, j);
                const int y0 = __shfl((int)b.y0, j), y1 = __shfl((int)b.y1, j);
                const bool o = (j < lane) && x0 <= b.x1 && b.x0 <= x1 && y0 <= b.y1 && b.y0 <= y1;
                ov |= (uint64_t)o << j;
            }
            uint64_t alive_m = __ballot(alive);
            uint64_t acc = 0;
            while (alive_m) {
                const int i = __ffsll((unsigned long long)alive_m) - 1;
                alive_m &= alive_m - 1;
                const uint64_t ov_i = __shfl(ov, i);
                if ((ov_i & acc) == 0) acc |= 1ull << i;
            }
            const bool keep = (acc >> lane) & 1ull;
            const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
            const int rank = n_kept + __popcll(acc & lt);
            if (keep) {
                if (rank < kMaxKept) kept[rank] = b;
                else overflow = true;
                if (rank < cap) out[s * (int64_t)cap + rank] = ecc_corner{ecc::xy_x(v), ecc::xy_y(v), rank};
                else overflow = true;
            }
            n_kept += __popcll(acc);
            if (n_kept > kMaxKept) n_kept = kMaxKept;
        }
        __syncthreads();  // orders the kept[] LDS writes before the next chunk's reads
    }
    if (wave != 0) return;
    overflow = __any(overflow);
    if (lane == 0) {
        out_count[s] = n_kept < cap ? n_kept : cap;
        if (overflow) atomicOr(err, 1);
    }
}


constexpr int kGridThreads = 64;
constexpr int kGridMaxCells = 16384;  // 64 KiB of LDS
constexpr uint32_t kNoCentre = 0xffffffffu;

__device__ __forceinline__ bool near_centre(uint32_t a, uint32_t b, int reach) {
    return abs(ecc::xy_x(a) - ecc::xy_x(b)) <= reach && abs(ecc::xy_y(a) - ecc::xy_y(b)) <= reach;
}

// Two-kernel grid form (bench sizes): candidates first, greedy second.
// nms_compact_kernel: one 256-lane workgroup per slice (chunks of 4096 events): 16-B flag loads,
// a block scan of the per-lane flag counts, and the flagged events' xy gathered into the slice's
// candidate list in event order (cand[s*S ...], count n_cand[s]).
constexpr int kCompactThreads = 256;

__global__ void __launch_bounds__(kCompactThreads)
nms_compact_kernel(const uint32_t *__restrict__ xy, const uint8_t *__restrict__ flags, int64_t n, int S,
                   uint32_t *__restrict__ cand, int32_t *__restrict__ n_cand) {
    __shared__ int wtot[kCompactThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t s = blockIdx.x;
    const int64_t lo = s * (int64_t)S;
    const int64_t len = ((lo + S < n) ? lo + S : n) - lo;
    int run = 0;
    // 16-B aligned slices: one unconditional 16-B load per lane through a buffer view of the
    // slice rounded up to 16 B (the round-up stays inside the allocation's last 16-B block; bytes
    // past len are masked) -- a per-lane choice of load form waited for every load
    const bool vec = ((reinterpret_cast<uintptr_t>(flags) + lo) & 15) == 0;  // uniform
    const __amdgpu_buffer_rsrc_t vf = ecc::buffer_view(flags + lo, (uint32_t)((len + 15) & ~15ll));
    for (int64_t c0 = 0; c0 < len; c0 += kCompactThreads * 16) {
        const int64_t my0 = c0 + (int64_t)tid * 16;
        uint32_t bits = 0;
        if (vec) {
            const uint4 q = ecc::buffer_load_u128(vf, (uint32_t)my0);
            const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int k = 0; k < 16; ++k)
                bits |= (((w4[k >> 2] >> (8 * (k & 3))) & 0xffu) && my0 + k < len ? 1u : 0u) << k;
        } else {
            for (int k = 0; k < 16; ++k)
                if (my0 + k < len && flags[lo + my0 + k]) bits |= 1u << k;
        }
        const int cnt = __popc(bits);
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wtot[wave] = incl;
        __syncthreads();
        int off = run + incl - cnt, tot = 0;
#pragma unroll
        for (int w = 0; w < kCompactThreads / 64; ++w) {
            off += w < wave ? wtot[w] : 0;
            tot += wtot[w];
        }
        while (bits) {
            const int k = __ffs(bits) - 1;
            bits &= bits - 1;
            cand[lo + off++] = xy[lo + my0 + k];
        }
        run += tot;
        __syncthreads();
    }
    if (tid == 0) n_cand[s] = run;
}

// nms_greedy_kernel: one wave per slice over its candidate list (the next 64 candidates are
// requested before the current 64 are decided); the kept-centre grid as in nms_grid_kernel.
__global__ void __launch_bounds__(kGridThreads)
nms_greedy_kernel(const uint32_t *__restrict__ cand, const int32_t *__restrict__ n_cand, int S, int W, int H,
                  int half, int gw, int gh, int cap, ecc_corner *__restrict__ out, int32_t *__restrict__ out_count,
                  int32_t *__restrict__ err) {
    extern __shared__ uint32_t grid[];  // [gh][gw] kept centre per cell
    const int lane = threadIdx.x;
    const int64_t s = blockIdx.x;
    const uint32_t *c = cand + s * (int64_t)S;
    const int total = n_cand[s];
    const int cs = 2 * half + 1, reach = 2 * half;
    const int pw = gw + 2;  // one border cell on every side: the 3x3 probes need no bounds checks
    for (int i = lane; i < pw * (gh + 2); i += kGridThreads) grid[i] = kNoCentre;
    const uint64_t lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    int n_kept = 0;
    bool overflow = false, bad_input = false;
    uint32_t nxt = lane < total ? c[lane] : 0u;
    __syncthreads();
    for (int p0 = 0; p0 < total; p0 += kGridThreads) {
        uint32_t v = nxt;
        const bool have = p0 + lane < total;
        nxt = (p0 + kGridThreads + lane < total) ? c[p0 + kGridThreads + lane] : 0u;
        int x = ecc::xy_x(v), y = ecc::xy_y(v);
        const bool outside = have && (x >= W || y >= H);
        if (outside) bad_input = true;  // skipped and reported (ecc_corner_nms_status)
        const bool valid = have && !outside;
        if (!valid) { v = 0u; x = 0; y = 0; }
        const int cx = x / cs, cy = y / cs;
        bool alive = valid;
        const int c0 = cy * pw + cx;  // padded cell (cx, cy) - (1, 1)
        uint32_t kc[9];
#pragma unroll
        for (int d = 0; d < 9; ++d) kc[d] = grid[c0 + (d / 3) * pw + d % 3];
#pragma unroll
        for (int d = 0; d < 9; ++d) alive &= !(kc[d] != kNoCentre && near_centre(kc[d], v, reach));
        uint64_t am = __ballot(alive), keepm = 0;
        while (am) {  // wave-uniform: each step keeps the first surviving lane
            const int i0 = __ffsll((unsigned long long)am) - 1;
            keepm |= 1ull << i0;
            am &= am - 1;
            const uint32_t vi = (uint32_t)__builtin_amdgcn_readlane((int)v, i0);
            am &= ~__ballot(lane > i0 && near_centre(vi, v, reach));
        }
        if ((keepm >> lane) & 1ull) {
            const int rank = n_kept + __popcll(keepm & lt_mask);
            grid[c0 + pw + 1] = v;
            if (rank < cap) out[s * (int64_t)cap + rank] = ecc_corner{x, y, rank};
            else overflow = true;
        }
        n_kept += __popcll(keepm);
        __syncthreads();
    }
    overflow = __any(overflow);
    bad_input = __any(bad_input);
    if (lane == 0) {
        out_count[s] = n_kept < cap ? n_kept : cap;
        if (overflow) atomicOr(err, 1);
        if (bad_input) atomicOr(err, 2);
    }
}

// Packs per-slice corner lists (slice s at in[s * cap], counts[s] <= cap) densely at
// out[offsets[s]]: one workgroup per slice.
__global__ void __launch_bounds__(256)
corner_pack_kernel(const ecc_corner *__restrict__ in, const int32_t *__restrict__ counts, int cap,
                   const int64_t *__restrict__ offsets, ecc_corner *__restrict__ out) {
    const int64_t s = blockIdx.x;
    const int c = min(max(counts[s], 0), cap);
    const int64_t o = offsets[s];
    for (int d = threadIdx.x; d < c; d += 256) out[o + d] = in[s * cap + d];
}

struct NmsState {
    void *buf = nullptr;
    size_t bytes = 0;
};
std::mutex g_nms_mu;
std::map<const ecc_ctx *, NmsState> g_nms;

}  // namespace

namespace ecc {
int nms_check_args(int64_t n, int32_t slice_events, int32_t width, int32_t height, int32_t box_size, int32_t cap) {
    if (n < 0 || slice_events < 1 || slice_events > kMaxCand || width < 1 || height < 1 || width > 32767 ||
        height > 32767 || box_size < 1 || cap < 0)
        return ECC_ERR_INVALID;
    return ECC_OK;
}

int nms_candidates(ecc_ctx *ctx, int64_t n, int32_t slice_events, int32_t width, int32_t height, int32_t box_size,
                   uint32_t **cand, int32_t **n_cand) {
    *cand = nullptr;
    *n_cand = nullptr;
    const int cs = 2 * (box_size / 2) + 1;
    const int gw = (width + cs - 1) / cs, gh = (height + cs - 1) / cs;
    if ((int64_t)(gw + 2) * (gh + 2) > kGridMaxCells) return ECC_OK;  // the one-kernel form takes it
    const int64_t n_slices = (n + slice_events - 1) / slice_events;
    // candidate lists: n xy words + n_slices counts, per context (grown, never shrunk)
    const size_t need = ecc::align_up((size_t)n * 4, 256) + (size_t)n_slices * 4;
    NmsState *st;
    {
        std::lock_guard<std::mutex> lk(g_nms_mu);
        st = &g_nms[ctx];
    }
    if (need > st->bytes) {
        if (st->buf) {
            ECC_CHECK_HIP(ctx, hipDeviceSynchronize(), "sync(nms buffer)");
            (void)hipFree(st->buf);
            st->buf = nullptr;
            st->bytes = 0;
        }
        const size_t want = ecc::align_up(need + need / 8, 1 << 20);
        if (hipMalloc(&st->buf, want) != hipSuccess) {
            st->buf = nullptr;
            return ECC_ERR_NOMEM;
        }
        st->bytes = want;
    }
    *cand = static_cast<uint32_t *>(st->buf);
    *n_cand = reinterpret_cast<int32_t *>(static_cast<char *>(st->buf) + ecc::align_up((size_t)n * 4, 256));
    return ECC_OK;
}

int nms_greedy(ecc_ctx *ctx, const uint32_t *cand, const int32_t *n_cand, int64_t n, int32_t slice_events,
               int32_t width, int32_t height, int32_t box_size, int32_t cap, ecc_corner *out, int32_t *out_count,
               hipStream_t s) {
    const int64_t n_slices = (n + slice_events - 1) / slice_events;
    const int half = box_size / 2, cs = 2 * half + 1;
    const int gw = (width + cs - 1) / cs, gh = (height + cs - 1) / cs;
    ECC_TIMED(ctx, s, "nms_kernel");
    hipLaunchKernelGGL(nms_greedy_kernel, dim3((unsigned)n_slices), dim3(kGridThreads), (size_t)(gw + 2) * (gh + 2) * 4,
                       s, cand, n_cand, slice_events, width, height, half, gw, gh, cap, out, out_count, ctx->flags + 1);
    return ECC_OK;
}
}  // namespace ecc

ECC_API int ecc_corner_nms(ecc_ctx *ctx, const uint32_t *xy, const uint8_t *corner_flags,
                           int64_t n, int32_t slice_events, int32_t width, int32_t height,
                           int32_t box_size, int32_t cap, ecc_corner *out, int32_t *out_count,
                           ecc_stream_t stream) {
    if (!ctx || ecc::nms_check_args(n, slice_events, width, height, box_size, cap)) return ECC_ERR_INVALID;
    if (n == 0) return ECC_OK;
    if (!xy || !corner_flags || !out_count || (cap > 0 && !out)) return ECC_ERR_INVALID;
    const int64_t n_slices = (n + slice_events - 1) / slice_events;
    if (n_slices > INT32_MAX) return ECC_ERR_INVALID;
    hipStream_t s = ecc::as_stream(stream);
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    ECC_CHECK_HIP(ctx, hipMemsetAsync(ctx->flags + 1, 0, 4, s), "memset(nms err)");
    uint32_t *cand = nullptr;
    int32_t *n_cand = nullptr;
    int rc = ecc::nms_candidates(ctx, n, slice_events, width, height, box_size, &cand, &n_cand);
    if (rc) return rc;
    if (cand) {
        {
            ECC_TIMED(ctx, s, "nms_compact_kernel");
            hipLaunchKernelGGL(nms_compact_kernel, dim3((unsigned)n_slices), dim3(kCompactThreads), 0, s, xy,
                               corner_flags, n, slice_events, cand, n_cand);
        }
        rc = ecc::nms_greedy(ctx, cand, n_cand, n, slice_events, width, height, box_size, cap, out, out_count, s);
        if (rc) return rc;
    } else {
        ECC_TIMED(ctx, s, "nms_kernel");
        hipLaunchKernelGGL(nms_kernel, dim3((unsigned)n_slices), dim3(kThreads), 0, s, xy,
                           corner_flags, n, slice_events, width, height, box_size / 2, cap, out,
                           out_count, ctx->flags + 1);
    }
    ECC_CHECK_LAUNCH(ctx, "nms_kernel");
    return ECC_OK;
}

ECC_API int ecc_corner_pack(ecc_ctx *ctx, const ecc_corner *in, const int32_t *counts, int32_t n_slices,
                            int32_t cap, ecc_corner *out, int64_t *offsets, ecc_stream_t stream) {
    if (!ctx || n_slices < 0 || cap < 0 || !offsets || (n_slices > 0 && !counts)) return ECC_ERR_INVALID;
    if (n_slices > 0 && cap > 0 && (!in || !out)) return ECC_ERR_INVALID;
    hipStream_t s = ecc::as_stream(stream);
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    int rc = ecc::ws_reserve(ctx, ecc::scan_scratch_bytes(n_slices));
    if (rc) return rc;
    rc = ecc::exclusive_scan_i32_i64(ctx, counts, n_slices, offsets, reinterpret_cast<int64_t *>(ctx->ws), s);
    if (rc) return rc;
    if (n_slices == 0 || cap == 0) return ECC_OK;
    {
        ECC_TIMED(ctx, s, "corner_pack_kernel");
        hipLaunchKernelGGL(corner_pack_kernel, dim3((unsigned)n_slices), dim3(256), 0, s, in, counts, cap,
                           (const int64_t *)offsets, out);
    }
    ECC_CHECK_LAUNCH(ctx, "corner_pack");
    return ECC_OK;
}

ECC_API int ecc_corner_nms_status(ecc_ctx *ctx, ecc_stream_t stream) {
    if (!ctx) return ECC_ERR_INVALID;
    int32_t f = 0;
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(&f, ctx->flags + 1, 4, hipMemcpyDeviceToHost, ecc::as_stream(stream)),
                  "read nms flag");
    ECC_CHECK_HIP(ctx, hipStreamSynchronize(ecc::as_stream(stream)), "sync");
    if (f & 2) return ECC_ERR_INVALID;
    return (f & 1) ? ECC_ERR_CAPACITY : ECC_OK;
}

namespace ecc {
void nms_state_release(const ecc_ctx *ctx) {
    std::lock_guard<std::mutex> lk(g_nms_mu);
    auto it = g_nms.find(ctx);
    if (it == g_nms.end()) return;
    if (it->second.buf) (void)hipFree(it->second.buf);
    g_nms.erase(it);
}
}  // namespace ecc
