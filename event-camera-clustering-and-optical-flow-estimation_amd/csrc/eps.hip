// eps-neighbourhoods for DBSCAN / OPTICS over 2-D pixel points.
//
// Reference: DBSCANSimpleCluster::radiusSearch (PCC/DBSCAN_simple.h:118-142, O(N) per query,
// d^2 <= eps^2 in double, self first), DBSCANPrecompCluster::precomp (PCC/DBSCAN_precomp.h:
// 22-44, O(N^2) adjacency), kdt::KDTree::radius_search (OPT/include/optics/kdTree.hpp:307-422)
// and optics::compute_core_dist (OPT/include/optics/optics.hpp:286-299: nth_element of the
// squared distances at min_pts-1, self included).
//
// MI355X design: one 1024-lane workgroup (16 waves) per segment (<= 16384 points, e.g. one
// downsample window), the segment binned in LDS into a uniform grid of cell size > eps
// (eps_grid.hpp).  Queries run in cell order, so a wave's lanes walk the same row runs
// (broadcast LDS reads, uniform trip counts): exact integer d^2 against floor(eps^2), the
// count, and the (min_pts-1)-th smallest d^2 in a register insertion network (no
// runtime-indexed arrays), so core distance = sqrt of an exact integer (fp64, correctly rounded -
// bit-exact vs the oracle).  Results are staged in LDS by segment index and written out
// coalesced (no 4/8-B scatter).  The list kernel emits each query's neighbours with a 9-way merge
// of the cells' ascending runs, i.e. ascending segment-local indices (the order of
// DBSCAN_precomp's adjacency lists), at offsets from a device exclusive scan of the counts.
// Algorithmic bytes: 4 B/point in + 4 B/point (count) [+ 8 B core distance] out; lists: + 4 B
// per neighbour out.
#include "eps_grid.hpp"

namespace {

using ecc::epsg::CellGrid;
using ecc::epsg::kCells;
using ecc::epsg::kNT;
constexpr int kMaxPts = 16384;

struct SegView {
    const int32_t *counts;
    int64_t n_segs, stride;
};

__device__ __forceinline__ int seg_points(const SegView &sv, int64_t s) {
    int m = sv.counts ? sv.counts[s] : (int)sv.stride;
    return m < 0 ? 0 : (m > (int)sv.stride ? (int)sv.stride : m);
}

// Counts (+ core distances when K > 0: the K smallest d^2 kept, K >= min_pts).  Dynamic LDS:
// cend[kCells + 1] | spt[stride] | sidx[stride] and, when kStage, st_cnt[stride] (u16) |
// st_d2[stride] (u32, K > 0): the results by segment index, written out coalesced after the
// queries.  ~120 KB at stride 8192 with core distances.
template <int K, bool kStage>
__global__ void __launch_bounds__(kNT)
eps_counts_kernel(const uint32_t *__restrict__ xy, SegView sv, int e_int, uint32_t r2i, int min_pts,
                  int32_t *__restrict__ counts, double *__restrict__ core) {
    extern __shared__ uint32_t lds_c[];
    uint32_t *cend = lds_c;
    uint32_t *spt = cend + kCells + 1;
    uint16_t *sidx = reinterpret_cast<uint16_t *>(spt + sv.stride);
    uint16_t *st_cnt = sidx + sv.stride;
    uint32_t *st_d2 = reinterpret_cast<uint32_t *>(st_cnt + ((sv.stride + 1) & ~1ll));
    __shared__ int red[64];
    const int tid = threadIdx.x;
    for (int64_t s = blockIdx.x; s < sv.n_segs; s += gridDim.x) {
        const int m = seg_points(sv, s);
        const int64_t base = s * sv.stride;
        const CellGrid g = ecc::epsg::bin_cells(xy, base, m, e_int, r2i, cend, spt, sidx, red, false, true);
        ecc::epsg::with_narrow(g, [&](auto narrow) {
            constexpr bool kN = decltype(narrow)::value;
            for (int q = tid; q < m; q += kNT) {
                const uint32_t v = spt[q];
                const int i = sidx[q];
                int cnt = 0;
                int best[K > 0 ? K : 1];
#pragma unroll
                for (int k = 0; k < (K > 0 ? K : 1); ++k) best[k] = 0x7fffffff;
                ecc::epsg::for_candidates(g, cend, spt, v, [&](int, uint32_t w, bool ok) {
                    uint32_t d2;
                    const bool in = ecc::epsg::in_eps<kN>(v, w, e_int, r2i, &d2) & ok;
                    cnt += in ? 1 : 0;
                    if (K > 0) {  // insertion network keeps the K smallest, sorted
                        int val = in ? (int)d2 : 0x7fffffff;
#pragma unroll
                        for (int k = 0; k < (K > 0 ? K : 1); ++k) {
                            const int lo2 = min(best[k], val);
                            val = max(best[k], val);
                            best[k] = lo2;
                        }
                    }
                });
                uint32_t sel = 0xffffffffu;  // not a core point
                if (K > 0 && cnt >= min_pts) {
#pragma unroll
                    for (int k = 0; k < (K > 0 ? K : 1); ++k) sel = (k == min_pts - 1) ? (uint32_t)best[k] : sel;
                }
                if (kStage) {
                    st_cnt[i] = (uint16_t)cnt;
                    if (K > 0) st_d2[i] = sel;
                } else {
                    counts[base + i] = cnt;
                    if (K > 0) core[base + i] = sel == 0xffffffffu ? -1.0 : sqrt((double)sel);
                }
            }
        });
        if (kStage) __syncthreads();
        for (int i = tid; i < sv.stride; i += kNT) {
            if (!kStage && i < m) continue;  // written by its query
            const bool has = kStage && i < m;
            counts[base + i] = has ? (int32_t)st_cnt[i] : 0;
            if (K > 0) {
                const uint32_t sel = has ? st_d2[i] : 0xffffffffu;
                core[base + i] = sel == 0xffffffffu ? -1.0 : sqrt((double)sel);  // correctly rounded
            }
        }
        __syncthreads();
    }
}

// Ascending neighbour lists.  Dynamic LDS: cend[kCells + 1] | spt[stride] | sidx[stride] with
// every cell's run sorted by segment index; each query merges its (up to) 9 cell runs with the
// run heads cached in registers, so one step = a 9-way min and one LDS read.
__global__ void __launch_bounds__(kNT)
eps_lists_kernel(const uint32_t *__restrict__ xy, SegView sv, int e_int, uint32_t r2i,
                 const int64_t *__restrict__ offsets, int32_t *__restrict__ nbr, int64_t nbr_cap,
                 int32_t *__restrict__ err) {
    extern __shared__ uint32_t lds_l[];
    uint32_t *cend = lds_l;
    uint32_t *spt = cend + kCells + 1;
    uint16_t *sidx = reinterpret_cast<uint16_t *>(spt + sv.stride);
    __shared__ int red[64];
    const int tid = threadIdx.x;
    for (int64_t s = blockIdx.x; s < sv.n_segs; s += gridDim.x) {
        const int m = seg_points(sv, s);
        const int64_t base = s * sv.stride;
        const CellGrid g = ecc::epsg::bin_cells(xy, base, m, e_int, r2i, cend, spt, sidx, red, true, false);
        for (int q = tid; q < m; q += kNT) {
            const uint32_t v = spt[q];
            const int i = sidx[q];
            const int cx = ecc::epsg::cell_x(g, v), cy = ecc::epsg::cell_y(g, v);
            int lo[9], hi[9], head[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const int x = cx + (k % 3) - 1, y = cy + (k / 3) - 1;
                const bool ok = x >= 0 && y >= 0 && x < g.gx && y < g.gy;
                const int c = y * g.gx + x;
                lo[k] = ok ? (c == 0 ? 0 : (int)cend[c - 1]) : 0;
                hi[k] = ok ? (int)cend[c] : 0;
                head[k] = lo[k] < hi[k] ? (int)sidx[lo[k]] : 0x7fffffff;
            }
            int64_t out = offsets[base + i];
            const int64_t end = offsets[base + i + 1];
            for (;;) {
                int bk = 0, bi = head[0];
#pragma unroll
                for (int k = 1; k < 9; ++k) {
                    const bool lt = head[k] < bi;
                    bi = lt ? head[k] : bi;
                    bk = lt ? k : bk;
                }
                if (bi == 0x7fffffff) break;
                int pos = 0, h = 0;
#pragma unroll
                for (int k = 0; k < 9; ++k) {
                    pos = (k == bk) ? lo[k] : pos;
                    h = (k == bk) ? hi[k] : h;
                }
                uint32_t d2;
                const bool in = g.narrow ? ecc::epsg::in_eps<true>(v, spt[pos], e_int, r2i, &d2)
                                         : ecc::epsg::in_eps<false>(v, spt[pos], e_int, r2i, &d2);
                const int nxt = pos + 1;
                const int nh = nxt < h ? (int)sidx[nxt] : 0x7fffffff;
#pragma unroll
                for (int k = 0; k < 9; ++k) {
                    lo[k] = (k == bk) ? nxt : lo[k];
                    head[k] = (k == bk) ? nh : head[k];
                }
                if (in) {
                    if (out < end && out < nbr_cap) nbr[out] = bi;
                    else *err = 1;
                    ++out;
                }
            }
        }
        __syncthreads();
    }
}

int check_segs(const ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t stride,
               double eps) {
    if (!ctx || n_segs < 0 || stride < 1 || !(eps >= 0.0) || eps > 32767.0) return ECC_ERR_INVALID;
    if (n_segs > 0 && !xy) return ECC_ERR_INVALID;
    if (stride > kMaxPts) return ECC_ERR_INVALID;  // segments hold <= 16384 points
    return ECC_OK;
}

}  // namespace

ECC_API int ecc_eps_counts(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                           const int32_t *seg_counts, double eps, int32_t min_pts,
                           int32_t *counts, double *core_dist, ecc_stream_t stream) {
    int rc = check_segs(ctx, xy, n_segs, seg_stride, eps);
    if (rc) return rc;
    if (!counts || (core_dist && (min_pts < 1 || min_pts > 64))) return ECC_ERR_INVALID;
    if (n_segs == 0) return ECC_OK;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    SegView sv{seg_counts, n_segs, seg_stride};
    // d^2 <= eps^2 (fp64) <=> d^2 <= floor(eps^2) for integer d^2; |dx|, |dy| <= floor(eps)
    const double r2 = eps * eps;
    const int r2i = (int)std::floor(r2), e_int = (int)std::floor(eps);
    const int K = core_dist ? min_pts : 0;
    // results staged in LDS (coalesced writes) when the staging fits next to the grid
    const size_t grid_lds = (size_t)(kCells + 1 + seg_stride) * 4 + (size_t)seg_stride * 2;
    const size_t stage_lds = (size_t)((seg_stride + 1) & ~1ll) * 2 + (core_dist ? (size_t)seg_stride * 4 : 0);
    const bool stage = grid_lds + stage_lds + 256 <= 160 * 1024;
    using Kern = void (*)(const uint32_t *, SegView, int, uint32_t, int, int32_t *, double *);
#define ECC_EPS_PICK(S)                                                                                        \
    (K == 0 ? eps_counts_kernel<0, S> : K <= 1 ? eps_counts_kernel<1, S> : K <= 2 ? eps_counts_kernel<2, S>     \
     : K <= 4 ? eps_counts_kernel<4, S> : K <= 8 ? eps_counts_kernel<8, S> : K <= 16 ? eps_counts_kernel<16, S> \
     : K <= 32 ? eps_counts_kernel<32, S> : eps_counts_kernel<64, S>)
    const Kern kern = stage ? (Kern)ECC_EPS_PICK(true) : (Kern)ECC_EPS_PICK(false);
#undef ECC_EPS_PICK
    const size_t lds = grid_lds + (stage ? stage_lds : 0);
    ECC_CHECK_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                  "eps_counts lds");
    // segments are grid-strided; enough workgroups for every CU at the occupancy the LDS allows
    const unsigned grid = (unsigned)std::min<int64_t>(n_segs, 2048);
    {
        ECC_TIMED(ctx, ecc::as_stream(stream), "eps_counts_kernel");
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kNT), lds, ecc::as_stream(stream), xy, sv, e_int, (uint32_t)r2i,
                           min_pts, counts, core_dist);
    }
    ECC_CHECK_LAUNCH(ctx, "eps_counts_kernel");
    return ECC_OK;
}

ECC_API int ecc_eps_lists(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                          const int32_t *seg_counts, double eps, const int32_t *counts,
                          int64_t *offsets, int32_t *nbr, int64_t nbr_cap, ecc_stream_t stream) {
    int rc = check_segs(ctx, xy, n_segs, seg_stride, eps);
    if (rc) return rc;
    if (!counts || !offsets || (nbr_cap > 0 && !nbr) || nbr_cap < 0) return ECC_ERR_INVALID;
    if (n_segs == 0) return ECC_OK;
    const int64_t n = n_segs * seg_stride;
    rc = ecc::ws_reserve(ctx, ecc::scan_scratch_bytes(n));
    if (rc) return rc;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    rc = ecc::exclusive_scan_i32_i64(ctx, counts, n, offsets, reinterpret_cast<int64_t *>(ctx->ws), s);
    if (rc) return rc;
    ECC_CHECK_HIP(ctx, hipMemsetAsync(ctx->flags + 2, 0, 4, s), "memset(eps err)");
    SegView sv{seg_counts, n_segs, seg_stride};
    const int r2i = (int)std::floor(eps * eps), e_int = (int)std::floor(eps);
    const size_t lds = (size_t)(kCells + 1 + seg_stride) * 4 + (size_t)seg_stride * 2;
    ECC_CHECK_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void *>(eps_lists_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                  "eps_lists lds");
    const unsigned grid = (unsigned)std::min<int64_t>(n_segs, 2048);
    {
        ECC_TIMED(ctx, s, "eps_lists_kernel");
        hipLaunchKernelGGL(eps_lists_kernel, dim3(grid), dim3(kNT), lds, s, xy, sv, e_int, (uint32_t)r2i,
                           (const int64_t *)offsets, nbr, nbr_cap, ctx->flags + 2);
    }
    ECC_CHECK_LAUNCH(ctx, "eps_lists_kernel");
    return ECC_OK;
}

ECC_API int ecc_eps_total(ecc_ctx *ctx, const int64_t *offsets, int64_t n, int64_t *total,
                          ecc_stream_t stream) {
    if (!ctx || !offsets || !total || n < 0) return ECC_ERR_INVALID;
    hipStream_t s = ecc::as_stream(stream);
    int32_t err = 0;
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(total, offsets + n, 8, hipMemcpyDeviceToHost, s), "read total");
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(&err, ctx->flags + 2, 4, hipMemcpyDeviceToHost, s), "read err");
    ECC_CHECK_HIP(ctx, hipStreamSynchronize(s), "sync");
    return err ? ECC_ERR_CAPACITY : ECC_OK;
}
