// eps-neighbourhoods for DBSCAN / OPTICS over 2-D pixel points.
//
// Reference: DBSCANSimpleCluster::radiusSearch (PCC/DBSCAN_simple.h:118-142, O(N) per query,
// d^2 <= eps^2 in double, self first), DBSCANPrecompCluster::precomp (PCC/DBSCAN_precomp.h:
// 22-44, O(N^2) adjacency), kdt::KDTree::radius_search (OPT/include/optics/kdTree.hpp:307-422)
// and optics::compute_core_dist (OPT/include/optics/optics.hpp:286-299: nth_element of the
// squared distances at min_pts-1, self included).
//
// MI355X design: one workgroup per segment (<= 16384 points, e.g. one downsample window).  The
// segment is binned in LDS into a uniform grid of cell size >= eps (counting sort with LDS
// atomics; each cell's index list is then sorted so lists come out ascending), and every lane
// answers one query from the 3x3 surrounding cells: exact integer d^2 compared against eps^2
// in fp64, the count, and the (min_pts-1)-th smallest d^2 kept in a register insertion network
// (no runtime-indexed arrays), so core distance = sqrt of an exact integer (fp64, correctly
// rounded — bit-exact vs the oracle).  The list kernel emits each query's neighbours with a
// 9-way merge of the cells' sorted lists, i.e. ascending segment-local indices (the order of
// DBSCAN_precomp's adjacency lists), at offsets from a device exclusive scan of the counts.
// Algorithmic bytes: 4 B/point in + 4 B/point (count) [+ 8 B core distance] out.
#include "ecc_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxPts = 16384;
constexpr int kMaxCells = 8192;

struct SegView {
    const int32_t *counts;
    int64_t n_segs, stride;
};

struct Grid {
    int xmin, ymin, cs, gx, gy;
};

// Loads segment s into LDS, bins it and sorts each cell's list. Returns m (points) and grid.
__device__ int bin_segment(const uint32_t *__restrict__ xy, const SegView &sv, int64_t s,
                           double eps, uint32_t *pxy, uint16_t *sorted, uint32_t *cend,
                           int *red, Grid &g) {
    const int tid = threadIdx.x;
    int m = sv.counts ? sv.counts[s] : (int)sv.stride;
    if (m > kMaxPts) m = kMaxPts;  // validated on the host
    const int64_t base = s * sv.stride;
    int xmn = 0x7fffffff, ymn = 0x7fffffff, xmx = -1, ymx = -1;
    for (int i = tid; i < m; i += kThreads) {
        const uint32_t v = xy[base + i];
        pxy[i] = v;
        const int x = ecc::xy_x(v), y = ecc::xy_y(v);
        xmn = min(xmn, x); ymn = min(ymn, y); xmx = max(xmx, x); ymx = max(ymx, y);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        xmn = min(xmn, __shfl_xor(xmn, o)); ymn = min(ymn, __shfl_xor(ymn, o));
        xmx = max(xmx, __shfl_xor(xmx, o)); ymx = max(ymx, __shfl_xor(ymx, o));
    }
    if ((tid & 63) == 0) {
        red[4 * (tid >> 6) + 0] = xmn; red[4 * (tid >> 6) + 1] = ymn;
        red[4 * (tid >> 6) + 2] = xmx; red[4 * (tid >> 6) + 3] = ymx;
    }
    for (int c = tid; c < kMaxCells; c += kThreads) cend[c] = 0;
    __syncthreads();
    xmn = red[0]; ymn = red[1]; xmx = red[2]; ymx = red[3];
    for (int w = 1; w < kThreads / 64; ++w) {
        xmn = min(xmn, red[4 * w]); ymn = min(ymn, red[4 * w + 1]);
        xmx = max(xmx, red[4 * w + 2]); ymx = max(ymx, red[4 * w + 3]);
    }
    if (m == 0) { xmn = ymn = 0; xmx = ymx = 0; }
    int cs = (int)ceil(eps);
    if (cs < 1) cs = 1;
    while ((int64_t)((xmx - xmn) / cs + 1) * ((ymx - ymn) / cs + 1) > kMaxCells) cs *= 2;
    g = Grid{xmn, ymn, cs, (xmx - xmn) / cs + 1, (ymx - ymn) / cs + 1};
    __syncthreads();
    // counting sort by cell (cend[] ends as the END of each cell's range)
    for (int i = tid; i < m; i += kThreads) {
        const uint32_t v = pxy[i];
        const int c = ((ecc::xy_y(v) - g.ymin) / g.cs) * g.gx + (ecc::xy_x(v) - g.xmin) / g.cs;
        atomicAdd(&cend[c], 1u);
    }
    __syncthreads();
    // exclusive scan of the cell counts (kMaxCells / kThreads values per thread)
    {
        constexpr int per = kMaxCells / kThreads;
        uint32_t loc[per];
        uint32_t sum = 0;
#pragma unroll
        for (int k = 0; k < per; ++k) { loc[k] = cend[tid * per + k]; sum += loc[k]; }
        // inclusive wave scan of sum
        uint32_t inc = sum;
        const int lane = tid & 63;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o);
            if (lane >= o) inc += y;
        }
        __syncthreads();
        if (lane == 63) red[16 + (tid >> 6)] = (int)inc;
        __syncthreads();
        uint32_t off = inc - sum;
        for (int w = 0; w < (tid >> 6); ++w) off += (uint32_t)red[16 + w];
#pragma unroll
        for (int k = 0; k < per; ++k) { cend[tid * per + k] = off; off += loc[k]; }
    }
    __syncthreads();
    for (int i = tid; i < m; i += kThreads) {
        const uint32_t v = pxy[i];
        const int c = ((ecc::xy_y(v) - g.ymin) / g.cs) * g.gx + (ecc::xy_x(v) - g.xmin) / g.cs;
        const uint32_t pos = atomicAdd(&cend[c], 1u);
        sorted[pos] = (uint16_t)i;
    }
    __syncthreads();
    // sort each cell's index list ascending (cells are small: insertion sort per thread)
    for (int c = tid; c < g.gx * g.gy; c += kThreads) {
        const int lo = c == 0 ? 0 : (int)cend[c - 1], hi = (int)cend[c];
        for (int a = lo + 1; a < hi; ++a) {
            const uint16_t key = sorted[a];
            int b = a - 1;
            while (b >= lo && sorted[b] > key) { sorted[b + 1] = sorted[b]; --b; }
            sorted[b + 1] = key;
        }
    }
    __syncthreads();
    return m;
}

__device__ __forceinline__ void cell_range(const Grid &g, const uint32_t *cend, int cx, int cy,
                                           int &lo, int &hi) {
    if (cx < 0 || cy < 0 || cx >= g.gx || cy >= g.gy) { lo = hi = 0; return; }
    const int c = cy * g.gx + cx;
    lo = c == 0 ? 0 : (int)cend[c - 1];
    hi = (int)cend[c];
}

// Counts (+ core distances): the segment's coordinates are counting-sorted by grid cell straight
// into LDS (one 4-B read per candidate; a query's three cells of one grid row are one contiguous
// run), and the exact test d^2 <= eps^2 (fp64 in the reference) is the integer test
// d^2 <= floor(eps^2) on integer d^2.  Queries run in cell order too, so a wave's lanes walk
// the same runs.  Dynamic LDS = (kCountCells + 1) cell ends + the segment stride's points and
// indices: 56 KB at 8192, two workgroups per CU.
constexpr int kCountCells = 2048;

template <int K>
__global__ void __launch_bounds__(kThreads)
eps_counts_kernel(const uint32_t *__restrict__ xy, SegView sv, int e_int, int r2i, int min_pts,
                  int32_t *__restrict__ counts, double *__restrict__ core) {
    extern __shared__ uint32_t lds_c[];
    uint32_t *cend = lds_c;                     // [kCountCells + 1]: cell ends after the scatter
    uint32_t *spt = lds_c + kCountCells + 1;    // [stride]: coordinates in cell order
    uint16_t *sidx = reinterpret_cast<uint16_t *>(spt + sv.stride);  // [stride]: their indices
    __shared__ int red[32];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int64_t s = blockIdx.x; s < sv.n_segs; s += gridDim.x) {
        int m = sv.counts ? sv.counts[s] : (int)sv.stride;
        m = m < 0 ? 0 : (m > (int)sv.stride ? (int)sv.stride : m);
        const int64_t base = s * sv.stride;
        // bounding box -> grid (cell >= eps, at most kCountCells cells)
        int xmn = 0x7fffffff, ymn = 0x7fffffff, xmx = -1, ymx = -1;
        for (int i = tid; i < m; i += kThreads) {
            const uint32_t v = xy[base + i];
            const int x = ecc::xy_x(v), y = ecc::xy_y(v);
            xmn = min(xmn, x); ymn = min(ymn, y); xmx = max(xmx, x); ymx = max(ymx, y);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            xmn = min(xmn, __shfl_xor(xmn, o)); ymn = min(ymn, __shfl_xor(ymn, o));
            xmx = max(xmx, __shfl_xor(xmx, o)); ymx = max(ymx, __shfl_xor(ymx, o));
        }
        if (lane == 0) {
            red[4 * (tid >> 6) + 0] = xmn; red[4 * (tid >> 6) + 1] = ymn;
            red[4 * (tid >> 6) + 2] = xmx; red[4 * (tid >> 6) + 3] = ymx;
        }
        for (int c = tid; c <= kCountCells; c += kThreads) cend[c] = 0u;
        __syncthreads();
        xmn = red[0]; ymn = red[1]; xmx = red[2]; ymx = red[3];
        for (int w = 1; w < kThreads / 64; ++w) {
            xmn = min(xmn, red[4 * w]); ymn = min(ymn, red[4 * w + 1]);
            xmx = max(xmx, red[4 * w + 2]); ymx = max(ymx, red[4 * w + 3]);
        }
        if (m == 0) { xmn = ymn = 0; xmx = ymx = 0; }
        int cs = e_int + 1;  // > eps: a neighbour lies in the same or an adjacent cell
        while ((int64_t)((xmx - xmn) / cs + 1) * ((ymx - ymn) / cs + 1) > kCountCells) cs *= 2;
        const int gx = (xmx - xmn) / cs + 1, gy = (ymx - ymn) / cs + 1;
        __syncthreads();  // red reusable
        for (int i = tid; i < m; i += kThreads) {
            const uint32_t v = xy[base + i];
            atomicAdd(&cend[((ecc::xy_y(v) - ymn) / cs) * gx + (ecc::xy_x(v) - xmn) / cs], 1u);
        }
        __syncthreads();
        {  // exclusive scan of the cell counts in place (kCountCells / kThreads per thread)
            constexpr int per = kCountCells / kThreads;
            uint32_t loc[per], sum = 0;
#pragma unroll
            for (int k = 0; k < per; ++k) { loc[k] = cend[tid * per + k]; sum += loc[k]; }
            uint32_t inc = sum;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(inc, o);
                if (lane >= o) inc += y;
            }
            if (lane == 63) red[16 + (tid >> 6)] = (int)inc;
            __syncthreads();
            uint32_t off = inc - sum;
            for (int w = 0; w < (tid >> 6); ++w) off += (uint32_t)red[16 + w];
#pragma unroll
            for (int k = 0; k < per; ++k) { cend[tid * per + k] = off; off += loc[k]; }
        }
        __syncthreads();
        for (int i = tid; i < m; i += kThreads) {  // scatter; afterwards cend[c] = end of cell c
            const uint32_t v = xy[base + i];
            const uint32_t at = atomicAdd(&cend[((ecc::xy_y(v) - ymn) / cs) * gx + (ecc::xy_x(v) - xmn) / cs], 1u);
            spt[at] = v;
            sidx[at] = (uint16_t)i;
        }
        for (int i = m + tid; i < sv.stride; i += kThreads) {
            counts[base + i] = 0;
            if (core) core[base + i] = -1.0;
        }
        __syncthreads();
        // queries in cell order: a wave's lanes walk the same or neighbouring runs (broadcast reads)
        for (int q = tid; q < m; q += kThreads) {
            const uint32_t v = spt[q];
            const int i = sidx[q];
            const int x = ecc::xy_x(v), y = ecc::xy_y(v);
            const int cx = (x - xmn) / cs, cy = (y - ymn) / cs;
            const int c0 = max(cx - 1, 0), c1 = min(cx + 1, gx - 1);
            int cnt = 0;
            int best[K];
#pragma unroll
            for (int k = 0; k < K; ++k) best[k] = 0x7fffffff;
            for (int ry = max(cy - 1, 0); ry <= min(cy + 1, gy - 1); ++ry) {
                const int cl = ry * gx + c0, ch = ry * gx + c1;
                const int hi = (int)cend[ch];
#pragma unroll 4
                for (int a = cl == 0 ? 0 : (int)cend[cl - 1]; a < hi; ++a) {
                    const uint32_t w = spt[a];
                    const uint32_t ax = (uint32_t)abs(ecc::xy_x(w) - x), ay = (uint32_t)abs(ecc::xy_y(w) - y);
                    const uint32_t d2 = ax * ax + ay * ay;  // exact whenever ax, ay <= e_int <= 32767
                    const bool in = ax <= (uint32_t)e_int && ay <= (uint32_t)e_int && d2 <= (uint32_t)r2i;
                    cnt += in ? 1 : 0;
                    if (in) {
                        if (core) {
                            int val = (int)d2;  // insertion network keeps the K smallest, sorted
#pragma unroll
                            for (int k = 0; k < K; ++k) {
                                const int lo2 = min(best[k], val);
                                val = max(best[k], val);
                                best[k] = lo2;
                            }
                        }
                    }
                }
            }
            counts[base + i] = cnt;
            if (core) {
                double cd = -1.0;
                if (cnt >= min_pts && min_pts >= 1) {
                    int sel = 0;
#pragma unroll
                    for (int k = 0; k < K; ++k) sel = (k == min_pts - 1) ? best[k] : sel;
                    cd = sqrt((double)sel);
                }
                core[base + i] = cd;
            }
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(kThreads)
eps_lists_kernel(const uint32_t *__restrict__ xy, SegView sv, double eps,
                 const int64_t *__restrict__ offsets, int32_t *__restrict__ nbr, int64_t nbr_cap,
                 int32_t *__restrict__ err) {
    __shared__ uint32_t pxy[kMaxPts];
    __shared__ uint16_t sorted[kMaxPts];
    __shared__ uint32_t cend[kMaxCells];
    __shared__ int red[32];
    const double r2 = eps * eps;
    for (int64_t s = blockIdx.x; s < sv.n_segs; s += gridDim.x) {
        Grid g;
        const int m = bin_segment(xy, sv, s, eps, pxy, sorted, cend, red, g);
        const int64_t base = s * sv.stride;
        for (int i = threadIdx.x; i < m; i += kThreads) {
            const uint32_t v = pxy[i];
            const int x = ecc::xy_x(v), y = ecc::xy_y(v);
            const int cx = (x - g.xmin) / g.cs, cy = (y - g.ymin) / g.cs;
            int lo[9], hi[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) cell_range(g, cend, cx + (k % 3) - 1, cy + (k / 3) - 1, lo[k], hi[k]);
            int64_t out = offsets[base + i];
            const int64_t end = offsets[base + i + 1];
            // 9-way merge of ascending cell lists
            for (;;) {
                int bestk = -1, besti = 0x7fffffff;
#pragma unroll
                for (int k = 0; k < 9; ++k) {
                    if (lo[k] < hi[k]) {
                        const int idx = sorted[lo[k]];
                        if (idx < besti) { besti = idx; bestk = k; }
                    }
                }
                if (bestk < 0) break;
#pragma unroll
                for (int k = 0; k < 9; ++k) lo[k] += (k == bestk) ? 1 : 0;
                const uint32_t w = pxy[besti];
                const int ex = ecc::xy_x(w) - x, ey = ecc::xy_y(w) - y;
                if ((double)(ex * ex + ey * ey) <= r2) {
                    if (out < end && out < nbr_cap) nbr[out] = besti;
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
    const int K = core_dist ? min_pts : 1;
    auto kern = K <= 1 ? eps_counts_kernel<1> : K <= 2 ? eps_counts_kernel<2> : K <= 4 ? eps_counts_kernel<4>
              : K <= 8 ? eps_counts_kernel<8> : K <= 16 ? eps_counts_kernel<16> : K <= 32 ? eps_counts_kernel<32>
              : eps_counts_kernel<64>;
    const size_t lds = (size_t)(kCountCells + 1 + seg_stride) * sizeof(uint32_t) + (size_t)seg_stride * sizeof(uint16_t);
    ECC_CHECK_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                  "eps_counts lds");
    // enough workgroups for every CU at the occupancy the LDS allows (segments are grid-strided)
    const unsigned grid = (unsigned)std::min<int64_t>(n_segs, 8192);
    {
        ECC_TIMED(ctx, ecc::as_stream(stream), "eps_counts_kernel");
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, ecc::as_stream(stream), xy, sv, e_int, r2i,
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
    const unsigned grid = (unsigned)std::min<int64_t>(n_segs, 4096);
    {
        ECC_TIMED(ctx, s, "eps_lists_kernel");
        hipLaunchKernelGGL(eps_lists_kernel, dim3(grid), dim3(kThreads), 0, s, xy, sv, eps,
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
