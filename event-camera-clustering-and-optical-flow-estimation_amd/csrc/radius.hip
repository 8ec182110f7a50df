// Radius (eps-ball) neighbourhoods of an arbitrary fp64 point set in 1-3 dimensions: counts,
// OPTICS core distances and neighbour lists for ONE global problem of any size (SURVEY.md §8a
// rows a11-a12, §8f rank 3; the generalisation the int 2-D, <= 16384-point windows of eps.hip
// do not cover).
//
// Reference: kdt::KDTree::radius_search, OPT/include/optics/kdTree.hpp:407-422 — a leaf keeps
// index i iff square_distance(points[i], p) <= radius * radius (:218-226), square_distance =
// sum over dimensions of d * d with d = p1[i] - p2[i] in double (:180-192); neighbours include
// the point itself.  optics::compute_core_dist (optics.hpp:286-299): no core point below
// min_pts neighbours, else the distance to the (min_pts-1)-th nearest of the ball (nth_element
// of the squared distances, then dist = sqrt of that squared distance).  The result of the
// OPTICS expansion (optics.hpp:525-555) does not depend on the order of a neighbour list, so the
// lists come out in grid order.
//
// MI355X design: a uniform grid over the point set's bounding box with cells slightly wider than
// eps (so a neighbour is in the 3^D cells around a point), as many cells as 4 per point at most
// (the cell doubles until they fit): bounding box by a reduction into order-preserving int64
// keys, the grid geometry by one lane, a counting sort of the points by cell (histogram, device
// scan, scatter of the coordinates into cell-ordered SoA arrays), then one lane per point in
// cell order (neighbouring lanes walk the same cells: coalesced, L2-resident candidate reads)
// computing d^2 in the reference's operation order (no FMA contraction), the count, the K
// smallest d^2 in a register insertion network (core distance = correctly rounded sqrt) and, in
// the list pass, the indices at offsets from a device scan of the counts.
#include "ecc_internal.hpp"

#include <cmath>

namespace {

constexpr int kThreads = 256;
constexpr int kFlagWord = 6;   // ctx->flags[6]: bit 1 list capacity exceeded
constexpr int kGridWord = 16;  // ctx->flags[16..]: bounding-box keys, then the grid geometry

struct GridF64 {
    double mn[3];
    double cs;
    int64_t dims[3];
    int64_t n_cells;
    int dim;
};

// order-preserving int64 key of a double (and back)
__device__ __forceinline__ int64_t dkey(double v) {
    const int64_t b = __double_as_longlong(v);
    return b >= 0 ? b : b ^ 0x7fffffffffffffffll;
}
__device__ __forceinline__ double dval(int64_t k) {
    return __longlong_as_double(k >= 0 ? k : k ^ 0x7fffffffffffffffll);
}

__global__ void __launch_bounds__(kThreads)
bbox_init_kernel(int64_t *keys) {
    if (threadIdx.x < 3) keys[threadIdx.x] = 0x7fffffffffffffffll;            // min
    else if (threadIdx.x < 6) keys[threadIdx.x] = (int64_t)0x8000000000000000ull;  // max
}

__global__ void __launch_bounds__(kThreads)
bbox_kernel(const double *__restrict__ pts, int64_t n, int dim, int64_t *keys) {
    int64_t mn[3] = {0x7fffffffffffffffll, 0x7fffffffffffffffll, 0x7fffffffffffffffll};
    int64_t mx[3] = {(int64_t)0x8000000000000000ull, (int64_t)0x8000000000000000ull, (int64_t)0x8000000000000000ull};
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            if (d >= dim) break;
            const int64_t k = dkey(pts[i * dim + d]);
            mn[d] = k < mn[d] ? k : mn[d];
            mx[d] = k > mx[d] ? k : mx[d];
        }
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int64_t a = __shfl_xor(mn[d], o), b = __shfl_xor(mx[d], o);
            mn[d] = a < mn[d] ? a : mn[d];
            mx[d] = b > mx[d] ? b : mx[d];
        }
    }
    if ((threadIdx.x & 63) == 0)
        for (int d = 0; d < dim; ++d) {
            atomicMin(reinterpret_cast<long long *>(keys + d), (long long)mn[d]);
            atomicMax(reinterpret_cast<long long *>(keys + 3 + d), (long long)mx[d]);
        }
}

// The grid: cells of eps * (1 + 1e-6) (so that |p - q| <= eps keeps the floor of (p - mn) / cs
// within one cell despite rounding), doubled until at most max_cells cells.
__global__ void grid_setup_kernel(const int64_t *keys, int dim, double eps, int64_t max_cells, GridF64 *g) {
    if (threadIdx.x != 0) return;
    GridF64 r{};
    r.dim = dim;
    double cs = eps > 0.0 ? eps * (1.0 + 1e-6) : 1.0;
    double span[3] = {0.0, 0.0, 0.0};
    for (int d = 0; d < dim; ++d) {
        r.mn[d] = dval(keys[d]);
        span[d] = dval(keys[3 + d]) - r.mn[d];
    }
    for (;;) {
        int64_t cells = 1;
        bool ok = true;
        for (int d = 0; d < dim; ++d) {
            const double c = floor(span[d] / cs) + 1.0;
            if (!(c < 4.0e18)) { ok = false; break; }
            r.dims[d] = (int64_t)c;
            if (cells > max_cells / r.dims[d] + 1) { ok = false; break; }
            cells *= r.dims[d];
        }
        if (ok && cells <= max_cells) {
            r.n_cells = cells;
            break;
        }
        cs *= 2.0;
    }
    for (int d = dim; d < 3; ++d) r.dims[d] = 1;
    r.cs = cs;
    *g = r;
}

__device__ __forceinline__ int64_t cell_coord(double v, double mn, double cs, int64_t dims) {
    int64_t c = (int64_t)floor((v - mn) / cs);
    return c < 0 ? 0 : (c >= dims ? dims - 1 : c);
}

__global__ void __launch_bounds__(kThreads)
cell_count_kernel(const double *__restrict__ pts, int64_t n, const GridF64 *__restrict__ gp, int32_t *__restrict__ cell_of,
                  int32_t *__restrict__ cell_cnt) {
    const GridF64 g = *gp;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
        int64_t c = 0;
        for (int d = g.dim - 1; d >= 0; --d) c = c * g.dims[d] + cell_coord(pts[i * g.dim + d], g.mn[d], g.cs, g.dims[d]);
        cell_of[i] = (int32_t)c;
        atomicAdd(&cell_cnt[c], 1);
    }
}

__global__ void __launch_bounds__(kThreads)
cell_scatter_kernel(const double *__restrict__ pts, int64_t n, int dim, const int32_t *__restrict__ cell_of,
                    const int64_t *__restrict__ cell_off, int32_t *__restrict__ cursor, int32_t *__restrict__ sidx,
                    double *__restrict__ sc) {
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
        const int32_t c = cell_of[i];
        const int64_t pos = cell_off[c] + atomicAdd(&cursor[c], 1);
        sidx[pos] = (int32_t)i;
        for (int d = 0; d < dim; ++d) sc[(int64_t)d * n + pos] = pts[i * dim + d];
    }
}

// One lane per point in cell order.  K = 0: counts only; otherwise the K smallest d^2 (K >=
// min_pts).  kLists: write the neighbour indices at offsets[i].
template <int D, int K, bool kLists>
__global__ void __launch_bounds__(kThreads)
radius_query_kernel(const GridF64 *__restrict__ gp, int64_t n, const int32_t *__restrict__ sidx, const double *__restrict__ sc,
                    const int64_t *__restrict__ cell_off, double eps2, int min_pts, int32_t *__restrict__ counts,
                    double *__restrict__ core, const int64_t *__restrict__ offsets, int32_t *__restrict__ nbr,
                    double *__restrict__ nbr_dist, int64_t nbr_cap, int32_t *__restrict__ err) {
    const GridF64 g = *gp;
    const int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (k >= n) return;
    const int32_t i = sidx[k];
    double p[3];
    int64_t c[3];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        p[d] = sc[(int64_t)d * n + k];
        c[d] = cell_coord(p[d], g.mn[d], g.cs, g.dims[d]);
    }
    int cnt = 0;
    double best[K > 0 ? K : 1];
#pragma unroll
    for (int q = 0; q < (K > 0 ? K : 1); ++q) best[q] = __longlong_as_double(0x7ff0000000000000ll);  // +inf
    int64_t out = kLists ? offsets[i] : 0;
    const int64_t end = kLists ? offsets[i + 1] : 0;
    // the 3^D cells around the point; the last dimension's neighbours are contiguous runs
    const int64_t z0 = D >= 3 ? (c[2] > 0 ? c[2] - 1 : 0) : 0, z1 = D >= 3 ? (c[2] + 1 < g.dims[2] ? c[2] + 1 : c[2]) : 0;
    const int64_t y0 = D >= 2 ? (c[1] > 0 ? c[1] - 1 : 0) : 0, y1 = D >= 2 ? (c[1] + 1 < g.dims[1] ? c[1] + 1 : c[1]) : 0;
    const int64_t x0 = c[0] > 0 ? c[0] - 1 : 0, x1 = c[0] + 1 < g.dims[0] ? c[0] + 1 : c[0];
    for (int64_t z = z0; z <= z1; ++z)
        for (int64_t y = y0; y <= y1; ++y) {
            const int64_t row = (z * g.dims[1] + y) * g.dims[0];
            const int64_t lo = cell_off[row + x0], hi = cell_off[row + x1 + 1];
            for (int64_t j = lo; j < hi; ++j) {
                // square_distance (kdTree.hpp:180-192): d = p1[i] - p2[i], result += d * d
                double s = 0.0;
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    const double dd = sc[(int64_t)d * n + j] - p[d];
                    s = __dadd_rn(s, __dmul_rn(dd, dd));
                }
                if (!(s <= eps2)) continue;
                ++cnt;
                if (K > 0) {
                    double v = s;
#pragma unroll
                    for (int q = 0; q < (K > 0 ? K : 1); ++q) {
                        const double lo2 = fmin(best[q], v);
                        v = fmax(best[q], v);
                        best[q] = lo2;
                    }
                }
                if (kLists) {
                    if (out < end && out < nbr_cap) {
                        nbr[out] = sidx[j];
                        if (nbr_dist) nbr_dist[out] = sqrt(s);  // geom::dist = sqrt(square_dist)
                    } else {
                        *err = 1;
                    }
                    ++out;
                }
            }
        }
    if (!kLists) {
        counts[i] = cnt;
        if (core) {
            double cd = -1.0;
            if (K > 0 && cnt >= min_pts) {
                double sel = 0.0;
#pragma unroll
                for (int q = 0; q < (K > 0 ? K : 1); ++q) sel = (q == min_pts - 1) ? best[q] : sel;
                cd = sqrt(sel);  // correctly rounded
            }
            core[i] = cd;
        }
    }
}

struct RadiusWs {
    int64_t *keys;
    GridF64 *grid;
    int32_t *cell_cnt, *cell_of, *sidx;
    int64_t *cell_off, *scan;
    double *sc;
    int64_t max_cells;
};

int radius_build(ecc_ctx *ctx, const double *pts, int64_t n, int dim, double eps, hipStream_t s, RadiusWs &w) {
    w.max_cells = std::max<int64_t>(4 * n, 4096);
    const size_t need = ecc::align_up((size_t)w.max_cells * 4, 256) + ecc::align_up((size_t)(w.max_cells + 1) * 8, 256) +
                        ecc::align_up(ecc::scan_scratch_bytes(std::max<int64_t>(w.max_cells, n)), 256) +
                        2 * ecc::align_up((size_t)n * 4, 256) + ecc::align_up((size_t)n * 8 * dim, 256) +
                        ecc::align_up((size_t)(n + 1) * 8, 256);
    int rc = ecc::ws_reserve(ctx, need);
    if (rc) return rc;
    char *p = static_cast<char *>(ctx->ws);
    auto carve = [&](size_t bytes) { char *r = p; p += ecc::align_up(bytes, 256); return r; };
    w.cell_cnt = reinterpret_cast<int32_t *>(carve((size_t)w.max_cells * 4));
    w.cell_off = reinterpret_cast<int64_t *>(carve((size_t)(w.max_cells + 1) * 8));
    w.scan = reinterpret_cast<int64_t *>(carve(ecc::scan_scratch_bytes(std::max<int64_t>(w.max_cells, n))));
    w.cell_of = reinterpret_cast<int32_t *>(carve((size_t)n * 4));
    w.sidx = reinterpret_cast<int32_t *>(carve((size_t)n * 4));
    w.sc = reinterpret_cast<double *>(carve((size_t)n * 8 * dim));
    w.keys = reinterpret_cast<int64_t *>(ctx->flags + kGridWord);
    w.grid = reinterpret_cast<GridF64 *>(ctx->flags + kGridWord + 12);
    const unsigned blocks = (unsigned)std::min<int64_t>((n + kThreads - 1) / kThreads, 4096);
    hipLaunchKernelGGL(bbox_init_kernel, dim3(1), dim3(kThreads), 0, s, w.keys);
    {
        ECC_TIMED(ctx, s, "radius_grid_kernels");
        hipLaunchKernelGGL(bbox_kernel, dim3(blocks), dim3(kThreads), 0, s, pts, n, dim, w.keys);
        hipLaunchKernelGGL(grid_setup_kernel, dim3(1), dim3(64), 0, s, (const int64_t *)w.keys, dim, eps, w.max_cells,
                           w.grid);
        ECC_CHECK_HIP(ctx, hipMemsetAsync(w.cell_cnt, 0, (size_t)w.max_cells * 4, s), "memset(cells)");
        hipLaunchKernelGGL(cell_count_kernel, dim3(blocks), dim3(kThreads), 0, s, pts, n, (const GridF64 *)w.grid,
                           w.cell_of, w.cell_cnt);
    }
    rc = ecc::exclusive_scan_i32_i64(ctx, w.cell_cnt, w.max_cells, w.cell_off, w.scan, s);
    if (rc) return rc;
    ECC_CHECK_HIP(ctx, hipMemsetAsync(w.cell_cnt, 0, (size_t)w.max_cells * 4, s), "memset(cursor)");
    {
        ECC_TIMED(ctx, s, "radius_scatter_kernel");
        hipLaunchKernelGGL(cell_scatter_kernel, dim3(blocks), dim3(kThreads), 0, s, pts, n, dim, (const int32_t *)w.cell_of,
                           (const int64_t *)w.cell_off, w.cell_cnt, w.sidx, w.sc);
    }
    ECC_CHECK_LAUNCH(ctx, "radius grid");
    return ECC_OK;
}

template <int D>
int radius_query(ecc_ctx *ctx, const RadiusWs &w, int64_t n, double eps, int min_pts, int32_t *counts, double *core,
                 const int64_t *offsets, int32_t *nbr, double *nbr_dist, int64_t nbr_cap, hipStream_t s) {
    const double eps2 = eps * eps;  // radius * radius (kdTree.hpp:220)
    const unsigned blocks = (unsigned)((n + kThreads - 1) / kThreads);
    using Kern = void (*)(const GridF64 *, int64_t, const int32_t *, const double *, const int64_t *, double, int, int32_t *,
                          double *, const int64_t *, int32_t *, double *, int64_t, int32_t *);
    Kern kern;
    if (nbr) {
        kern = radius_query_kernel<D, 0, true>;
    } else {
        const int K = core ? min_pts : 0;
        kern = K == 0 ? radius_query_kernel<D, 0, false> : K <= 2 ? radius_query_kernel<D, 2, false>
             : K <= 4 ? radius_query_kernel<D, 4, false> : K <= 8 ? radius_query_kernel<D, 8, false>
             : K <= 16 ? radius_query_kernel<D, 16, false> : K <= 32 ? radius_query_kernel<D, 32, false>
             : radius_query_kernel<D, 64, false>;
    }
    {
        ECC_TIMED(ctx, s, nbr ? "radius_lists_kernel" : "radius_counts_kernel");
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(kThreads), 0, s, (const GridF64 *)w.grid, n, (const int32_t *)w.sidx,
                           (const double *)w.sc, (const int64_t *)w.cell_off, eps2, min_pts, counts, core, offsets, nbr,
                           nbr_dist, nbr_cap, ctx->flags + kFlagWord);
    }
    ECC_CHECK_LAUNCH(ctx, "radius_query_kernel");
    return ECC_OK;
}

int check_args(ecc_ctx *ctx, const double *pts, int64_t n, int32_t dim, double eps) {
    if (!ctx || n < 0 || dim < 1 || dim > 3 || !(eps >= 0.0) || !std::isfinite(eps)) return ECC_ERR_INVALID;
    if (n > 0 && !pts) return ECC_ERR_INVALID;
    if (n >= INT32_MAX) return ECC_ERR_INVALID;
    return ECC_OK;
}

int dispatch_query(ecc_ctx *ctx, const RadiusWs &w, int64_t n, int dim, double eps, int min_pts, int32_t *counts,
                   double *core, const int64_t *offsets, int32_t *nbr, double *nbr_dist, int64_t nbr_cap, hipStream_t s) {
    switch (dim) {
        case 1: return radius_query<1>(ctx, w, n, eps, min_pts, counts, core, offsets, nbr, nbr_dist, nbr_cap, s);
        case 2: return radius_query<2>(ctx, w, n, eps, min_pts, counts, core, offsets, nbr, nbr_dist, nbr_cap, s);
        default: return radius_query<3>(ctx, w, n, eps, min_pts, counts, core, offsets, nbr, nbr_dist, nbr_cap, s);
    }
}

}  // namespace

ECC_API int ecc_radius_counts_f64(ecc_ctx *ctx, const double *pts, int64_t n, int32_t dim, double eps, int32_t min_pts,
                                  int32_t *counts, double *core_dist, ecc_stream_t stream) {
    int rc = check_args(ctx, pts, n, dim, eps);
    if (rc) return rc;
    if (!counts || (core_dist && (min_pts < 1 || min_pts > 64))) return ECC_ERR_INVALID;
    if (n == 0) return ECC_OK;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    RadiusWs w;
    rc = radius_build(ctx, pts, n, dim, eps, s, w);
    if (rc) return rc;
    return dispatch_query(ctx, w, n, dim, eps, min_pts, counts, core_dist, nullptr, nullptr, nullptr, 0, s);
}

ECC_API int ecc_radius_lists_f64(ecc_ctx *ctx, const double *pts, int64_t n, int32_t dim, double eps,
                                 const int32_t *counts, int64_t *offsets, int32_t *nbr, double *nbr_dist,
                                 int64_t nbr_cap, ecc_stream_t stream) {
    int rc = check_args(ctx, pts, n, dim, eps);
    if (rc) return rc;
    if (!counts || !offsets || nbr_cap < 0 || (nbr_cap > 0 && !nbr)) return ECC_ERR_INVALID;
    if (n == 0) return ECC_OK;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    ECC_CHECK_HIP(ctx, hipMemsetAsync(ctx->flags + kFlagWord, 0, 4, s), "memset(radius err)");
    if (!nbr) {  // size query: the offsets only (offsets[n] = entries needed)
        rc = ecc::ws_reserve(ctx, ecc::scan_scratch_bytes(n));
        if (rc) return rc;
        return ecc::exclusive_scan_i32_i64(ctx, counts, n, offsets, reinterpret_cast<int64_t *>(ctx->ws), s);
    }
    RadiusWs w;
    rc = radius_build(ctx, pts, n, dim, eps, s, w);
    if (rc) return rc;
    rc = ecc::exclusive_scan_i32_i64(ctx, counts, n, offsets, w.scan, s);
    if (rc) return rc;
    return dispatch_query(ctx, w, n, dim, eps, 1, nullptr, nullptr, offsets, nbr, nbr_dist, nbr_cap, s);
}

ECC_API int ecc_radius_status(ecc_ctx *ctx, ecc_stream_t stream) {
    if (!ctx) return ECC_ERR_INVALID;
    int32_t f = 0;
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(&f, ctx->flags + kFlagWord, 4, hipMemcpyDeviceToHost, ecc::as_stream(stream)),
                  "read radius err");
    ECC_CHECK_HIP(ctx, hipStreamSynchronize(ecc::as_stream(stream)), "sync");
    return f ? ECC_ERR_CAPACITY : ECC_OK;
}
