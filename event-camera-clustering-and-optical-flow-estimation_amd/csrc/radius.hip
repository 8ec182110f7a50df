// Radius (eps-ball) neighbourhoods of an arbitrary fp64 or fp32 point set in 1-3 dimensions: counts,
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
// the list pass, the indices at offsets from a device scan of the counts.  min_pts above the
// network's 64 takes a wave-per-point radix select (8 passes of 8 bits over the d^2 bit
// patterns, an LDS histogram per wave) after the count pass: no cap on min_pts, as
// compute_core_dist has none.  The grid itself is radius_grid.hpp (shared with the any-N DBSCAN).
#include "radius_grid.hpp"
#include "sort_internal.hpp"

namespace {

using ecc::rgrid::Grid;
using ecc::rgrid::kThreads;
constexpr int kFlagWord = 6;  // ctx->flags[6]: bit 1 list capacity exceeded

// One lane per point in cell order.  K = 0: counts only; otherwise the K smallest d^2 (K >=
// min_pts).  kLists: write the neighbour indices at offsets[i].
template <typename T, int D, int K, bool kLists>
__global__ void __launch_bounds__(kThreads)
radius_query_kernel(const Grid *__restrict__ gp, int64_t n, const int32_t *__restrict__ sidx, const T *__restrict__ sc,
                    const int64_t *__restrict__ cell_off, double eps2, int min_pts, int32_t *__restrict__ counts,
                    double *__restrict__ core, const int64_t *__restrict__ offsets, int32_t *__restrict__ nbr,
                    double *__restrict__ nbr_dist, int64_t nbr_cap, int32_t *__restrict__ err) {
    const Grid g = *gp;
    const int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (k >= n) return;
    const int32_t i = sidx[k];
    T p[3];
#pragma unroll
    for (int d = 0; d < D; ++d) p[d] = sc[(int64_t)d * n + k];
    int cnt = 0;
    double best[K > 0 ? K : 1];
#pragma unroll
    for (int q = 0; q < (K > 0 ? K : 1); ++q) best[q] = __longlong_as_double(0x7ff0000000000000ll);  // +inf
    int64_t out = kLists ? offsets[i] : 0;
    const int64_t end = kLists ? offsets[i + 1] : 0;
    ecc::rgrid::for_runs<T, D>(g, cell_off, p, [&](int64_t lo, int64_t hi) {
        for (int64_t j = lo; j < hi; ++j) {
            const double s = ecc::rgrid::sq_dist<T, D>(sc, n, j, p);
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
    });
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

// Core distance for min_pts above the register network: one wave per point (in cell order),
// the (min_pts-1)-th smallest d^2 of its eps-ball by an 8-pass radix select over the d^2 bit
// patterns (d^2 >= 0: the IEEE bits order like the values), each pass a wave walk of the
// candidate runs into a 256-bin LDS histogram.  Points with count < min_pts get -1.
constexpr int kSelWaves = kThreads / 64;

template <typename T, int D>
__global__ void __launch_bounds__(kThreads)
radius_core_select_kernel(const Grid *__restrict__ gp, int64_t n, const int32_t *__restrict__ sidx,
                          const T *__restrict__ sc, const int64_t *__restrict__ cell_off, double eps2, int min_pts,
                          const int32_t *__restrict__ counts, double *__restrict__ core) {
    __shared__ uint32_t hist[kSelWaves][256];
    const Grid g = *gp;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t *h = hist[wv];
    for (int64_t k = (int64_t)blockIdx.x * kSelWaves + wv; k < n; k += (int64_t)gridDim.x * kSelWaves) {
        const int32_t i = sidx[k];
        if (counts[i] < min_pts) {
            if (lane == 0) core[i] = -1.0;
            continue;
        }
        T p[3];
#pragma unroll
        for (int d = 0; d < D; ++d) p[d] = sc[(int64_t)d * n + k];
        uint64_t prefix = 0;
        uint32_t rank = (uint32_t)(min_pts - 1);  // 0-based rank among the remaining candidates
        for (int pass = 0; pass < 8; ++pass) {
            const int shift = 56 - 8 * pass;
            for (int b = lane; b < 256; b += 64) h[b] = 0;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            const uint64_t hi_mask = pass == 0 ? 0ull : (~0ull << (shift + 8));
            ecc::rgrid::for_runs<T, D>(g, cell_off, p, [&](int64_t lo, int64_t hi) {
                for (int64_t j = lo + lane; j < hi; j += 64) {
                    const double s = ecc::rgrid::sq_dist<T, D>(sc, n, j, p);
                    if (!(s <= eps2)) continue;
                    const uint64_t key = (uint64_t)__double_as_longlong(s);
                    if ((key & hi_mask) != prefix) continue;
                    atomicAdd(&h[(key >> shift) & 255u], 1u);
                }
            });
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            // lane owns bins 4*lane .. 4*lane+3; find the bin holding rank
            const uint32_t c0 = h[4 * lane], c1 = h[4 * lane + 1], c2 = h[4 * lane + 2], c3 = h[4 * lane + 3];
            const uint32_t mine = c0 + c1 + c2 + c3;
            uint32_t inc = mine;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(inc, o);
                if (lane >= o) inc += y;
            }
            const uint32_t before = inc - mine;
            const bool here = rank >= before && rank < inc;
            uint32_t digit = 0, below = 0;
            if (here) {
                uint32_t r = rank - before;
                if (r < c0) { digit = 0; below = 0; }
                else if (r < c0 + c1) { digit = 1; below = c0; }
                else if (r < c0 + c1 + c2) { digit = 2; below = c0 + c1; }
                else { digit = 3; below = c0 + c1 + c2; }
                digit += 4 * lane;
                below += before;
            }
            const uint64_t ball = __ballot(here);
            const int src = ball ? __ffsll((unsigned long long)ball) - 1 : 0;
            digit = __shfl(digit, src);
            below = __shfl(below, src);
            prefix |= (uint64_t)digit << shift;
            rank -= below;
            __builtin_amdgcn_wave_barrier();
        }
        if (lane == 0) core[i] = sqrt(__longlong_as_double((long long)prefix));  // correctly rounded
    }
}

template <typename T, int D>
int radius_query(ecc_ctx *ctx, const ecc::rgrid::Ws &w, int64_t n, double eps, int min_pts, int32_t *counts,
                 double *core, const int64_t *offsets, int32_t *nbr, double *nbr_dist, int64_t nbr_cap, hipStream_t s) {
    const double eps2 = eps * eps;  // radius * radius (kdTree.hpp:220)
    const unsigned blocks = (unsigned)((n + kThreads - 1) / kThreads);
    using Kern = void (*)(const Grid *, int64_t, const int32_t *, const T *, const int64_t *, double, int, int32_t *,
                          double *, const int64_t *, int32_t *, double *, int64_t, int32_t *);
    Kern kern;
    const bool select = !nbr && core && min_pts > 64;
    if (nbr) {
        kern = radius_query_kernel<T, D, 0, true>;
    } else {
        const int K = core && !select ? min_pts : 0;
        kern = K == 0 ? radius_query_kernel<T, D, 0, false> : K <= 2 ? radius_query_kernel<T, D, 2, false>
             : K <= 4 ? radius_query_kernel<T, D, 4, false> : K <= 8 ? radius_query_kernel<T, D, 8, false>
             : K <= 16 ? radius_query_kernel<T, D, 16, false> : K <= 32 ? radius_query_kernel<T, D, 32, false>
             : radius_query_kernel<T, D, 64, false>;
    }
    const T *sc = reinterpret_cast<const T *>(w.sc);
    {
        ECC_TIMED(ctx, s, nbr ? "radius_lists_kernel" : "radius_counts_kernel");
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(kThreads), 0, s, (const Grid *)w.grid, n, (const int32_t *)w.sidx, sc,
                           (const int64_t *)w.cell_off, eps2, min_pts, counts, select ? nullptr : core, offsets, nbr,
                           nbr_dist, nbr_cap, ctx->flags + kFlagWord);
    }
    ECC_CHECK_LAUNCH(ctx, "radius_query_kernel");
    if (select) {
        const unsigned sb = (unsigned)std::min<int64_t>((n + kSelWaves - 1) / kSelWaves, 65536);
        ECC_TIMED(ctx, s, "radius_core_select_kernel");
        hipLaunchKernelGGL((radius_core_select_kernel<T, D>), dim3(sb), dim3(kThreads), 0, s, (const Grid *)w.grid, n,
                           (const int32_t *)w.sidx, sc, (const int64_t *)w.cell_off, eps2, min_pts,
                           (const int32_t *)counts, core);
        ECC_CHECK_LAUNCH(ctx, "radius_core_select_kernel");
    }
    return ECC_OK;
}

int check_args(ecc_ctx *ctx, const void *pts, int64_t n, int32_t dim, double eps) {
    if (!ctx || n < 0 || dim < 1 || dim > 3 || !(eps >= 0.0) || !std::isfinite(eps)) return ECC_ERR_INVALID;
    if (n > 0 && !pts) return ECC_ERR_INVALID;
    if (n >= INT32_MAX) return ECC_ERR_INVALID;
    return ECC_OK;
}

template <typename T>
int dispatch_query(ecc_ctx *ctx, const ecc::rgrid::Ws &w, int64_t n, int dim, double eps, int min_pts, int32_t *counts,
                   double *core, const int64_t *offsets, int32_t *nbr, double *nbr_dist, int64_t nbr_cap, hipStream_t s) {
    switch (dim) {
        case 1: return radius_query<T, 1>(ctx, w, n, eps, min_pts, counts, core, offsets, nbr, nbr_dist, nbr_cap, s);
        case 2: return radius_query<T, 2>(ctx, w, n, eps, min_pts, counts, core, offsets, nbr, nbr_dist, nbr_cap, s);
        default: return radius_query<T, 3>(ctx, w, n, eps, min_pts, counts, core, offsets, nbr, nbr_dist, nbr_cap, s);
    }
}

template <typename T>
int radius_build_ws(ecc_ctx *ctx, const T *pts, int64_t n, int dim, double eps, hipStream_t s, ecc::rgrid::Ws &w) {
    int rc = ecc::ws_reserve(ctx, ecc::rgrid::ws_bytes(n, dim, sizeof(T)));
    if (rc) return rc;
    return ecc::rgrid::build<T>(ctx, pts, n, dim, eps, s, static_cast<char *>(ctx->ws), w);
}

template <typename T>
int radius_counts(ecc_ctx *ctx, const T *pts, int64_t n, int32_t dim, double eps, int32_t min_pts, int32_t *counts,
                  double *core_dist, ecc_stream_t stream) {
    int rc = check_args(ctx, pts, n, dim, eps);
    if (rc) return rc;
    if (!counts || (core_dist && min_pts < 1)) return ECC_ERR_INVALID;
    if (n == 0) return ECC_OK;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    ecc::rgrid::Ws w;
    rc = radius_build_ws<T>(ctx, pts, n, dim, eps, s, w);
    if (rc) return rc;
    return dispatch_query<T>(ctx, w, n, dim, eps, min_pts, counts, core_dist, nullptr, nullptr, nullptr, 0, s);
}

template <typename T>
int radius_lists(ecc_ctx *ctx, const T *pts, int64_t n, int32_t dim, double eps, const int32_t *counts,
                 int64_t *offsets, int32_t *nbr, double *nbr_dist, int64_t nbr_cap, ecc_stream_t stream) {
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
    ecc::rgrid::Ws w;
    rc = radius_build_ws<T>(ctx, pts, n, dim, eps, s, w);
    if (rc) return rc;
    rc = ecc::exclusive_scan_i32_i64(ctx, counts, n, offsets, w.scan, s);
    if (rc) return rc;
    return dispatch_query<T>(ctx, w, n, dim, eps, 1, nullptr, nullptr, offsets, nbr, nbr_dist, nbr_cap, s);
}

}  // namespace

ECC_API int ecc_radius_counts_f64(ecc_ctx *ctx, const double *pts, int64_t n, int32_t dim, double eps, int32_t min_pts,
                                  int32_t *counts, double *core_dist, ecc_stream_t stream) {
    return radius_counts<double>(ctx, pts, n, dim, eps, min_pts, counts, core_dist, stream);
}

ECC_API int ecc_radius_lists_f64(ecc_ctx *ctx, const double *pts, int64_t n, int32_t dim, double eps,
                                 const int32_t *counts, int64_t *offsets, int32_t *nbr, double *nbr_dist,
                                 int64_t nbr_cap, ecc_stream_t stream) {
    return radius_lists<double>(ctx, pts, n, dim, eps, counts, offsets, nbr, nbr_dist, nbr_cap, stream);
}

ECC_API int ecc_radius_counts_f32(ecc_ctx *ctx, const float *pts, int64_t n, int32_t dim, double eps, int32_t min_pts,
                                  int32_t *counts, double *core_dist, ecc_stream_t stream) {
    return radius_counts<float>(ctx, pts, n, dim, eps, min_pts, counts, core_dist, stream);
}

ECC_API int ecc_radius_lists_f32(ecc_ctx *ctx, const float *pts, int64_t n, int32_t dim, double eps,
                                 const int32_t *counts, int64_t *offsets, int32_t *nbr, double *nbr_dist,
                                 int64_t nbr_cap, ecc_stream_t stream) {
    return radius_lists<float>(ctx, pts, n, dim, eps, counts, offsets, nbr, nbr_dist, nbr_cap, stream);
}

ECC_API int ecc_radius_status(ecc_ctx *ctx, ecc_stream_t stream) {
    if (!ctx) return ECC_ERR_INVALID;
    int32_t f[2] = {0, 0};
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(f, ctx->flags + kFlagWord, 8, hipMemcpyDeviceToHost, ecc::as_stream(stream)),
                  "read radius err");
    ECC_CHECK_HIP(ctx, hipStreamSynchronize(ecc::as_stream(stream)), "sync");
    if (f[1]) return ECC_ERR_INVALID;  // flags[7]: a non-finite coordinate
    return f[0] ? ECC_ERR_CAPACITY : ECC_OK;
}

ECC_API int ecc_lists_sort_ascending(ecc_ctx *ctx, int64_t n, const int64_t *offsets, int64_t total, int32_t *nbr,
                                     double *nbr_dist, ecc_stream_t stream) {
    if (!ctx || n < 0 || total < 0 || total > UINT32_MAX || n > UINT32_MAX) return ECC_ERR_INVALID;
    if (n == 0 || total == 0) return ECC_OK;
    if (!offsets || !nbr) return ECC_ERR_INVALID;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    // the sort is out of place: keys (and values) go to the workspace, then back
    const size_t tmp = ecc::segsort_i32_temp_bytes(total, n, nbr_dist != nullptr);
    const size_t kb = ecc::align_up((size_t)total * 4, 256), vb = nbr_dist ? ecc::align_up((size_t)total * 8, 256) : 0;
    int rc = ecc::ws_reserve(ctx, kb + vb + ecc::align_up(tmp, 256));
    if (rc) return rc;
    char *p = static_cast<char *>(ctx->ws);
    int32_t *k2 = reinterpret_cast<int32_t *>(p);
    double *v2 = nbr_dist ? reinterpret_cast<double *>(p + kb) : nullptr;
    void *t = p + kb + vb;
    rc = ecc::segsort_i32(ctx, t, tmp, nbr, k2, nbr_dist, v2, total, n, offsets, s);
    if (rc) return rc;
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(nbr, k2, (size_t)total * 4, hipMemcpyDeviceToDevice, s), "copy lists");
    if (nbr_dist)
        ECC_CHECK_HIP(ctx, hipMemcpyAsync(nbr_dist, v2, (size_t)total * 8, hipMemcpyDeviceToDevice, s), "copy dists");
    return ECC_OK;
}
