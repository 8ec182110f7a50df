// DBSCAN over ONE point cloud of any size in 1-3 dimensions (fp32 pcl::PointXYZ-style or fp64
// coordinates): SURVEY.md §8a rows a9-a10 at the reference's own input type.
//
// Reference: DBSCANSimpleCluster::extract, PCC/DBSCAN_simple.h:27-90, with radiusSearch
// (:118-142, brute force: float per-axis differences widened to double, d^2 <= eps^2 in double,
// the point itself included) or DBSCANPrecompCluster's adjacency (DBSCAN_precomp.h:22-44, the
// same test).  The driver runs it on a float (x, y, z) cloud with eps 20, minPts 20 and clusters
// of 100..25000 points (PCC/pcl_cluster.cpp:112-123); north_star's event clouds are (x, y, t).
//
// The seed queue's outcome in closed form (as dbscan.hip, which does it per <= 16384-point
// window in LDS): a cluster is a core-connected component created in order of its smallest core
// index (the seed); a non-core point joins the first-created cluster holding one of its core
// neighbours, and also every later cluster whose SEED is its neighbour (a duplicate membership
// the reference emits); clusters of size in [min, max] are output by (size desc, smallest
// member asc, creation asc) — Q23 fixes the tie order of the reference's unstable std::sort.
//
// MI355X design, global memory throughout (no size cap):
//   grid (radius_grid.hpp: counting sort of the points by cell, cells > eps)
//   -> count + core flags (lane per point in cell order; 3^(D-1) contiguous candidate runs)
//   -> union over core-core pairs (global lock-free union-find: a CAS hooks the larger root
//      under the smaller, so a root is its component's minimum = the seed)
//   -> roots flagged, component ids by a device scan in ascending root (= creation) order
//   -> memberships: core points by component, non-core points' first claim and later seeds by
//      one walk of their candidates; sizes and first members by global atomics
//   -> output order: one stable radix sort (rocPRIM) of (size desc, first member asc) keys in
//      component order -> ranks
//   -> labels (coalesced, original order) + duplicate memberships.
// No neighbour lists are ever stored: every phase that needs a neighbourhood re-walks the cell
// runs, so the whole DBSCAN reads O(n) bytes plus the grid.
#include "radius_grid.hpp"
#include "sort_internal.hpp"

namespace {

using ecc::rgrid::Grid;
using ecc::rgrid::kThreads;
constexpr int kFlagWord = 8;  // ctx->flags[8]: bit 1 duplicate capacity exceeded
constexpr uint64_t kSentinel = (1ull << 62) - 1;

__device__ __forceinline__ int uf_find(int *parent, int x) {
    int p = parent[x];
    while (p != x) {
        const int gp = parent[p];
        if (gp != p) parent[x] = gp;  // path halving: gp is an ancestor of x (ancestry is permanent)
        x = p;
        p = gp;
    }
    return x;
}

__device__ __forceinline__ int uf_root(const int *parent, int x) {
    int p = parent[x];
    while (p != x) {
        x = p;
        p = parent[x];
    }
    return x;
}

__device__ __forceinline__ void uf_union(int *parent, int a, int b) {
    for (;;) {
        a = uf_find(parent, a);
        b = uf_find(parent, b);
        if (a == b) return;
        if (a > b) {
            const int t = a;
            a = b;
            b = t;
        }
        const int old = atomicCAS(&parent[b], b, a);  // hook the larger root under the smaller
        if (old == b) return;
        b = old;
    }
}

struct Cloud {
    const int32_t *sidx;
    const int64_t *cell_off;
    const void *sc;
    int64_t n;
    double eps2;
    int min_pts;
};

// 1. counts -> core flags; parent[i] = i for core points, -1 otherwise
template <typename T, int D>
__global__ void __launch_bounds__(kThreads)
db_core_kernel(const Grid *__restrict__ gp, Cloud c, int32_t *__restrict__ parent, uint8_t *__restrict__ core_s) {
    const Grid g = *gp;
    const int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (k >= c.n) return;
    const T *sc = static_cast<const T *>(c.sc);
    T p[3];
#pragma unroll
    for (int d = 0; d < D; ++d) p[d] = sc[(int64_t)d * c.n + k];
    // the point itself counts unconditionally (radiusSearch pushes `index` first,
    // DBSCAN_simple.h:124-125; DBSCAN_precomp.h:25-26): a non-finite point, whose distance to
    // itself is NaN, still has one neighbour and is core when min_pts <= 1.  Its cell coordinates
    // are the same in the count and the query (cell_coord), so the walk always reaches it.
    int cnt = 0;
    ecc::rgrid::for_runs<T, D>(g, c.cell_off, p, [&](int64_t lo, int64_t hi) {
        for (int64_t j = lo; j < hi; ++j) cnt += (j == k || ecc::rgrid::sq_dist<T, D>(sc, c.n, j, p) <= c.eps2) ? 1 : 0;
    });
    const bool core = cnt >= c.min_pts;
    const int32_t i = c.sidx[k];
    parent[i] = core ? i : -1;
    core_s[k] = core ? 1 : 0;
}

// 2. union over core-core pairs within eps (each unordered pair once: original index j > i)
template <typename T, int D>
__global__ void __launch_bounds__(kThreads)
db_union_kernel(const Grid *__restrict__ gp, Cloud c, const uint8_t *__restrict__ core_s, int32_t *parent) {
    const Grid g = *gp;
    const int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (k >= c.n || !core_s[k]) return;
    const T *sc = static_cast<const T *>(c.sc);
    T p[3];
#pragma unroll
    for (int d = 0; d < D; ++d) p[d] = sc[(int64_t)d * c.n + k];
    const int32_t i = c.sidx[k];
    ecc::rgrid::for_runs<T, D>(g, c.cell_off, p, [&](int64_t lo, int64_t hi) {
        for (int64_t j = lo; j < hi; ++j) {
            if (!core_s[j]) continue;
            const int32_t q = c.sidx[j];
            if (q <= i || !(ecc::rgrid::sq_dist<T, D>(sc, c.n, j, p) <= c.eps2)) continue;
            uf_union(parent, i, q);
        }
    });
}

// 3a. roots (core points that are their own parent) -> scan input
__global__ void __launch_bounds__(kThreads)
db_roots_kernel(int64_t n, const int32_t *__restrict__ parent, int32_t *__restrict__ is_root) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i < n) is_root[i] = parent[i] == (int32_t)i ? 1 : 0;
}

// 3b. component of every core point (ascending root order); sizes / first members of the core
//     memberships
__global__ void __launch_bounds__(kThreads)
db_comp_kernel(int64_t n, const int32_t *__restrict__ parent, const int64_t *__restrict__ cid,
               int32_t *__restrict__ comp, int32_t *c_size, int32_t *c_front) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    if (parent[i] == -1) {
        comp[i] = -1;
        return;
    }
    const int r = uf_root(parent, (int)i);
    const int cc = (int)cid[r];
    comp[i] = cc;
    atomicAdd(&c_size[cc], 1);
    atomicMin(&c_front[cc], (int)i);
}

// 4. non-core memberships: first claim (smallest component among core neighbours) and every
//    other cluster whose seed is a neighbour
template <typename T, int D>
__global__ void __launch_bounds__(kThreads)
db_member_kernel(const Grid *__restrict__ gp, Cloud c, const int32_t *__restrict__ comp,
                 const int32_t *__restrict__ is_root, int32_t *__restrict__ claim, uint8_t *__restrict__ more,
                 int32_t *c_size, int32_t *c_front) {
    const Grid g = *gp;
    const int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (k >= c.n) return;
    const int32_t i = c.sidx[k];
    if (comp[i] >= 0) return;
    const T *sc = static_cast<const T *>(c.sc);
    T p[3];
#pragma unroll
    for (int d = 0; d < D; ++d) p[d] = sc[(int64_t)d * c.n + k];
    int first = 0x7fffffff, n_seed = 0, seed_c = -1;
    ecc::rgrid::for_runs<T, D>(g, c.cell_off, p, [&](int64_t lo, int64_t hi) {
        for (int64_t j = lo; j < hi; ++j) {
            const int32_t q = c.sidx[j];
            const int cq = comp[q];
            if (cq < 0 || !(ecc::rgrid::sq_dist<T, D>(sc, c.n, j, p) <= c.eps2)) continue;
            first = cq < first ? cq : first;
            if (is_root[q]) {
                ++n_seed;
                seed_c = cq;
            }
        }
    });
    if (first == 0x7fffffff) {
        claim[i] = -1;  // noise
        more[i] = 0;
        return;
    }
    claim[i] = first;
    atomicAdd(&c_size[first], 1);
    atomicMin(&c_front[first], (int)i);
    const bool extra = !(n_seed == 0 || (n_seed == 1 && seed_c == first));
    more[i] = extra ? 1 : 0;
    if (!extra) return;
    ecc::rgrid::for_runs<T, D>(g, c.cell_off, p, [&](int64_t lo, int64_t hi) {
        for (int64_t j = lo; j < hi; ++j) {
            const int32_t q = c.sidx[j];
            if (!is_root[q] || comp[q] == first || !(ecc::rgrid::sq_dist<T, D>(sc, c.n, j, p) <= c.eps2)) continue;
            atomicAdd(&c_size[comp[q]], 1);
            atomicMin(&c_front[comp[q]], (int)i);
        }
    });
}

// 5a. sort keys: kept clusters (size in range) by (size desc, first member asc); the stable sort
//     keeps ascending component (creation) order among equal keys
__global__ void __launch_bounds__(kThreads)
db_keys_kernel(int64_t n, const int64_t *__restrict__ cid_total, const int32_t *__restrict__ c_size,
               const int32_t *__restrict__ c_front, int min_size, int max_size, uint64_t *__restrict__ keys,
               int32_t *__restrict__ vals) {
    const int64_t c = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (c >= n) return;
    const int64_t nc = *cid_total;
    uint64_t key = kSentinel;
    if (c < nc) {
        const int sz = c_size[c];
        if (sz >= min_size && sz <= max_size)
            key = ((uint64_t)(0x7fffffff - sz) << 31) | (uint64_t)(uint32_t)c_front[c];
    }
    keys[c] = key;
    vals[c] = (int32_t)c;
}

// 5b. ranks from the sorted order; n_clusters = number of kept clusters
__global__ void __launch_bounds__(kThreads)
db_rank_kernel(int64_t n, const uint64_t *__restrict__ keys, const int32_t *__restrict__ vals, int32_t *__restrict__ rank,
               int32_t *__restrict__ n_clusters) {
    const int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (p >= n || keys[p] == kSentinel) return;
    rank[vals[p]] = (int32_t)p;
    if (p == n - 1 || keys[p + 1] == kSentinel) *n_clusters = (int32_t)(p + 1);
}

// 6. labels (first claim) in original order + the further memberships as (point, cluster) pairs
template <typename T, int D>
__global__ void __launch_bounds__(kThreads)
db_label_kernel(const Grid *__restrict__ gp, Cloud c, const T *__restrict__ pts, const int32_t *__restrict__ comp,
                const int32_t *__restrict__ claim, const uint8_t *__restrict__ more, const int32_t *__restrict__ is_root,
                const int32_t *__restrict__ rank, int32_t *__restrict__ labels, int64_t *__restrict__ dups, int64_t dup_cap,
                unsigned long long *n_dups, int32_t *err) {
    const Grid g = *gp;
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= c.n) return;
    const int ci = comp[i];
    if (ci >= 0) {
        labels[i] = rank[ci];
        return;
    }
    const int first = claim[i];
    labels[i] = first >= 0 ? rank[first] : -1;
    if (first < 0 || !more[i]) return;
    const T *sc = static_cast<const T *>(c.sc);
    T p[3];
#pragma unroll
    for (int d = 0; d < D; ++d) p[d] = pts[i * D + d];
    ecc::rgrid::for_runs<T, D>(g, c.cell_off, p, [&](int64_t lo, int64_t hi) {
        for (int64_t j = lo; j < hi; ++j) {
            const int32_t q = c.sidx[j];
            if (!is_root[q]) continue;
            const int cq = comp[q];
            if (cq == first || rank[cq] < 0 || !(ecc::rgrid::sq_dist<T, D>(sc, c.n, j, p) <= c.eps2)) continue;
            const unsigned long long at = atomicAdd(n_dups, 1ull);
            if ((int64_t)at < dup_cap) {
                dups[2 * at] = i;
                dups[2 * at + 1] = rank[cq];
            } else {
                atomicOr(err, 2);
            }
        }
    });
}

template <typename T, int D>
int run_phases(ecc_ctx *ctx, const T *pts, const ecc::rgrid::Ws &w, Cloud c, char *p, int min_size, int max_size,
               int32_t *labels, int32_t *n_clusters, int64_t *dups, int64_t dup_cap, int64_t *n_dups, size_t sort_tmp,
               hipStream_t s) {
    const int64_t n = c.n;
    auto carve = [&](size_t bytes) { char *r = p; p += ecc::align_up(bytes, 256); return r; };
    int32_t *parent = reinterpret_cast<int32_t *>(carve((size_t)n * 4));
    int32_t *is_root = reinterpret_cast<int32_t *>(carve((size_t)n * 4));
    int64_t *cid = reinterpret_cast<int64_t *>(carve((size_t)(n + 1) * 8));
    int32_t *comp = reinterpret_cast<int32_t *>(carve((size_t)n * 4));
    int32_t *claim = reinterpret_cast<int32_t *>(carve((size_t)n * 4));
    int32_t *c_size = reinterpret_cast<int32_t *>(carve((size_t)n * 4));
    int32_t *c_front = reinterpret_cast<int32_t *>(carve((size_t)n * 4));
    int32_t *rank = reinterpret_cast<int32_t *>(carve((size_t)n * 4));
    int32_t *vals = reinterpret_cast<int32_t *>(carve((size_t)n * 4));
    int32_t *vals2 = reinterpret_cast<int32_t *>(carve((size_t)n * 4));
    uint64_t *keys = reinterpret_cast<uint64_t *>(carve((size_t)n * 8));
    uint64_t *keys2 = reinterpret_cast<uint64_t *>(carve((size_t)n * 8));
    uint8_t *core_s = reinterpret_cast<uint8_t *>(carve((size_t)n));
    uint8_t *more = reinterpret_cast<uint8_t *>(carve((size_t)n));
    void *tmp = carve(sort_tmp);
    int32_t *err = ctx->flags + kFlagWord;
    const unsigned blocks = (unsigned)((n + kThreads - 1) / kThreads);
    const Grid *g = w.grid;
    ECC_CHECK_HIP(ctx, hipMemsetAsync(c_size, 0, (size_t)n * 4, s), "memset(c_size)");
    ECC_CHECK_HIP(ctx, hipMemsetAsync(c_front, 0x7f, (size_t)n * 4, s), "memset(c_front)");
    ECC_CHECK_HIP(ctx, hipMemsetAsync(rank, 0xff, (size_t)n * 4, s), "memset(rank)");
    ECC_CHECK_HIP(ctx, hipMemsetAsync(n_clusters, 0, 4, s), "memset(n_clusters)");
    {
        ECC_TIMED(ctx, s, "dbscan_cloud_core_kernel");
        hipLaunchKernelGGL((db_core_kernel<T, D>), dim3(blocks), dim3(kThreads), 0, s, g, c, parent, core_s);
    }
    {
        ECC_TIMED(ctx, s, "dbscan_cloud_union_kernel");
        hipLaunchKernelGGL((db_union_kernel<T, D>), dim3(blocks), dim3(kThreads), 0, s, g, c, (const uint8_t *)core_s,
                           parent);
    }
    hipLaunchKernelGGL(db_roots_kernel, dim3(blocks), dim3(kThreads), 0, s, n, (const int32_t *)parent, is_root);
    int rc = ecc::exclusive_scan_i32_i64(ctx, is_root, n, cid, w.scan, s);
    if (rc) return rc;
    hipLaunchKernelGGL(db_comp_kernel, dim3(blocks), dim3(kThreads), 0, s, n, (const int32_t *)parent,
                       (const int64_t *)cid, comp, c_size, c_front);
    {
        ECC_TIMED(ctx, s, "dbscan_cloud_member_kernel");
        hipLaunchKernelGGL((db_member_kernel<T, D>), dim3(blocks), dim3(kThreads), 0, s, g, c, (const int32_t *)comp,
                           (const int32_t *)is_root, claim, more, c_size, c_front);
    }
    hipLaunchKernelGGL(db_keys_kernel, dim3(blocks), dim3(kThreads), 0, s, n, (const int64_t *)(cid + n),
                       (const int32_t *)c_size, (const int32_t *)c_front, min_size, max_size, keys, vals);
    ECC_CHECK_LAUNCH(ctx, "dbscan_cloud phases");
    rc = ecc::sort_pairs_u64_i32(ctx, tmp, sort_tmp, keys, keys2, vals, vals2, n, 62, s);
    if (rc) return rc;
    hipLaunchKernelGGL(db_rank_kernel, dim3(blocks), dim3(kThreads), 0, s, n, (const uint64_t *)keys2,
                       (const int32_t *)vals2, rank, n_clusters);
    {
        ECC_TIMED(ctx, s, "dbscan_cloud_label_kernel");
        hipLaunchKernelGGL((db_label_kernel<T, D>), dim3(blocks), dim3(kThreads), 0, s, g, c, pts, (const int32_t *)comp,
                           (const int32_t *)claim, (const uint8_t *)more, (const int32_t *)is_root, (const int32_t *)rank,
                           labels, dups, dup_cap, reinterpret_cast<unsigned long long *>(n_dups), err);
    }
    ECC_CHECK_LAUNCH(ctx, "dbscan_cloud labels");
    return ECC_OK;
}

template <typename T>
int dbscan_cloud(ecc_ctx *ctx, const T *pts, int64_t n, int32_t dim, double eps, int32_t min_pts,
                 int32_t min_cluster_size, int32_t max_cluster_size, int32_t *labels, int32_t *n_clusters, int64_t *dups,
                 int64_t dup_cap, int64_t *n_dups, ecc_stream_t stream) {
    if (!ctx || n < 0 || dim < 1 || dim > 3 || !std::isfinite(eps) || dup_cap < 0 || n >= INT32_MAX / 2)
        return ECC_ERR_INVALID;
    if (!n_clusters || !n_dups || (n > 0 && (!pts || !labels)) || (dup_cap > 0 && !dups)) return ECC_ERR_INVALID;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    ECC_CHECK_HIP(ctx, hipMemsetAsync(ctx->flags + kFlagWord, 0, 4, s), "memset(dbscan cloud err)");
    ECC_CHECK_HIP(ctx, hipMemsetAsync(n_dups, 0, 8, s), "memset(n_dups)");
    if (n == 0) {
        ECC_CHECK_HIP(ctx, hipMemsetAsync(n_clusters, 0, 4, s), "memset(n_clusters)");
        return ECC_OK;
    }
    // radius_square = radius * radius (DBSCAN_simple.h:127): a negative tolerance acts as |eps|
    const double eps2 = eps * eps, aeps = std::fabs(eps);
    const size_t sort_tmp = ecc::sort_pairs_u64_i32_temp_bytes(n, 62);
    const size_t gbytes = ecc::align_up(ecc::rgrid::ws_bytes(n, dim, sizeof(T)), 256);
    const size_t pbytes = 9 * ecc::align_up((size_t)n * 4, 256) + ecc::align_up((size_t)(n + 1) * 8, 256) +
                          2 * ecc::align_up((size_t)n * 8, 256) + 2 * ecc::align_up((size_t)n, 256) +
                          ecc::align_up(sort_tmp, 256) + 4096;
    int rc = ecc::ws_reserve(ctx, gbytes + pbytes);
    if (rc) return rc;
    char *base = static_cast<char *>(ctx->ws);
    ecc::rgrid::Ws w;
    rc = ecc::rgrid::build<T>(ctx, pts, n, dim, aeps, s, base, w);
    if (rc) return rc;
    Cloud c{w.sidx, w.cell_off, w.sc, n, eps2, min_pts};
    char *p = base + gbytes;
    switch (dim) {
        case 1: return run_phases<T, 1>(ctx, pts, w, c, p, min_cluster_size, max_cluster_size, labels, n_clusters, dups,
                                        dup_cap, n_dups, sort_tmp, s);
        case 2: return run_phases<T, 2>(ctx, pts, w, c, p, min_cluster_size, max_cluster_size, labels, n_clusters, dups,
                                        dup_cap, n_dups, sort_tmp, s);
        default: return run_phases<T, 3>(ctx, pts, w, c, p, min_cluster_size, max_cluster_size, labels, n_clusters,
                                         dups, dup_cap, n_dups, sort_tmp, s);
    }
}

}  // namespace

ECC_API int ecc_dbscan_cloud_f32(ecc_ctx *ctx, const float *pts, int64_t n, int32_t dim, double eps, int32_t min_pts,
                                 int32_t min_cluster_size, int32_t max_cluster_size, int32_t *labels,
                                 int32_t *n_clusters, int64_t *dups, int64_t dup_cap, int64_t *n_dups,
                                 ecc_stream_t stream) {
    return dbscan_cloud<float>(ctx, pts, n, dim, eps, min_pts, min_cluster_size, max_cluster_size, labels, n_clusters,
                               dups, dup_cap, n_dups, stream);
}

ECC_API int ecc_dbscan_cloud_f64(ecc_ctx *ctx, const double *pts, int64_t n, int32_t dim, double eps, int32_t min_pts,
                                 int32_t min_cluster_size, int32_t max_cluster_size, int32_t *labels,
                                 int32_t *n_clusters, int64_t *dups, int64_t dup_cap, int64_t *n_dups,
                                 ecc_stream_t stream) {
    return dbscan_cloud<double>(ctx, pts, n, dim, eps, min_pts, min_cluster_size, max_cluster_size, labels, n_clusters,
                                dups, dup_cap, n_dups, stream);
}

// Only the duplicate-capacity bit of this path's own word (a radius call in between cannot change
// it).  Non-finite points are not an error: as in the reference's radiusSearch they are nobody
// else's neighbour, so they come out as noise (label -1), or as singleton clusters when
// min_pts <= 1 (the point itself always counts), and the other clusters are unaffected.
ECC_API int ecc_dbscan_cloud_status(ecc_ctx *ctx, ecc_stream_t stream) {
    if (!ctx) return ECC_ERR_INVALID;
    int32_t f = 0;
    hipStream_t s = ecc::as_stream(stream);
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(&f, ctx->flags + kFlagWord, 4, hipMemcpyDeviceToHost, s), "read dbscan err");
    ECC_CHECK_HIP(ctx, hipStreamSynchronize(s), "sync");
    return (f & 2) ? ECC_ERR_CAPACITY : ECC_OK;
}
