// DBSCAN cluster extraction on the GPU.
//
// Reference: DBSCANSimpleCluster::extract, PCC/DBSCAN_simple.h:27-90 — a seed-queue expansion
// in point order: the first unprocessed core point i (|N_eps(i)| >= minPts, self included)
// seeds a cluster, ALL of its neighbours are queued (:43-48), and every queued core point
// queues its UN_PROCESSED neighbours (:56-64); noise flags never block a later claim.
//
// The queue's outcome has a closed form, which is what this kernel computes in parallel:
//   * a cluster = one core-connected component; clusters are created in order of their
//     smallest core index (the seed, since every core point of a component is PROCESSED by
//     the first expansion that reaches it);
//   * a non-core point b joins the first-created cluster holding one of its core neighbours
//     (b is PROCESSED after that), and also every LATER cluster whose seed is b's neighbour
//     (the seed's neighbours are queued whatever their state);
//   * core points belong to their own component only (a core neighbour of a seed is in the
//     seed's component).
// MI355X design: one workgroup (1024 lanes) per segment (<= 16384 points, one downsample
// window).  Union-find lives in LDS: a lock-free CAS union that always hooks the larger root
// under the smaller, so every root is its component's minimum (= the seed) and ascending
// roots = creation order; find() halves paths.  Component ids come from a block scan over the
// roots, and sizes / first members / the output order (size desc, first index asc, creation
// asc) from LDS atomics and an O(C^2) rank over the <= 4096 components.  Neighbour lists are
// read from HBM (ecc_eps_lists: int64 offsets + int32 segment-local indices).
#include "ecc_internal.hpp"

namespace {

constexpr int kThreads = 1024;
constexpr int kMaxPts = 16384;
constexpr int kMaxComp = 4096;
constexpr int kFlagWord = 4;  // ctx->flags[4]: bit 1 capacity

__device__ __forceinline__ int uf_find(int *parent, int x) {
    int p = parent[x];
    while (p != x) {
        const int gp = parent[p];
        if (gp != p) parent[x] = gp;  // path halving: gp is an ancestor of x
        x = p;
        p = gp;
    }
    return x;
}

// Read-only root walk for the compress phase: a halving find there could overwrite another
// lane's freshly compressed parent[j] = root with an intermediate ancestor.
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

// parent[] encoding after labelling: -1 non-core; >= 0 core (its root); <= -2 root of
// component id -(v + 2).
__device__ __forceinline__ int comp_of(const int *parent, int j) {
    const int v = parent[j];
    if (v == -1) return -1;
    return v <= -2 ? -v - 2 : -parent[v] - 2;
}

__global__ void __launch_bounds__(kThreads)
dbscan_extract_kernel(int64_t n_segs, int64_t stride, const int32_t *__restrict__ seg_counts,
                      const int64_t *__restrict__ offsets, const int32_t *__restrict__ nbr, int64_t nbr_len,
                      int min_pts, int min_size,
                      int max_size, int32_t *__restrict__ labels, int32_t *__restrict__ n_clusters,
                      int64_t *__restrict__ dups, int64_t dup_cap, unsigned long long *n_dups, int32_t *err) {
    __shared__ int parent[kMaxPts];
    __shared__ int c_size[kMaxComp], c_front[kMaxComp], c_rank[kMaxComp];
    __shared__ int wsum[kThreads / 64];
    __shared__ int s_kept;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int64_t s = blockIdx.x; s < n_segs; s += gridDim.x) {
        const int m = seg_counts ? min(seg_counts[s], (int)stride) : (int)stride;
        const int64_t base = s * stride;
        if (offsets[base] < 0 || offsets[base + m] > nbr_len) {  // lists not (fully) present
            if (threadIdx.x == 0) {
                atomicOr(err, 2);
                n_clusters[s] = 0;
            }
            for (int j = threadIdx.x; j < m; j += kThreads) labels[base + j] = -1;
            __syncthreads();
            continue;
        }
        // 1. core flags: |N_eps| >= min_pts (self included)
        for (int j = tid; j < m; j += kThreads) {
            const int64_t c = offsets[base + j + 1] - offsets[base + j];
            parent[j] = c >= min_pts ? j : -1;
        }
        __syncthreads();
        // 2. union over core-core edges (each undirected edge once: q > j)
        for (int j = tid; j < m; j += kThreads) {
            if (parent[j] == -1) continue;
            const int64_t e0 = offsets[base + j], e1 = offsets[base + j + 1];
            for (int64_t e = e0; e < e1; ++e) {
                const int q = nbr[e];
                if (q > j && parent[q] != -1) uf_union(parent, j, q);
            }
        }
        __syncthreads();
        // 3. compress; roots -> component ids in ascending root order (block scan over j)
        constexpr int kPer = kMaxPts / kThreads;  // 16 consecutive points per lane
        int roots[kPer], nr = 0;
        const int j0 = tid * kPer;
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int j = j0 + u;
            roots[u] = 0;
            if (j < m && parent[j] != -1) {
                const int r = uf_find(parent, j);
                roots[u] = r == j;
                nr += roots[u];
            }
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kPer; ++u) {  // non-roots point at their root (only root values are written)
            const int j = j0 + u;
            if (j < m && parent[j] != -1 && !roots[u]) parent[j] = uf_root(parent, j);
        }
        int x = nr;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int o = __shfl_up(x, d);
            if (lane >= d) x += o;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        int pre = 0, nc = 0;
        for (int w = 0; w < kThreads / 64; ++w) {
            if (w < wave) pre += wsum[w];
            nc += wsum[w];
        }
        int cid = pre + x - nr;
        if (nc <= kMaxComp) {
#pragma unroll
            for (int u = 0; u < kPer; ++u)
                if (roots[u]) parent[j0 + u] = -(cid++) - 2;
        }
        __syncthreads();
        if (nc > kMaxComp) {  // too many components for the LDS tables
            if (tid == 0) {
                atomicOr(err, 2);
                n_clusters[s] = 0;
            }
            for (int j = tid; j < m; j += kThreads) labels[base + j] = -1;
            __syncthreads();
            continue;
        }
        for (int c = tid; c < nc; c += kThreads) {
            c_size[c] = 0;
            c_front[c] = 0x7fffffff;
        }
        __syncthreads();
        // 4. memberships -> sizes and first members
        for (int j = tid; j < m; j += kThreads) {
            const int cj = comp_of(parent, j);
            if (cj >= 0) {
                atomicAdd(&c_size[cj], 1);
                atomicMin(&c_front[cj], j);
                continue;
            }
            const int64_t e0 = offsets[base + j], e1 = offsets[base + j + 1];
            int first = 0x7fffffff;
            for (int64_t e = e0; e < e1; ++e) {
                const int c = comp_of(parent, nbr[e]);
                if (c >= 0 && c < first) first = c;
            }
            if (first == 0x7fffffff) continue;  // noise
            atomicAdd(&c_size[first], 1);
            atomicMin(&c_front[first], j);
            for (int64_t e = e0; e < e1; ++e) {  // later clusters seeded by a neighbour
                const int v = parent[nbr[e]];
                if (v <= -2 && -v - 2 != first) {
                    atomicAdd(&c_size[-v - 2], 1);
                    atomicMin(&c_front[-v - 2], j);
                }
            }
        }
        __syncthreads();
        // 5. output order: kept clusters by (size desc, front asc, creation asc)
        if (tid == 0) s_kept = 0;
        __syncthreads();
        for (int c = tid; c < nc; c += kThreads) {
            const int sz = c_size[c], fr = c_front[c];
            int r = -1;
            if (sz >= min_size && sz <= max_size) {
                r = 0;
                for (int o = 0; o < nc; ++o) {
                    const int so = c_size[o];
                    if (so < min_size || so > max_size) continue;
                    r += so > sz || (so == sz && (c_front[o] < fr || (c_front[o] == fr && o < c)));
                }
                atomicAdd(&s_kept, 1);
            }
            c_rank[c] = r;
        }
        __syncthreads();
        if (tid == 0) n_clusters[s] = s_kept;
        // 6. labels (first claim) and further memberships
        for (int j = tid; j < m; j += kThreads) {
            const int cj = comp_of(parent, j);
            if (cj >= 0) {
                labels[base + j] = c_rank[cj];
                continue;
            }
            const int64_t e0 = offsets[base + j], e1 = offsets[base + j + 1];
            int first = 0x7fffffff;
            for (int64_t e = e0; e < e1; ++e) {
                const int c = comp_of(parent, nbr[e]);
                if (c >= 0 && c < first) first = c;
            }
            labels[base + j] = first == 0x7fffffff ? -1 : c_rank[first];
            if (first == 0x7fffffff) continue;
            for (int64_t e = e0; e < e1; ++e) {
                const int v = parent[nbr[e]];
                if (v <= -2 && -v - 2 != first && c_rank[-v - 2] >= 0) {
                    const unsigned long long at = atomicAdd(n_dups, 1ull);
                    if ((int64_t)at < dup_cap) {
                        dups[2 * at] = base + j;
                        dups[2 * at + 1] = c_rank[-v - 2];
                    } else {
                        atomicOr(err, 2);
                    }
                }
            }
        }
        __syncthreads();
    }
}

}  // namespace

ECC_API int ecc_dbscan_extract(ecc_ctx *ctx, int64_t n_segs, int64_t seg_stride, const int32_t *seg_counts,
                               const int64_t *offsets, const int32_t *nbr, int64_t nbr_len, int32_t min_pts,
                               int32_t min_cluster_size,
                               int32_t max_cluster_size, int32_t *labels, int32_t *n_clusters, int64_t *dups,
                               int64_t dup_cap, int64_t *n_dups, ecc_stream_t stream) {
    if (!ctx || n_segs < 0 || seg_stride < 1 || seg_stride > kMaxPts || min_pts < 1 || dup_cap < 0 || nbr_len < 0)
        return ECC_ERR_INVALID;
    if (n_segs > 0 && (!offsets || !nbr || !labels || !n_clusters || !n_dups || (dup_cap > 0 && !dups)))
        return ECC_ERR_INVALID;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    int32_t *err = ctx->flags + kFlagWord;
    ECC_CHECK_HIP(ctx, hipMemsetAsync(err, 0, 4, s), "memset(dbscan err)");
    if (n_dups) ECC_CHECK_HIP(ctx, hipMemsetAsync(n_dups, 0, 8, s), "memset(n_dups)");
    if (n_segs == 0) return ECC_OK;
    const unsigned grid = (unsigned)std::min<int64_t>(n_segs, 4096);
    ECC_TIMED(ctx, s, "dbscan_extract_kernel");
    hipLaunchKernelGGL(dbscan_extract_kernel, dim3(grid), dim3(kThreads), 0, s, n_segs, seg_stride, seg_counts,
                       offsets, nbr, nbr_len, min_pts, min_cluster_size, max_cluster_size, labels, n_clusters, dups, dup_cap,
                       reinterpret_cast<unsigned long long *>(n_dups), err);
    ECC_CHECK_LAUNCH(ctx, "dbscan_extract");
    return ECC_OK;
}

ECC_API int ecc_dbscan_status(ecc_ctx *ctx, ecc_stream_t stream) {
    if (!ctx) return ECC_ERR_INVALID;
    int32_t f = 0;
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(&f, ctx->flags + kFlagWord, 4, hipMemcpyDeviceToHost, ecc::as_stream(stream)),
                  "read dbscan err");
    ECC_CHECK_HIP(ctx, hipStreamSynchronize(ecc::as_stream(stream)), "sync");
    return (f & 2) ? ECC_ERR_CAPACITY : ECC_OK;
}
