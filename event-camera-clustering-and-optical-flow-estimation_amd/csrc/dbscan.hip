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
//
// ecc_dbscan_grid is the same closed form with no lists at all: the segment's points are binned
// into an LDS cell grid (eps_grid.hpp, cell > eps) and every phase that walks a neighbour list
// walks the 3x3 cells instead (exact integer eps test), so the whole DBSCAN of a segment reads
// its 4-B points once and writes its labels once (+ the duplicate memberships).
#include "eps_grid.hpp"

#include <cmath>
#include <cstdlib>

namespace {

constexpr int kThreads = 1024;
constexpr int kMaxPts = 16384;
constexpr int kMaxComp = 4096;
constexpr int kFlagWord = 4;  // ctx->flags[4]: bit 1 capacity
constexpr int kLeftWord = 11;  // ctx->flags[11]: segments dbscan_run_kernel left to dbscan_grid_kernel

bool getenv_flag(const char *name) {
    const char *v = std::getenv(name);
    return v && v[0] && v[0] != '0';
}

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

// Walks the points j = wave, wave + kW, ... of a segment, one WAVE per point: lane L of the wave
// prefetches the list range of the wave's next 64 points (no dependent offset load per point) and
// body(j, e0, e1) is called wave-uniformly; its lanes read the list e0 + lane, e0 + lane + 64, ...
// so every list read is one coalesced load per 64 entries (a lane walking its own list touched a
// different line per lane and load: ~7 ms per C4 call).
template <class F>
__device__ __forceinline__ void for_points_by_wave(int m, int64_t base, const int64_t *__restrict__ offsets,
                                                   F &&body) {
    constexpr int kW = kThreads / 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int t0 = 0; wave + kW * t0 < m; t0 += 64) {
        const int jl = wave + kW * (t0 + lane);
        const int64_t pe0 = jl < m ? offsets[base + jl] : 0, pe1 = jl < m ? offsets[base + jl + 1] : 0;
        for (int tt = 0; tt < 64; ++tt) {
            const int j = wave + kW * (t0 + tt);
            if (j >= m) break;  // wave-uniform
            body(j, ecc::lane_value64(pe0, tt), ecc::lane_value64(pe1, tt));  // readlane: tt is uniform
        }
    }
}

// A list entry of point j of an m-point segment.  An entry outside [0, m) (a malformed list:
// parent[] is sized by the stride) reads as j itself, which no phase acts on (self-unions are
// no-ops; a non-core j has no component), and sets the segment's LDS flag (bit 4 of the status
// word; an LDS store on the rare path, so no register is carried through the list walks).
__device__ __forceinline__ int nbr_at(const int32_t *__restrict__ nbr, int64_t e, int m, int j, int *bad) {
    const int q = nbr[e];
    if ((unsigned)q < (unsigned)m) return q;
    *bad = 1;
    return j;
}

// Smallest component among the core neighbours of j's list, reduced over the wave (0x7fffffff: none).
__device__ __forceinline__ int wave_first_comp(const int *parent, const int32_t *__restrict__ nbr, int64_t e0,
                                               int64_t e1, int m, int j, int *bad) {
    int first = 0x7fffffff;
    for (int64_t e = e0 + (threadIdx.x & 63); e < e1; e += 64) {
        const int c = comp_of(parent, nbr_at(nbr, e, m, j, bad));
        if (c >= 0 && c < first) first = c;
    }
    return ecc::wave_min_i32(first);  // DPP
}

__global__ void __launch_bounds__(kThreads, 8)  // 64 VGPRs: two 16-wave workgroups per CU
dbscan_extract_kernel(int64_t n_segs, int64_t stride, const int32_t *__restrict__ seg_counts,
                      const int64_t *__restrict__ offsets, const int32_t *__restrict__ nbr, int64_t nbr_len,
                      int min_pts, int min_size,
                      int max_size, int32_t *__restrict__ labels, int32_t *__restrict__ n_clusters,
                      int64_t *__restrict__ dups, int64_t dup_cap, unsigned long long *n_dups, int32_t *err) {
    // parent[] sized by the stride (dynamic), the ranks in 16 bits: 72 KB at stride 8192, so
    // two workgroups share a CU (the static 16384-entry parent[] held one per CU)
    extern __shared__ int parent[];  // [stride]
    __shared__ int c_size[kMaxComp], c_front[kMaxComp];
    __shared__ int16_t c_rank[kMaxComp];
    __shared__ int wsum[kThreads / 64];
    __shared__ int s_kept, s_bad;
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
        if (tid == 0) s_bad = 0;  // a list entry outside [0, m); read after the segment's last barrier
        // 1. core flags: |N_eps| >= min_pts (self included)
        for (int j = tid; j < m; j += kThreads) {
            const int64_t c = offsets[base + j + 1] - offsets[base + j];
            parent[j] = c >= min_pts ? j : -1;
        }
        __syncthreads();
        // 2. union over core-core edges (each undirected edge once: q > j)
        for_points_by_wave(m, base, offsets, [&](int j, int64_t e0, int64_t e1) {
            if (parent[j] == -1) return;  // non-core stays -1 during the unions: uniform
            for (int64_t e = e0 + lane; e < e1; e += 64) {
                const int q = nbr_at(nbr, e, m, j, &s_bad);
                if (q > j && parent[q] != -1) uf_union(parent, j, q);
            }
        });
        __syncthreads();
        // 3. compress; roots -> component ids in ascending root order (block scan over j)
        constexpr int kPer = kMaxPts / kThreads;  // 16 consecutive points per lane
        uint32_t roots = 0;  // bit u: point j0 + u is a root
        int nr = 0;
        const int j0 = tid * kPer;
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int j = j0 + u;
            if (j < m && parent[j] != -1 && uf_find(parent, j) == j) roots |= 1u << u;
        }
        nr = __popc(roots);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kPer; ++u) {  // non-roots point at their root (only root values are written)
            const int j = j0 + u;
            if (j < m && parent[j] != -1 && !((roots >> u) & 1u)) parent[j] = uf_root(parent, j);
        }
        const int x = ecc::wave_incl_scan(nr);  // DPP
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
                if ((roots >> u) & 1u) parent[j0 + u] = -(cid++) - 2;
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
        // 4. memberships -> sizes and first members (core points by lane, the others by wave)
        for (int j = tid; j < m; j += kThreads) {
            const int cj = comp_of(parent, j);
            if (cj >= 0) {
                atomicAdd(&c_size[cj], 1);
                atomicMin(&c_front[cj], j);
            }
        }
        for_points_by_wave(m, base, offsets, [&](int j, int64_t e0, int64_t e1) {
            if (parent[j] != -1) return;  // core: counted above (uniform)
            const int first = wave_first_comp(parent, nbr, e0, e1, m, j, &s_bad);
            if (first == 0x7fffffff) return;  // noise
            if (lane == 0) {
                atomicAdd(&c_size[first], 1);
                atomicMin(&c_front[first], j);
            }
            for (int64_t e = e0 + lane; e < e1; e += 64) {  // later clusters seeded by a neighbour
                const int v = parent[nbr_at(nbr, e, m, j, &s_bad)];
                if (v <= -2 && -v - 2 != first) {
                    atomicAdd(&c_size[-v - 2], 1);
                    atomicMin(&c_front[-v - 2], j);
                }
            }
        });
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
            c_rank[c] = (int16_t)r;
        }
        __syncthreads();
        if (tid == 0) n_clusters[s] = s_kept;
        // 6. labels (first claim) and further memberships (core points by lane, the others by wave)
        for (int j = tid; j < m; j += kThreads) {
            const int cj = comp_of(parent, j);
            if (cj >= 0) labels[base + j] = c_rank[cj];
        }
        for_points_by_wave(m, base, offsets, [&](int j, int64_t e0, int64_t e1) {
            if (parent[j] != -1) return;  // core: labelled above (uniform)
            const int first = wave_first_comp(parent, nbr, e0, e1, m, j, &s_bad);
            if (lane == 0) labels[base + j] = first == 0x7fffffff ? -1 : c_rank[first];
            if (first == 0x7fffffff) return;
            for (int64_t e = e0 + lane; e < e1; e += 64) {
                const int v = parent[nbr_at(nbr, e, m, j, &s_bad)];
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
        });
        __syncthreads();
        if (tid == 0 && s_bad) atomicOr(err, 4);
    }
}


// The segment's eps test (g.narrow is uniform per segment: a scalar select, no divergence).
__device__ __forceinline__ bool eps_in(const ecc::epsg::CellGrid &g, uint32_t v, uint32_t w, int e_int, uint32_t r2i) {
    uint32_t d2;
    return g.narrow ? ecc::epsg::in_eps<true>(v, w, e_int, r2i, &d2) : ecc::epsg::in_eps<false>(v, w, e_int, r2i, &d2);
}

#ifndef ECC_DBSCAN_PROFILE
#define ECC_DBSCAN_PROFILE 0
#endif
#if ECC_DBSCAN_PROFILE
// profiling builds (make DBSCAN_PROFILE=1): dbscan_grid_kernel's summed per-segment phase ticks
__device__ unsigned long long g_db_prof[8];
#define DB_MARK(k)                                                        \
    do {                                                                  \
        if (tid == 0) {                                                   \
            const unsigned long long now_ = wall_clock64();               \
            atomicAdd(&g_db_prof[k], now_ - db_t_);                       \
            db_t_ = now_;                                                 \
        }                                                                 \
    } while (0)
#else
#define DB_MARK(k) do { } while (0)
#endif

// ---- fused grid DBSCAN (no neighbour lists) ----------------------------------------------------
// Dynamic LDS: cend[kCells + 1] | spt[stride] | sidx[stride] | parent[stride]; ~90 KB at stride
// 8192, plus the 48 KB component tables.
constexpr int kGridMaxPts = 8192;
constexpr int kGridPer = kGridMaxPts / kThreads;  // queries per lane

__global__ void __launch_bounds__(kThreads)
dbscan_grid_kernel(const uint32_t *__restrict__ xy, int64_t n_segs, int64_t stride, const int32_t *__restrict__ seg_counts,
                   int e_int, uint32_t r2i, int min_pts, int min_size, int max_size, int32_t *__restrict__ labels,
                   int32_t *__restrict__ n_clusters, int64_t *__restrict__ dups, int64_t dup_cap,
                   unsigned long long *n_dups, int32_t *err, const int32_t *__restrict__ left) {
    // left != null: only the segments dbscan_run_kernel left (n_clusters[s] == -1)
    if (left && *left == 0) return;  // uniform
    extern __shared__ uint32_t lds_d[];
    uint32_t *cend = lds_d;
    uint32_t *spt = cend + ecc::epsg::kCells + 1;
    uint16_t *sidx = reinterpret_cast<uint16_t *>(spt + stride);
    int *parent = reinterpret_cast<int *>(sidx + ((stride + 1) & ~1ll));
    __shared__ int c_size[kMaxComp], c_front[kMaxComp], c_rank[kMaxComp];
    __shared__ int wsum[kThreads / 64];
    __shared__ int red[64];
    __shared__ int s_kept;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int64_t s = blockIdx.x; s < n_segs; s += gridDim.x) {
        if (left && n_clusters[s] != -1) continue;  // uniform: done by the row-run kernel
        int m = seg_counts ? seg_counts[s] : (int)stride;
        m = m < 0 ? 0 : (m > (int)stride ? (int)stride : m);
        const int64_t base = s * stride;
#if ECC_DBSCAN_PROFILE
        unsigned long long db_t_ = wall_clock64();
#endif
        const ecc::epsg::CellGrid g = ecc::epsg::bin_cells(xy, base, m, e_int, r2i, cend, spt, sidx, red, false, true);
        // 1. core flags: |N_eps| >= min_pts (self included)
        for (int q = tid; q < m; q += kThreads) {
            const uint32_t v = spt[q];
            int cnt = 0;
            ecc::epsg::for_candidates(g, cend, spt, v, [&](int a, uint32_t w, bool ok) {
                cnt += (eps_in(g, v, w, e_int, r2i) & ok) ? 1 : 0;
            });
            const int i = sidx[q];
            parent[i] = cnt >= min_pts ? i : -1;
        }
        __syncthreads();
        DB_MARK(0);  // bin + counts
        // 2. core connectivity by cells.  A cell pair at offset (dxc, dyc) is a CLIQUE when its
        //    farthest two points are within eps: ((|dxc|+1)cs-1)^2 + ((|dyc|+1)cs-1)^2 <= eps^2
        //    (at eps 20 the fine cells of 7 px: the cell itself and its 8 neighbours).  Then all
        //    core points of the pair are one component: every core point hangs under its cell's
        //    smallest core index (rep; a valid forest, parents < children) and clique neighbours'
        //    reps are united.  Every other cell pair the eps pattern reaches is tested point by
        //    point only while the two cells' components still differ, and one close core pair
        //    unites them (cells that are not cliques themselves — coarse grids — test every pair).  The component tables are free until phase 4: c_size holds the reps.
        int *rep = c_size;
        const int n_cells = g.gx * g.gy;
        const int cs1 = g.cs - 1;
        auto clique = [&](int dxc, int dyc) {
            const int64_t ax = (int64_t)(abs(dxc) + 1) * g.cs - 1, ay = (int64_t)(abs(dyc) + 1) * g.cs - 1;
            return ax * ax + ay * ay <= (int64_t)r2i;
        };
        const bool self_clique = 2 * (int64_t)cs1 * cs1 <= (int64_t)r2i;
        for (int c = tid; c < n_cells; c += kThreads) {
            const int lo = c == 0 ? 0 : (int)cend[c - 1], hi = (int)cend[c];
            int r = 0x7fffffff;
            for (int p = lo; p < hi; ++p) {
                const int k = sidx[p];
                r = (parent[k] != -1 && k < r) ? k : r;
            }
            rep[c] = r;
            if (self_clique && r != 0x7fffffff)
                for (int p = lo; p < hi; ++p) {
                    const int k = sidx[p];
                    if (parent[k] != -1 && k != r) parent[k] = r;
                }
        }
        __syncthreads();
        // (clique unions first, so that the point-pair tests below mostly find the two cells'
        //  components already merged)
        for (int c = tid; c < n_cells; c += kThreads) {
            const int ra = rep[c];
            if (ra == 0x7fffffff || !self_clique) continue;
            const int cx = c % g.gx, cy = c / g.gx;
#pragma unroll  // g.kx[r] stays in registers (a dynamic index would put it in scratch)
            for (int r = 0; r <= 2 * ecc::epsg::kMaxR; ++r) {
                const int dyc = r - ecc::epsg::kMaxR, kx = g.kx[r], ry = cy + dyc;
                if (kx < 0 || dyc < 0 || ry >= g.gy) continue;
                for (int dxc = -kx; dxc <= kx; ++dxc) {
                    const int rx = cx + dxc;
                    if ((dyc == 0 && dxc <= 0) || rx < 0 || rx >= g.gx || !clique(dxc, dyc)) continue;
                    const int rb = rep[ry * g.gx + rx];
                    if (rb != 0x7fffffff) uf_union(parent, ra, rb);
                }
            }
        }
        __syncthreads();
        for (int c = tid; c < n_cells; c += kThreads) {
            const int ra = rep[c];
            if (ra == 0x7fffffff) continue;
            const int cx = c % g.gx, cy = c / g.gx;
            const int alo = c == 0 ? 0 : (int)cend[c - 1], ahi = (int)cend[c];
            // point-pair test of cells [alo, ahi) x [blo, bhi) (same: only pairs p < p')
            auto pair_test = [&](int blo, int bhi, bool same) {
                for (int p = alo; p < ahi; ++p) {
                    const int i = sidx[p];
                    if (parent[i] == -1) continue;
                    const uint32_t v = spt[p];
                    for (int p2 = same ? p + 1 : blo; p2 < bhi; ++p2) {
                        const int j = sidx[p2];
                        if (parent[j] == -1 || !eps_in(g, v, spt[p2], e_int, r2i)) continue;
                        uf_union(parent, i, j);
                        if (self_clique) return;  // both cells are cliques: their components are one now
                    }
                }
            };
            if (!self_clique) pair_test(alo, ahi, true);
#pragma unroll  // g.kx[r] stays in registers (a dynamic index would put it in scratch)
            for (int r = 0; r <= 2 * ecc::epsg::kMaxR; ++r) {
                const int dyc = r - ecc::epsg::kMaxR, kx = g.kx[r], ry = cy + dyc;
                if (kx < 0 || dyc < 0 || ry >= g.gy) continue;
                for (int dxc = -kx; dxc <= kx; ++dxc) {
                    const int rx = cx + dxc;
                    if ((dyc == 0 && dxc <= 0) || rx < 0 || rx >= g.gx) continue;  // each pair once
                    const int cb = ry * g.gx + rx, rb = rep[cb];
                    if (rb == 0x7fffffff) continue;
                    if (self_clique && clique(dxc, dyc)) continue;  // united above
                    if (!self_clique || uf_find(parent, ra) != uf_find(parent, rb)) {
                        pair_test(cb == 0 ? 0 : (int)cend[cb - 1], (int)cend[cb], false);
                    }
                }
            }
        }
        __syncthreads();
        DB_MARK(1);  // unions
        // 3. compress; roots -> component ids in ascending root order (block scan over j)
        uint32_t rootm = 0u;  // bit u: j0 + u is a root
        const int j0 = tid * kGridPer;
#pragma unroll
        for (int u = 0; u < kGridPer; ++u) {
            const int j = j0 + u;
            if (j < m && parent[j] != -1 && uf_find(parent, j) == j) rootm |= 1u << u;
        }
        const int nr = __popc(rootm);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kGridPer; ++u) {
            const int j = j0 + u;
            if (j < m && parent[j] != -1 && !((rootm >> u) & 1u)) parent[j] = uf_root(parent, j);
        }
        const int x = ecc::wave_incl_scan(nr);  // DPP
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
            for (int u = 0; u < kGridPer; ++u)
                if ((rootm >> u) & 1u) parent[j0 + u] = -(cid++) - 2;
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
        DB_MARK(2);  // compress + ids
        // 4. memberships -> sizes and first members.  A non-core point's first claim (the
        //    first-created cluster with a core neighbour) and whether a LATER cluster's seed is
        //    its neighbour come from one walk over its cells; the claim stays in registers for
        //    the labels (16 bits each, two per register), the (rare) further memberships are
        //    walked again in phase 6.
        uint32_t claim2[kGridPer / 2];  // claim + 1 of query u in bits 16 (u & 1) of word u / 2
        uint32_t more = 0u;  // bit u: query u has further memberships
#pragma unroll
        for (int u = 0; u < kGridPer / 2; ++u) claim2[u] = 0u;
        auto get16 = [&](int u) { return (int)((claim2[u >> 1] >> ((u & 1) * 16)) & 0xffffu) - 1; };
        auto set16 = [&](int u, int v) {  // v >= -1
            const int sh = (u & 1) * 16;
            claim2[u >> 1] = (claim2[u >> 1] & ~(0xffffu << sh)) | (uint32_t)(v + 1) << sh;
        };
        static_assert(kMaxComp < 0xffff, "claims in 16 bits");
#pragma unroll
        for (int u = 0; u < kGridPer; ++u) {
            const int q = u * kThreads + tid;
            if (q >= m) continue;
            const int i = sidx[q];
            const int ci = comp_of(parent, i);
            if (ci >= 0) {
                set16(u, ci);
                atomicAdd(&c_size[ci], 1);
                atomicMin(&c_front[ci], i);
                continue;
            }
            const uint32_t v = spt[q];
            int first = 0x7fffffff, n_seed = 0, seed_c = -1;
            ecc::epsg::for_candidates(g, cend, spt, v, [&](int a, uint32_t w, bool ok) {
                if (!(eps_in(g, v, w, e_int, r2i) & ok)) return;
                const int pv = parent[sidx[a]];
                if (pv == -1) return;
                const int c = pv <= -2 ? -pv - 2 : -parent[pv] - 2;
                first = c < first ? c : first;
                n_seed += pv <= -2 ? 1 : 0;
                seed_c = pv <= -2 ? c : seed_c;
            });
            if (first == 0x7fffffff) continue;  // noise
            set16(u, first);
            atomicAdd(&c_size[first], 1);
            atomicMin(&c_front[first], i);
            if (n_seed == 0 || (n_seed == 1 && seed_c == first)) continue;
            more |= 1u << u;
            ecc::epsg::for_candidates(g, cend, spt, v, [&](int a, uint32_t w, bool ok) {  // later clusters seeded by a neighbour
                if (!(eps_in(g, v, w, e_int, r2i) & ok)) return;
                const int pv = parent[sidx[a]];
                if (pv <= -2 && -pv - 2 != first) {
                    atomicAdd(&c_size[-pv - 2], 1);
                    atomicMin(&c_front[-pv - 2], i);
                }
            });
        }
        __syncthreads();
        DB_MARK(3);  // memberships
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
        DB_MARK(4);  // ranks
        // 6. labels (the first claim, staged over parent[] by segment index for a coalesced
        //    write; the label replaces the claim in its register half) and the further memberships
#pragma unroll
        for (int u = 0; u < kGridPer; ++u) {
            const int q = u * kThreads + tid;
            if (q >= m) break;
            const int first = get16(u);
            set16(u, first >= 0 ? c_rank[first] : -1);
            if (!((more >> u) & 1u)) continue;
            const int i = sidx[q];
            const uint32_t v = spt[q];
            ecc::epsg::for_candidates(g, cend, spt, v, [&](int a, uint32_t w, bool ok) {
                if (!(eps_in(g, v, w, e_int, r2i) & ok)) return;
                const int pv = parent[sidx[a]];
                if (pv <= -2 && -pv - 2 != first && c_rank[-pv - 2] >= 0) {
                    const unsigned long long at = atomicAdd(n_dups, 1ull);
                    if ((int64_t)at < dup_cap) {
                        dups[2 * at] = base + i;
                        dups[2 * at + 1] = c_rank[-pv - 2];
                    } else {
                        atomicOr(err, 2);
                    }
                }
            });
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kGridPer; ++u) {
            const int q = u * kThreads + tid;
            if (q < m) parent[sidx[q]] = get16(u);
        }
        __syncthreads();
        for (int j = tid; j < m; j += kThreads) labels[base + j] = parent[j];
        __syncthreads();
        DB_MARK(5);  // labels + dups
#if ECC_DBSCAN_PROFILE
        if (tid == 0) atomicAdd(&g_db_prof[7], 1ull);
#endif
    }
}

// ---- row-run DBSCAN (distinct-pixel segments: downsample windows) -------------------------------
// A downsample window's representatives are distinct pixels, so the segment is an occupancy
// bitmap over its bounding box (eps.hip's row-run form): word w of row y holds 32 pixels and the
// number of points in the words before it, so a pixel's raster rank is one word read + popc (the
// point's id in the union-find below).  A second bitmap marks the core points.
//   counts:  the disk's rows as prefix differences (eps_run_counts_kernel's count, self included);
//   unions:  the core points within eps of core point p in a row are a chord [x - w, x + w] of
//            that row.  Consecutive core points of one row within eps of each other (gap <= e)
//            are united left to right (a chain); a chord is at most 2e + 1 wide, so its core
//            points lie in at most two chains — the one holding its leftmost core point and the
//            one holding its rightmost.  Uniting p with those two (rows below p only: the pair is
//            symmetric, and the chord of q in p's row holds p) makes p core-connected to every
//            core point within eps, with no distance test and no candidate walk;
//   members: a non-core point walks the core bits of its disk's chords (fewer than min_pts);
// the rest (component ids in seed order, sizes, output order, labels, duplicate memberships) is
// dbscan_grid_kernel's closed form.  Segments that repeat a pixel, whose bitmap exceeds kDrWords,
// with more than kDrComp components or with eps >= kDrHw are marked (n_clusters[s] = -1, counted in *left) for dbscan_grid_kernel.
constexpr int kDrWords = 2880;  // (bits, prefix) pairs: 346x260 needs 2860 (LDS < 80 KiB in all)
constexpr int kDrHw = 512;      // disk half-width table: eps < 512
constexpr int kDrPer = kGridMaxPts / kThreads;
constexpr int kDrNarrow = 32;  // eps up to which a chord (2 eps + 1 pixels) spans at most 3 words
// A lane index the compiler cannot hoist or reuse across the kernel's phases: values derived
// from it are born in the phase that uses them (hoisted to the top and kept, they were spilled to
// scratch around the unions: one scratch round trip per value and segment).
__device__ __forceinline__ int opaque_lane(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

#ifndef ECC_DR_ROWS
#define ECC_DR_ROWS 4
#endif
constexpr int kDrRows = ECC_DR_ROWS;  // chord rows per union batch
constexpr int kDrComp = 1024;  // components per segment (more: dbscan_grid_kernel takes the segment)
constexpr int kDrJWords = kGridMaxPts / 32;  // one bit per segment index

// The union-find lives in raster-rank space (parent[rank]: a chord's core bit is its own id, no
// rank -> index table), and the roots (the smallest rank of each component) are renumbered in
// the seed order dbscan_grid_kernel uses — ascending smallest core index — through a bitmap over
// the segment's indices.  LDS < 80 KiB and 64 VGPRs: two 16-wave workgroups per CU.
__global__ void __launch_bounds__(kThreads, 8)
dbscan_run_kernel(const uint32_t *__restrict__ xy, int64_t n_segs, int64_t stride, const int32_t *__restrict__ seg_counts,
                  int e_int, uint32_t r2i, int min_pts, int min_size, int max_size, int32_t *__restrict__ labels,
                  int32_t *__restrict__ n_clusters, int64_t *__restrict__ dups, int64_t dup_cap,
                  unsigned long long *n_dups, int32_t *err, int32_t *left) {
    __shared__ uint2 wd[kDrWords + 1];     // occupancy bits | points before the word; [kDrWords] = 0
    __shared__ uint32_t cw[kDrWords + 1];  // core bits
    __shared__ int parent[kGridMaxPts];  // by raster rank: -1 non-core, >= 0 core (a parent), <= -2 root
    __shared__ int c_size[kDrComp], c_front[kDrComp];
    __shared__ int16_t c_rank[kDrComp];
    __shared__ uint16_t hwt[kDrHw];
    __shared__ uint32_t jb[kDrJWords];    // bit j: index j is the first core point of its component
    __shared__ uint32_t sb[kDrJWords];    // the same points by rank
    __shared__ uint16_t jpre[kDrJWords];  // set bits of jb before word w
    __shared__ int box[kThreads / 64][4];
    __shared__ int wsum[kThreads / 64];
    __shared__ int s_dup, s_kept, s_nc, s_nl;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int kW = kThreads / 64;
    if (tid == 0) {
        wd[kDrWords] = make_uint2(0u, 0u);
        cw[kDrWords] = 0u;
    }
    for (int a = tid; a < kDrHw && a <= e_int; a += kThreads) {  // exact integer square roots
        const uint32_t v = r2i - (uint32_t)(a * a);
        uint32_t h = (uint32_t)sqrtf((float)v);
        while (h * h > v) --h;
        while ((h + 1) * (h + 1) <= v) ++h;
        hwt[a] = (uint16_t)h;
    }
    for (int64_t s = blockIdx.x; s < n_segs; s += gridDim.x) {
        int m = seg_counts ? seg_counts[s] : (int)stride;
        m = m < 0 ? 0 : (m > (int)stride ? (int)stride : m);
        const int64_t base = s * stride;
#if ECC_DBSCAN_PROFILE
        unsigned long long db_t_ = wall_clock64();
#endif
        // points: lane tid holds j = u * kThreads + tid
        uint32_t v[kDrPer];
        int xmn = 0x7fffffff, ymn = 0x7fffffff, xmx = -1, ymx = -1;
#pragma unroll
        for (int u = 0; u < kDrPer; ++u) {
            const int j = u * kThreads + tid;
            v[u] = j < m ? xy[base + j] : 0u;
            if (j < m) {
                xmn = min(xmn, ecc::xy_x(v[u])); ymn = min(ymn, ecc::xy_y(v[u]));
                xmx = max(xmx, ecc::xy_x(v[u])); ymx = max(ymx, ecc::xy_y(v[u]));
            }
        }
        xmn = ecc::wave_min_i32(xmn); ymn = ecc::wave_min_i32(ymn);  // DPP
        xmx = ecc::wave_max_i32(xmx); ymx = ecc::wave_max_i32(ymx);
        if (lane == 0) {
            box[wave][0] = xmn; box[wave][1] = ymn;
            box[wave][2] = xmx; box[wave][3] = ymx;
        }
        if (tid == 0) s_dup = 0;
        __syncthreads();
        xmn = box[0][0]; ymn = box[0][1]; xmx = box[0][2]; ymx = box[0][3];
#pragma unroll
        for (int w = 1; w < kW; ++w) {
            xmn = min(xmn, box[w][0]); ymn = min(ymn, box[w][1]);
            xmx = max(xmx, box[w][2]); ymx = max(ymx, box[w][3]);
        }
        const int Wb = m ? xmx - xmn + 1 : 1, H = m ? ymx - ymn + 1 : 1;
        const int WW = (Wb >> 5) + 1;
        const int64_t words64 = (int64_t)H * WW;
        bool leftover = words64 > kDrWords || e_int >= kDrHw;  // uniform
        const int words = leftover ? 0 : (int)words64;
        for (int w = opaque_lane(tid); w < words; w += kThreads) {
            wd[w] = make_uint2(0u, 0u);
            cw[w] = 0u;
        }
        for (int w = opaque_lane(tid); w < kDrJWords; w += kThreads) jb[w] = sb[w] = 0u;
        __syncthreads();
        if (!leftover) {
#pragma unroll
            for (int u = 0; u < kDrPer; ++u) {
                if (u * kThreads + tid >= m) break;
                const int x = ecc::xy_x(v[u]) - xmn, y = ecc::xy_y(v[u]) - ymn;
                const uint32_t bit = 1u << (x & 31);
                if (atomicOr(&wd[y * WW + (x >> 5)].x, bit) & bit) s_dup = 1;
            }
        }
        __syncthreads();
        leftover = leftover || s_dup;  // uniform
        if (leftover) {
            if (tid == 0 && m > 0) {
                n_clusters[s] = -1;
                atomicAdd(left, 1);
            }
            __syncthreads();
            continue;
        }
        {  // points before each word (thread t: words [t * per, t * per + per))
            const int per = (words + kThreads - 1) / kThreads;
            const int w0 = opaque_lane(tid) * per, w1 = min(w0 + per, words);
            int loc = 0;
            for (int w = w0; w < w1; ++w) loc += __popc(wd[w].x);
            const int inc = ecc::wave_incl_scan(loc);
            if (lane == 63) wsum[opaque_lane(wave)] = inc;
            __syncthreads();
            int off = inc - loc;
            for (int w = 0; w < opaque_lane(wave); ++w) off += wsum[w];
            for (int w = w0; w < w1; ++w) {
                wd[w].y = (uint32_t)off;
                off += __popc(wd[w].x);
            }
        }
        __syncthreads();
        // raster rank of the pixel at (x, y) of the box (a set bit)
        auto rank_at = [&](int x, int y) -> int {
            const uint2 q = wd[y * WW + (x >> 5)];
            return (int)q.y + __popc(q.x & ((1u << (x & 31)) - 1u));
        };
        const int amax = min(e_int, H - 1);
        // the point of lane tid's slot u, re-read (an L2 hit) in the phases after the counts: its
        // register copy would not fit the 64 VGPRs beside the union batches
        auto pt = [&](int u) -> uint32_t {
            return __hip_atomic_load(xy + base + u * kThreads + opaque_lane(tid), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        };
        // counts -> core flags and bits
#pragma unroll
        for (int u = 0; u < kDrPer; ++u) {
            const int j = u * kThreads + opaque_lane(tid);
            if (j >= m) break;
            const int x = ecc::xy_x(v[u]) - xmn, y = ecc::xy_y(v[u]) - ymn;
            int cnt = 0;
#pragma unroll 4
            for (int a = 0; a <= amax; ++a) {  // (unrolled: four rows' word loads in flight)
                const int hw = hwt[a];
                const int xl = max(x - hw, 0), xh = min(x + hw + 1, Wb);
                const uint32_t ml = (1u << (xl & 31)) - 1u, mh = (1u << (xh & 31)) - 1u;
                const int cl = xl >> 5, ch = xh >> 5;
#pragma unroll
                for (int sgn = 0; sgn < 2; ++sgn) {
                    if (sgn && a == 0) break;
                    const int yy = sgn ? y - a : y + a;
                    const bool ok = (unsigned)yy < (unsigned)H;
                    const int rb = yy * WW;
                    const uint2 lo = wd[ok ? rb + cl : kDrWords], hi = wd[ok ? rb + ch : kDrWords];
                    cnt += (int)(hi.y - lo.y) + __popc(hi.x & mh) - __popc(lo.x & ml);
                }
            }
            const bool core = cnt >= min_pts;
            const int r = rank_at(x, y);
            parent[r] = core ? r : -1;
            if (core) atomicOr(&cw[y * WW + (x >> 5)], 1u << (x & 31));
        }
        __syncthreads();
        DB_MARK(0);  // bitmap + counts
        // lowest / highest core bit of row yy in columns [lo, hi] (-1: none)
        auto first_core = [&](int rb, int lo, int hi) -> int {
            for (int w = lo >> 5; w <= (hi >> 5); ++w) {
                uint32_t b = cw[rb + w];
                if (w == (lo >> 5)) b &= ~((1u << (lo & 31)) - 1u);
                if (w == (hi >> 5)) b &= (hi & 31) == 31 ? 0xffffffffu : ((2u << (hi & 31)) - 1u);
                if (b) return (w << 5) + __ffs(b) - 1;
            }
            return -1;
        };
        auto last_core = [&](int rb, int lo, int hi) -> int {
            for (int w = hi >> 5; w >= (lo >> 5); --w) {
                uint32_t b = cw[rb + w];
                if (w == (lo >> 5)) b &= ~((1u << (lo & 31)) - 1u);
                if (w == (hi >> 5)) b &= (hi & 31) == 31 ? 0xffffffffu : ((2u << (hi & 31)) - 1u);
                if (b) return (w << 5) + 31 - __clz(b);
            }
            return -1;
        };
        // Rows y + a0 .. y + a0 + kDrRows - 1: per row, the ranks of the first and last core point
        // of the point's chord there (eps <= kDrNarrow: a chord spans at most 3 words), -1 if none
        // or the same point.  A row past amax or the box reads the zero word cw[kDrWords]: -1.
        auto chord_ends_batch = [&](int a0, int x, int y, int (&cand)[2 * kDrRows]) {
            uint32_t b[kDrRows][3], lh[kDrRows];  // lh: lo | hi << 16
#pragma unroll
            for (int r = 0; r < kDrRows; ++r) {
                const int a = a0 + r, yy = y + a;
                const bool ok = a <= amax && yy < H;
                const int hw = hwt[ok ? a : 0];
                const int lo = max(x - hw, 0), hi = min(x + hw, Wb - 1);
                lh[r] = (uint32_t)lo | (uint32_t)hi << 16;
                const int w0 = lo >> 5, w1 = hi >> 5, rb = yy * WW;
                b[r][0] = cw[ok ? rb + w0 : kDrWords];
                b[r][1] = cw[ok && w1 > w0 ? rb + w0 + 1 : kDrWords];
                b[r][2] = cw[ok && w1 > w0 + 1 ? rb + w0 + 2 : kDrWords];
            }
#pragma unroll
            for (int r = 0; r < kDrRows; ++r) {
                const int lo = (int)(lh[r] & 0xffffu), hi = (int)(lh[r] >> 16);
                const int w0 = lo >> 5, nw = (hi >> 5) - w0;  // last word: 0..2
                const uint32_t hm = (hi & 31) == 31 ? 0xffffffffu : ((2u << (hi & 31)) - 1u);
                uint32_t b0 = b[r][0] & ~((1u << (lo & 31)) - 1u), b1 = b[r][1], b2 = b[r][2];
                if (nw == 0) b0 &= hm;
                else if (nw == 1) b1 &= hm;
                else b2 &= hm;
                const uint64_t lw = (uint64_t)b0 | ((uint64_t)b1 << 32);
                const int base = w0 << 5;
                const int cl = lw ? base + __builtin_ctzll(lw) : (b2 ? base + 64 + __builtin_ctz(b2) : -1);
                const int cr = b2 ? base + 95 - __builtin_clz(b2) : (lw ? base + 63 - __builtin_clzll(lw) : -1);
                cand[2 * r] = cl >= 0 ? rank_at(cl, y + a0 + r) : -1;
                cand[2 * r + 1] = cr > cl ? rank_at(cr, y + a0 + r) : -1;
            }
        };
        // rt[] -> the roots of rt[] (-1 stays -1), the chains walked in lockstep
        auto roots_batch = [&](int (&rt)[2 * kDrRows]) {
            for (;;) {
                int nxt[2 * kDrRows];
                bool more = false;
#pragma unroll
                for (int k = 0; k < 2 * kDrRows; ++k) nxt[k] = rt[k] >= 0 ? parent[rt[k]] : -1;
#pragma unroll
                for (int k = 0; k < 2 * kDrRows; ++k) {
                    more |= rt[k] >= 0 && nxt[k] != rt[k];
                    rt[k] = rt[k] >= 0 ? nxt[k] : -1;
                }
                if (!more) break;
            }
        };
        // unions: the row chain link to the right, then the two chains of every chord below.  The
        // point's own root is found once and carried (ra): a root that another lane hooks
        // meanwhile still lies in the component, and the hook itself only ever moves a root
        // that is still a root (the CAS), so a stale ra costs at most a retry of the full union.
        // Chords of at most 3 words (eps <= kDrNarrow) go kDrRows rows at a time: their core
        // words, ranks, indices and roots are loaded for all rows of the batch together (one
        // dependent LDS round trip per step instead of one per row and step).
#pragma unroll 1
        for (int u = 0; u < kDrPer; ++u) {
            if (u * kThreads + opaque_lane(tid) >= m) break;
            const int x = ecc::xy_x(pt(u)) - xmn, y = ecc::xy_y(pt(u)) - ymn;
            const int j = rank_at(x, y);  // the point's id in the union-find
            if (parent[j] == -1) continue;
            int ra = uf_find(parent, j);
            auto unite_root = [&](int q, int rb) {  // rb: q's root when looked up (may be stale)
                if (rb == ra) return;
                if (rb > ra) {
                    if (atomicCAS(&parent[rb], rb, ra) == rb) return;  // rb hooked under ra
                } else if (atomicCAS(&parent[ra], ra, rb) == ra) {
                    ra = rb;  // ra hooked under rb: rb is the root now
                    return;
                }
                uf_union(parent, j, q);  // lost a race: the general loop
                ra = uf_find(parent, j);
            };
            if (x + 1 < Wb && e_int > 0) {
                const int c = first_core(y * WW, x + 1, min(x + e_int, Wb - 1));
                if (c >= 0) {
                    const int q = rank_at(c, y);
                    unite_root(q, uf_find(parent, q));
                }
            }
            if (e_int <= kDrNarrow) {  // uniform
                for (int a0 = 1; a0 <= amax && y + a0 < H; a0 += kDrRows) {
                    int rt[2 * kDrRows];
                    chord_ends_batch(a0, x, y, rt);
                    roots_batch(rt);
#pragma unroll
                    for (int k = 0; k < 2 * kDrRows; ++k)  // a root stands for its chord point
                        if (rt[k] >= 0) unite_root(rt[k], rt[k]);
                }
            } else {
                for (int a = 1; a <= amax && y + a < H; ++a) {
                    const int hw = hwt[a];
                    const int lo = max(x - hw, 0), hi = min(x + hw, Wb - 1);
                    const int rb = (y + a) * WW;
                    const int cl = first_core(rb, lo, hi);
                    if (cl < 0) continue;
                    int q = rank_at(cl, y + a);
                    unite_root(q, uf_find(parent, q));
                    const int cr = last_core(rb, cl, hi);
                    if (cr > cl) {
                        q = rank_at(cr, y + a);
                        unite_root(q, uf_find(parent, q));
                    }
                }
            }
        }
        __syncthreads();
        DB_MARK(1);  // unions
        // compress (ranks r0 .. r0 + 7 per lane); each root then keeps the smallest index of its
        // component's core points (the seed), and the seeds' order gives the component ids
        uint32_t rootm = 0u;
        const int r0 = opaque_lane(tid) * kGridPer;
#pragma unroll
        for (int u = 0; u < kGridPer; ++u) {
            const int r = r0 + u;
            if (r < m && parent[r] != -1 && uf_find(parent, r) == r) rootm |= 1u << u;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kGridPer; ++u) {
            const int r = r0 + u;
            if (r < m && parent[r] != -1 && !((rootm >> u) & 1u)) parent[r] = uf_root(parent, r);
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kGridPer; ++u)
            if ((rootm >> u) & 1u) parent[r0 + u] = -2 - kGridMaxPts;  // no index yet
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kDrPer; ++u) {
            const int j = u * kThreads + opaque_lane(tid);
            if (j >= m) break;
            const int r = rank_at(ecc::xy_x(pt(u)) - xmn, ecc::xy_y(pt(u)) - ymn);
            const int pr = parent[r];
            if (pr != -1) atomicMax(&parent[pr >= 0 ? pr : r], -2 - j);  // -2 - j: larger = earlier
        }
        __syncthreads();
        // the seeds: index j in jb, rank in sb (the memberships' "neighbour is a seed" test)
#pragma unroll
        for (int u = 0; u < kDrPer; ++u) {
            const int j = u * kThreads + opaque_lane(tid);
            if (j >= m) break;
            const int r = rank_at(ecc::xy_x(pt(u)) - xmn, ecc::xy_y(pt(u)) - ymn);
            const int pr = parent[r];
            if (pr == -1 || -2 - parent[pr >= 0 ? pr : r] != j) continue;
            atomicOr(&jb[j >> 5], 1u << (j & 31));
            atomicOr(&sb[r >> 5], 1u << (r & 31));
        }
        __syncthreads();
        if (wave == 0) {  // seeds before each word of jb
            static_assert(kDrJWords == 4 * 64, "four jb words per lane");
            int c4[4], loc = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) loc += (c4[k] = __popc(jb[4 * opaque_lane(lane) + k]));
            const int inc = ecc::wave_incl_scan(loc);
            int off = inc - loc;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                jpre[4 * lane + k] = (uint16_t)off;
                off += c4[k];
            }
            if (lane == 63) s_nc = inc;
        }
        __syncthreads();
        const int nc = s_nc;
        if (nc > kDrComp) {  // uniform: too many components for the tables, the grid kernel redoes it
            if (tid == 0) {
                n_clusters[s] = -1;
                atomicAdd(left, 1);
            }
            __syncthreads();
            continue;
        }
#pragma unroll
        for (int u = 0; u < kGridPer; ++u) {
            if (!((rootm >> u) & 1u)) continue;
            const int j = -2 - parent[r0 + u];
            const int id = jpre[j >> 5] + __popc(jb[j >> 5] & ((1u << (j & 31)) - 1u));
            parent[r0 + u] = -id - 2;
        }
        for (int c = opaque_lane(tid); c < nc; c += kThreads) {
            c_size[c] = 0;
            c_front[c] = 0x7fffffff;
        }
        __syncthreads();
        DB_MARK(2);  // compress + ids
        // the core neighbours of a non-core point: f(q) for the index q of every core bit of the
        // chords of its disk (all rows: the relation is walked from the non-core side only)
        auto for_core_nbrs = [&](int x, int y, auto &&f) {
            for (int a = -amax; a <= amax; ++a) {
                const int yy = y + a;
                if ((unsigned)yy >= (unsigned)H) continue;
                const int hw = hwt[a < 0 ? -a : a];
                const int lo = max(x - hw, 0), hi = min(x + hw, Wb - 1);
                const int rb = yy * WW;
                for (int w = lo >> 5; w <= (hi >> 5); ++w) {
                    uint32_t b = cw[rb + w];
                    if (w == (lo >> 5)) b &= ~((1u << (lo & 31)) - 1u);
                    if (w == (hi >> 5)) b &= (hi & 31) == 31 ? 0xffffffffu : ((2u << (hi & 31)) - 1u);
                    if (!b) continue;
                    const uint2 q = wd[rb + w];
                    while (b) {
                        const int bit = __ffs(b) - 1;
                        b &= b - 1u;
                        f((int)q.y + __popc(q.x & ((1u << bit) - 1u)));  // the core point's rank
                    }
                }
            }
        };
        // memberships -> sizes and first members (first claim + later seeds, as the grid kernel).
        // Core points by their lane; the non-core points' disk walks are first listed workgroup-
        // wide (c_rank's 1 024 slots, unused until the ranks) and then walked one per lane, so a
        // wave does about one walk instead of one per slot u.  A walked point's claim goes to
        // labels[] (first | more << 16, -1 noise) until the labels pass translates it.
        uint32_t ncm = 0u;  // bit u: slot u holds a non-core point
#pragma unroll
        for (int u = 0; u < kDrPer; ++u) {
            const int j = u * kThreads + opaque_lane(tid);
            if (j >= m) continue;
            const int cj = comp_of(parent, rank_at(ecc::xy_x(pt(u)) - xmn, ecc::xy_y(pt(u)) - ymn));
            if (cj >= 0) {
                atomicAdd(&c_size[cj], 1);
                atomicMin(&c_front[cj], j);
            } else {
                ncm |= 1u << u;
            }
        }
        uint16_t *const walk = reinterpret_cast<uint16_t *>(c_rank);  // [kDrComp] non-core indices
        const uint32_t ncm0 = ncm;
        for (;;) {
            if (tid == 0) s_nl = 0;
            __syncthreads();
#pragma unroll
            for (int u = 0; u < kDrPer; ++u) {  // append (wave-aggregated), while there is room
                const bool nc_u = (ncm >> u) & 1u;
                const uint64_t bal = __ballot(nc_u);
                if (!bal) continue;  // uniform
                const int leader = __ffsll((unsigned long long)bal) - 1;
                int b = 0;
                if (lane == leader) b = atomicAdd(&s_nl, __popcll(bal));
                b = __shfl(b, leader);
                const int pos = b + __popcll(bal & ((1ull << opaque_lane(lane)) - 1ull));
                if (nc_u && pos < kDrComp) {
                    walk[pos] = (uint16_t)(u * kThreads + opaque_lane(tid));
                    ncm &= ~(1u << u);
                }
            }
            __syncthreads();
            const int n_walk = min(s_nl, kDrComp);
            if (tid < n_walk) {
                const int j = walk[opaque_lane(tid)];
                const uint32_t p = xy[base + j];
                const int x = ecc::xy_x(p) - xmn, y = ecc::xy_y(p) - ymn;
                int first = 0x7fffffff, n_seed = 0, seed_c = -1;
                for_core_nbrs(x, y, [&](int q) {
                    const int pv = parent[q];
                    const int c = pv <= -2 ? -pv - 2 : -parent[pv] - 2;
                    const bool seed = (sb[q >> 5] >> (q & 31)) & 1u;
                    first = c < first ? c : first;
                    n_seed += seed ? 1 : 0;
                    seed_c = seed ? c : seed_c;
                });
                int claim = -1;
                if (first != 0x7fffffff) {  // else noise
                    atomicAdd(&c_size[first], 1);
                    atomicMin(&c_front[first], j);
                    const bool more = !(n_seed == 0 || (n_seed == 1 && seed_c == first));
                    claim = first | (more ? 1 << 16 : 0);
                    if (more) {
                        for_core_nbrs(x, y, [&](int q) {  // later clusters seeded by a neighbour
                            if (!((sb[q >> 5] >> (q & 31)) & 1u)) return;
                            const int pv = parent[q];
                            const int c = pv <= -2 ? -pv - 2 : -parent[pv] - 2;
                            if (c != first) {
                                atomicAdd(&c_size[c], 1);
                                atomicMin(&c_front[c], j);
                            }
                        });
                    }
                }
                labels[base + j] = claim;
            }
            if (!__syncthreads_or(ncm != 0u)) break;  // also: the list is read before the next appends
        }
        __syncthreads();
        DB_MARK(3);  // memberships
        // output order: kept clusters by (size desc, front asc, creation asc)
        if (tid == 0) s_kept = 0;
        __syncthreads();
        for (int c = opaque_lane(tid); c < nc; c += kThreads) {
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
            c_rank[c] = (int16_t)r;
        }
        __syncthreads();
        if (tid == 0) n_clusters[s] = s_kept;
        DB_MARK(4);  // ranks
        // labels (first claim, coalesced: lane tid holds j = u * kThreads + tid) and the further
        // memberships; a non-core point's claim is read back from labels[] (written by the lane
        // that walked it, before the barriers since)
#pragma unroll
        for (int u = 0; u < kDrPer; ++u) {
            const int j = u * kThreads + opaque_lane(tid);
            if (j >= m) break;
            const int x = ecc::xy_x(pt(u)) - xmn, y = ecc::xy_y(pt(u)) - ymn;
            if (!((ncm0 >> u) & 1u)) {
                labels[base + j] = c_rank[comp_of(parent, rank_at(x, y))];
                continue;
            }
            const int claim = __hip_atomic_load(labels + base + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (claim < 0) continue;  // noise: -1 already
            const int first = claim & 0xffff;
            labels[base + j] = c_rank[first];
            if (!(claim >> 16)) continue;
            for_core_nbrs(x, y, [&](int q) {
                if (!((sb[q >> 5] >> (q & 31)) & 1u)) return;
                const int pv = parent[q];
                const int c = pv <= -2 ? -pv - 2 : -parent[pv] - 2;
                if (c != first && c_rank[c] >= 0) {
                    const unsigned long long at = atomicAdd(n_dups, 1ull);
                    if ((int64_t)at < dup_cap) {
                        dups[2 * at] = base + j;
                        dups[2 * at + 1] = c_rank[c];
                    } else {
                        atomicOr(err, 2);
                    }
                }
            });
        }
        __syncthreads();
        DB_MARK(5);  // labels + dups
#if ECC_DBSCAN_PROFILE
        if (tid == 0) atomicAdd(&g_db_prof[7], 1ull);
#endif
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
    // parent[] (dynamic): seg_stride <= kMaxPts = 16384 entries, at most 64 KiB, with the static
    // tables inside gfx950's 160 KiB
    const size_t lds = (size_t)seg_stride * sizeof(int);
    static_assert(kMaxPts * sizeof(int) <= 65536, "dynamic LDS of dbscan_extract_kernel");
    ECC_TIMED(ctx, s, "dbscan_extract_kernel");
    hipLaunchKernelGGL(dbscan_extract_kernel, dim3(grid), dim3(kThreads), lds, s, n_segs, seg_stride, seg_counts,
                       offsets, nbr, nbr_len, min_pts, min_cluster_size, max_cluster_size, labels, n_clusters, dups, dup_cap,
                       reinterpret_cast<unsigned long long *>(n_dups), err);
    ECC_CHECK_LAUNCH(ctx, "dbscan_extract");
    return ECC_OK;
}

ECC_API int ecc_dbscan_grid(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                            const int32_t *seg_counts, double eps, int32_t min_pts, int32_t min_cluster_size,
                            int32_t max_cluster_size, int32_t *labels, int32_t *n_clusters, int64_t *dups,
                            int64_t dup_cap, int64_t *n_dups, ecc_stream_t stream) {
    if (!ctx || n_segs < 0 || seg_stride < 1 || seg_stride > kGridMaxPts || min_pts < 1 || dup_cap < 0 ||
        !(eps >= 0.0) || eps > 32767.0)
        return ECC_ERR_INVALID;
    if (n_segs > 0 && (!xy || !labels || !n_clusters || !n_dups || (dup_cap > 0 && !dups))) return ECC_ERR_INVALID;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    int32_t *err = ctx->flags + kFlagWord;
    ECC_CHECK_HIP(ctx, hipMemsetAsync(err, 0, 4, s), "memset(dbscan err)");
    ECC_CHECK_HIP(ctx, hipMemsetAsync(n_dups, 0, 8, s), "memset(n_dups)");
    if (n_segs == 0) return ECC_OK;
    // d^2 <= eps^2 (fp64) <=> d^2 <= floor(eps^2) for integer d^2; |dx|, |dy| <= floor(eps)
    const int r2i = (int)std::floor(eps * eps), e_int = (int)std::floor(eps);
    const size_t lds = (size_t)(ecc::epsg::kCells + 1 + seg_stride) * 4 + (size_t)((seg_stride + 1) & ~1ll) * 2 +
                       (size_t)seg_stride * 4;
    ECC_CHECK_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void *>(dbscan_grid_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                  "dbscan_grid lds");
    // the row-run kernel first (distinct-pixel segments whose bitmap fits its LDS); the grid kernel
    // takes what it leaves, and exits at once when it leaves nothing
    const bool run = e_int < kDrHw && !getenv_flag("ECC_DBSCAN_GRID_ONLY");
    int32_t *left = ctx->flags + kLeftWord;
    if (run) {
        ECC_CHECK_HIP(ctx, hipMemsetAsync(left, 0, 4, s), "memset(dbscan leftovers)");
        ECC_TIMED(ctx, s, "dbscan_run_kernel");
        const unsigned grid = (unsigned)std::min<int64_t>(n_segs, 1 << 20);
        hipLaunchKernelGGL(dbscan_run_kernel, dim3(grid), dim3(kThreads), 0, s, xy, n_segs, seg_stride, seg_counts,
                           e_int, (uint32_t)r2i, min_pts, min_cluster_size, max_cluster_size, labels, n_clusters, dups,
                           dup_cap, reinterpret_cast<unsigned long long *>(n_dups), err, left);
    }
    const unsigned grid = (unsigned)std::min<int64_t>(n_segs, run ? (int64_t)ctx->n_cu : 2048);
    {
        ECC_TIMED(ctx, s, run ? "dbscan_grid_left_kernel" : "dbscan_grid_kernel");
        hipLaunchKernelGGL(dbscan_grid_kernel, dim3(grid), dim3(kThreads), lds, s, xy, n_segs, seg_stride, seg_counts,
                           e_int, (uint32_t)r2i, min_pts, min_cluster_size, max_cluster_size, labels, n_clusters, dups,
                           dup_cap, reinterpret_cast<unsigned long long *>(n_dups), err,
                           run ? (const int32_t *)left : nullptr);
    }
    ECC_CHECK_LAUNCH(ctx, "dbscan_grid");
    return ECC_OK;
}

ECC_API int ecc_dbscan_status(ecc_ctx *ctx, ecc_stream_t stream) {
    if (!ctx) return ECC_ERR_INVALID;
    int32_t f = 0;
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(&f, ctx->flags + kFlagWord, 4, hipMemcpyDeviceToHost, ecc::as_stream(stream)),
                  "read dbscan err");
    ECC_CHECK_HIP(ctx, hipStreamSynchronize(ecc::as_stream(stream)), "sync");
    if (f & 4) return ECC_ERR_INVALID;  // a neighbour index outside its segment (ecc_dbscan_extract)
    return (f & 2) ? ECC_ERR_CAPACITY : ECC_OK;
}

#if ECC_DBSCAN_PROFILE
// Profiling builds only: dbscan_grid_kernel's summed phase ticks since the last call (reset after
// reading); out[7] = segments timed; ticks_per_us from the device.
ECC_API int ecc_dbscan_profile(unsigned long long *out8, double *ticks_per_us) {
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_db_prof), 8 * sizeof(unsigned long long)) != hipSuccess) return ECC_ERR_HIP;
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_db_prof), z, sizeof(z));
    int khz = 0;
    hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    *ticks_per_us = khz / 1000.0;
    return ECC_OK;
}
#endif
