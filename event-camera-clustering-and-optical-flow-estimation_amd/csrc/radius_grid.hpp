// A global uniform cell grid over an arbitrary point set of 1-3 dimensions (fp32 or fp64
// coordinates), shared by the eps-ball kernels (radius.hip: OPTICS counts / core distances /
// lists) and the any-N DBSCAN (dbscan_cloud.hip).
//
// Distances follow the reference's operation order exactly:
//   * DBSCAN_simple.h:132-135 / DBSCAN_precomp.h:31-34 (pcl::PointXYZ, float fields):
//     `double distance_x = points[i].x - points[index].x` — the difference is taken in FLOAT
//     and then widened; distance_square = dx*dx + dy*dy + dz*dz in double;
//   * kdTree.hpp:180-192 (OPTICS, coordinate type T): d = p1[i] - p2[i] in T, result += d * d
//     in double.
// Both are `sq_dist<T, D>`: the per-axis difference in T, widened, squared and summed left to
// right in double with no FMA contraction.  A point is its own neighbour (d = 0).
//
// Grid: cells of eps * (1 + 1e-6) (|p - q| <= eps keeps floor((p - mn) / cs) within one cell
// despite the rounding of the fp32 difference, <= 2^-24 relative), doubled until at most
// max_cells cells.  Points are counting-sorted by cell into SoA arrays (sc[d * n + k]) with
// their original indices (sidx[k]); a query walks the 3^(D-1) contiguous runs of its 3^D cells.
#pragma once

#include "ecc_internal.hpp"

#include <algorithm>
#include <cmath>

namespace ecc {
namespace rgrid {

constexpr int kThreads = 256;
constexpr int kGridWord = 16;  // ctx->flags[16..]: bounding-box keys, then the grid geometry
constexpr int kBadWord = 7;    // ctx->flags[7]: bit 1 = a non-finite coordinate was seen (radius status)

struct Grid {
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

static __global__ void __launch_bounds__(kThreads)
bbox_init_kernel(int64_t *keys) {
    if (threadIdx.x < 3) keys[threadIdx.x] = 0x7fffffffffffffffll;                 // min
    else if (threadIdx.x < 6) keys[threadIdx.x] = (int64_t)0x8000000000000000ull;  // max
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
bbox_kernel(const T *__restrict__ pts, int64_t n, int dim, int64_t *keys, int32_t *bad) {
    int64_t mn[3] = {0x7fffffffffffffffll, 0x7fffffffffffffffll, 0x7fffffffffffffffll};
    int64_t mx[3] = {(int64_t)0x8000000000000000ull, (int64_t)0x8000000000000000ull, (int64_t)0x8000000000000000ull};
    bool fin = true;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
        // a point with a non-finite coordinate is left out of the box: its distance to every
        // other point is NaN or inf, never <= eps^2 (the reference's `d2 <= r2`), so whatever
        // cell it lands in it is nobody else's neighbour (the DBSCAN cloud counts the query point
        // itself unconditionally, as radiusSearch does; the radius entry points report such
        // input through `bad` instead)
        double v[3] = {0.0, 0.0, 0.0};
        bool pf = true;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            if (d >= dim) break;
            v[d] = (double)pts[i * dim + d];
            pf = pf && isfinite(v[d]);
        }
        fin = fin && pf;
        if (!pf) continue;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            if (d >= dim) break;
            const int64_t k = dkey(v[d]);
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
    if (!fin) atomicOr(bad, 2);
    if ((threadIdx.x & 63) == 0)
        for (int d = 0; d < dim; ++d) {
            atomicMin(reinterpret_cast<long long *>(keys + d), (long long)mn[d]);
            atomicMax(reinterpret_cast<long long *>(keys + 3 + d), (long long)mx[d]);
        }
}

static __global__ void grid_setup_kernel(const int64_t *keys, int dim, double eps, int64_t max_cells, Grid *g) {
    if (threadIdx.x != 0) return;
    Grid r{};
    r.dim = dim;
    double cs = eps > 0.0 ? eps * (1.0 + 1e-6) : 1.0;
    double span[3] = {0.0, 0.0, 0.0};
    for (int d = 0; d < dim; ++d) {
        r.mn[d] = dval(keys[d]);
        span[d] = dval(keys[3 + d]) - r.mn[d];
        if (!(span[d] >= 0.0)) span[d] = 0.0;  // no finite point at all: one cell
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
    const double f = floor((v - mn) / cs);
    if (!(f >= 0.0)) return 0;  // also NaN
    return f >= (double)dims ? dims - 1 : (int64_t)f;
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
cell_count_kernel(const T *__restrict__ pts, int64_t n, const Grid *__restrict__ gp, int32_t *__restrict__ cell_of,
                  int32_t *__restrict__ cell_cnt) {
    const Grid g = *gp;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
        int64_t c = 0;
        for (int d = g.dim - 1; d >= 0; --d)
            c = c * g.dims[d] + cell_coord((double)pts[i * g.dim + d], g.mn[d], g.cs, g.dims[d]);
        cell_of[i] = (int32_t)c;
        atomicAdd(&cell_cnt[c], 1);
    }
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
cell_scatter_kernel(const T *__restrict__ pts, int64_t n, int dim, const int32_t *__restrict__ cell_of,
                    const int64_t *__restrict__ cell_off, int32_t *__restrict__ cursor, int32_t *__restrict__ sidx,
                    T *__restrict__ sc) {
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
        const int32_t c = cell_of[i];
        const int64_t pos = cell_off[c] + atomicAdd(&cursor[c], 1);
        sidx[pos] = (int32_t)i;
        for (int d = 0; d < dim; ++d) sc[(int64_t)d * n + pos] = pts[i * dim + d];
    }
}

// squared distance in the reference's operation order (see the header comment)
template <typename T, int D>
__device__ __forceinline__ double sq_dist(const T *__restrict__ sc, int64_t n, int64_t j, const T *p) {
    double s = 0.0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const T diff = sc[(int64_t)d * n + j] - p[d];  // in the coordinate type
        const double dd = (double)diff;
        s = __dadd_rn(s, __dmul_rn(dd, dd));
    }
    return s;
}

// A query's cell coordinates and the 3^(D-1) contiguous runs [lo, hi) of sorted positions that
// hold its 3^D neighbour cells; f(lo, hi) per run.
template <typename T, int D, typename F>
__device__ __forceinline__ void for_runs(const Grid &g, const int64_t *__restrict__ cell_off, const T *p, F &&f) {
    int64_t c[3] = {0, 0, 0};
#pragma unroll
    for (int d = 0; d < D; ++d) c[d] = cell_coord((double)p[d], g.mn[d], g.cs, g.dims[d]);
    const int64_t z0 = D >= 3 ? (c[2] > 0 ? c[2] - 1 : 0) : 0, z1 = D >= 3 ? (c[2] + 1 < g.dims[2] ? c[2] + 1 : c[2]) : 0;
    const int64_t y0 = D >= 2 ? (c[1] > 0 ? c[1] - 1 : 0) : 0, y1 = D >= 2 ? (c[1] + 1 < g.dims[1] ? c[1] + 1 : c[1]) : 0;
    const int64_t x0 = c[0] > 0 ? c[0] - 1 : 0, x1 = c[0] + 1 < g.dims[0] ? c[0] + 1 : c[0];
    for (int64_t z = z0; z <= z1; ++z)
        for (int64_t y = y0; y <= y1; ++y) {
            const int64_t row = (z * g.dims[1] + y) * g.dims[0];
            f(cell_off[row + x0], cell_off[row + x1 + 1]);
        }
}

struct Ws {
    int64_t *keys;
    Grid *grid;
    int32_t *cell_cnt, *cell_of, *sidx;
    int64_t *cell_off, *scan;
    void *sc;
    int64_t max_cells;
};

inline int64_t max_cells_for(int64_t n) {
    // cell ids are int32 (cell_of), so at most 2^31 - 2 cells whatever n is
    return std::min<int64_t>(std::max<int64_t>(4 * n, 4096), (int64_t)INT32_MAX - 1);
}

// bytes of grid workspace for n points of `dim` coordinates of `tbytes` bytes
inline size_t ws_bytes(int64_t n, int dim, size_t tbytes) {
    const int64_t mc = max_cells_for(n);
    return align_up((size_t)mc * 4, 256) + align_up((size_t)(mc + 1) * 8, 256) +
           align_up(scan_scratch_bytes(std::max<int64_t>(mc, n)), 256) + 2 * align_up((size_t)n * 4, 256) +
           align_up((size_t)n * tbytes * dim, 256) + align_up((size_t)(n + 1) * 8, 256);
}

// Builds the grid in the workspace at `base` (ws_bytes(n, dim, sizeof(T)) bytes).
template <typename T>
int build(ecc_ctx *ctx, const T *pts, int64_t n, int dim, double eps, hipStream_t s, char *base, Ws &w) {
    w.max_cells = max_cells_for(n);
    char *p = base;
    auto carve = [&](size_t bytes) { char *r = p; p += align_up(bytes, 256); return r; };
    w.cell_cnt = reinterpret_cast<int32_t *>(carve((size_t)w.max_cells * 4));
    w.cell_off = reinterpret_cast<int64_t *>(carve((size_t)(w.max_cells + 1) * 8));
    w.scan = reinterpret_cast<int64_t *>(carve(scan_scratch_bytes(std::max<int64_t>(w.max_cells, n))));
    w.cell_of = reinterpret_cast<int32_t *>(carve((size_t)n * 4));
    w.sidx = reinterpret_cast<int32_t *>(carve((size_t)n * 4));
    w.sc = carve((size_t)n * sizeof(T) * dim);
    w.keys = reinterpret_cast<int64_t *>(ctx->flags + kGridWord);
    w.grid = reinterpret_cast<Grid *>(ctx->flags + kGridWord + 12);
    int32_t *bad = ctx->flags + kBadWord;
    const unsigned blocks = (unsigned)std::min<int64_t>((n + kThreads - 1) / kThreads, 4096);
    ECC_CHECK_HIP(ctx, hipMemsetAsync(bad, 0, 4, s), "memset(radius bad)");
    hipLaunchKernelGGL(bbox_init_kernel, dim3(1), dim3(kThreads), 0, s, w.keys);
    {
        ECC_TIMED(ctx, s, "radius_grid_kernels");
        hipLaunchKernelGGL(bbox_kernel<T>, dim3(blocks), dim3(kThreads), 0, s, pts, n, dim, w.keys, bad);
        hipLaunchKernelGGL(grid_setup_kernel, dim3(1), dim3(64), 0, s, (const int64_t *)w.keys, dim, eps, w.max_cells,
                           w.grid);
        ECC_CHECK_HIP(ctx, hipMemsetAsync(w.cell_cnt, 0, (size_t)w.max_cells * 4, s), "memset(cells)");
        hipLaunchKernelGGL(cell_count_kernel<T>, dim3(blocks), dim3(kThreads), 0, s, pts, n, (const Grid *)w.grid,
                           w.cell_of, w.cell_cnt);
    }
    int rc = exclusive_scan_i32_i64(ctx, w.cell_cnt, w.max_cells, w.cell_off, w.scan, s);
    if (rc) return rc;
    ECC_CHECK_HIP(ctx, hipMemsetAsync(w.cell_cnt, 0, (size_t)w.max_cells * 4, s), "memset(cursor)");
    {
        ECC_TIMED(ctx, s, "radius_scatter_kernel");
        hipLaunchKernelGGL(cell_scatter_kernel<T>, dim3(blocks), dim3(kThreads), 0, s, pts, n, dim,
                           (const int32_t *)w.cell_of, (const int64_t *)w.cell_off, w.cell_cnt, w.sidx,
                           reinterpret_cast<T *>(w.sc));
    }
    ECC_CHECK_LAUNCH(ctx, "radius grid");
    return ECC_OK;
}

// status word of the last build: a non-finite coordinate -> ECC_ERR_INVALID
inline int bad_status(ecc_ctx *ctx, hipStream_t s) {
    int32_t f = 0;
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(&f, ctx->flags + kBadWord, 4, hipMemcpyDeviceToHost, s), "read radius bad");
    ECC_CHECK_HIP(ctx, hipStreamSynchronize(s), "sync");
    return f ? ECC_ERR_INVALID : ECC_OK;
}

}  // namespace rgrid
}  // namespace ecc
