// LDS cell grid of one point segment, shared by the eps-neighbourhood kernels (eps.hip) and the
// fused grid DBSCAN (dbscan.hip).  One 1024-lane workgroup (16 waves) per segment: the points
// are counting-sorted by a uniform grid straight into LDS.  Coarse grids (cell e_int + 1 > eps,
// the ordered list merge) put a neighbour in the 3x3 cells around a point; fine grids (cell
// ~ (eps + 1) / 3) walk, per cell row dyc in [-R, R], only the cell columns that can hold a
// point within eps (|dxc| <= kx[dyc], from the row's smallest |dy|): ~0.56x the candidates of
// the 3x3 coarse walk at eps 20.  A row's cells are adjacent in cell order: one contiguous run.
//
// Reference: the radius search this replaces is DBSCANSimpleCluster::radiusSearch
// (PCC/DBSCAN_simple.h:118-142: d^2 <= eps^2 in double, self included) and the kd-tree's
// radius_search (OPT/include/optics/kdTree.hpp:407-422, square_distance <= r^2, :180-192).
// Integer coordinates make d^2 an exact integer, so d^2 <= eps^2 (fp64) <=> d^2 <= floor(eps^2)
// and |dx|, |dy| <= floor(eps).
#pragma once

#include "ecc_internal.hpp"

#include <type_traits>

namespace ecc {
namespace epsg {

constexpr int kNT = 1024;     // threads per workgroup
constexpr int kCells = 4096;  // grid cells held in LDS (the cell size doubles until they fit)
constexpr int kMaxR = 3;      // cell rows on each side of a query's row (fine grids)

struct CellGrid {
    int xmn, ymn, cs, gx, gy;
    bool narrow;  // both spans <= 32767: coordinate differences fit packed i16 lanes
    int R;        // cell rows walked on each side
    int kx[2 * kMaxR + 1];  // cell columns walked on each side, per row offset (-1: none)
};

typedef short v2i16 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int cell_x(const CellGrid &g, uint32_t v) { return (xy_x(v) - g.xmn) / g.cs; }
__device__ __forceinline__ int cell_y(const CellGrid &g, uint32_t v) { return (xy_y(v) - g.ymn) / g.cs; }

// Exact eps test on packed integer points, branch-free.  Narrow grids (both spans <= 32767;
// the caller picks the variant once per segment): one packed i16 subtract and one i16 dot
// product (v_pk_sub_i16 + v_dot2_i32_i16), d^2 <= 2 * 32767^2 < 2^31 exact.  Otherwise the
// per-axis bound keeps the u32 d^2 exact.
template <bool kNarrow>
__device__ __forceinline__ bool in_eps(uint32_t v, uint32_t w, int e_int, uint32_t r2i, uint32_t *d2out) {
    if (kNarrow) {
        const v2i16 d = __builtin_bit_cast(v2i16, w) - __builtin_bit_cast(v2i16, v);
        const uint32_t d2 = (uint32_t)__builtin_amdgcn_sdot2(d, d, 0, false);
        *d2out = d2;
        return d2 <= r2i;
    }
    const uint32_t ax = (uint32_t)abs(xy_x(w) - xy_x(v)), ay = (uint32_t)abs(xy_y(w) - xy_y(v));
    const uint32_t d2 = ax * ax + ay * ay;  // exact whenever ax, ay <= e_int <= 32767
    *d2out = d2;
    return (ax <= (uint32_t)e_int) & (ay <= (uint32_t)e_int) & (d2 <= r2i);
}

// Runs body(std::true_type{}) on narrow grids, body(std::false_type{}) otherwise: the eps test
// variant is chosen once per segment, outside the candidate loops.
template <class B>
__device__ __forceinline__ void with_narrow(const CellGrid &g, B &&body) {
    if (g.narrow) body(std::true_type{});
    else body(std::false_type{});
}

// Bins the m points xy[base, base + m) into LDS in cell order (kNT threads, all must call):
//   spt[p] = the packed point at cell-order position p, sidx[p] = its index in the segment;
//   cend[c] = exclusive end of cell c's run (cell c starts at c ? cend[c - 1] : 0).
// `ascending`: each cell's run is additionally sorted by segment index (insertion sort per cell).
// `fine`: the fine grid (for_candidates); otherwise the coarse 3x3 grid (cell e_int + 1).
// red: >= 64 ints of LDS scratch.  Returns the grid; ends with a barrier.
__device__ __forceinline__ CellGrid bin_cells(const uint32_t *__restrict__ xy, int64_t base, int m, int e_int,
                                              uint32_t r2i, uint32_t *cend, uint32_t *spt, uint16_t *sidx, int *red,
                                              bool ascending, bool fine) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int kW = kNT / 64;
    // the points stay in registers from the bounding box to the placement (<= 16 per lane)
    constexpr int kHold = 16;
    uint32_t pv[kHold];
    int xmn = 0x7fffffff, ymn = 0x7fffffff, xmx = -1, ymx = -1;
    // loads through a buffer view of the segment (0 past m), all unconditional (a load under a
    // per-lane condition waited for every earlier one: 16 round trips per segment)
    const __amdgpu_buffer_rsrc_t seg = buffer_view(xy + base, (uint32_t)m * 4u);
#pragma unroll
    for (int u = 0; u < kHold; ++u) pv[u] = buffer_load_u32(seg, (uint32_t)tid * 4u, (uint32_t)(u * kNT) * 4u);
#pragma unroll
    for (int u = 0; u < kHold; ++u) {
        if (u * kNT + tid < m) {
            xmn = min(xmn, xy_x(pv[u])); ymn = min(ymn, xy_y(pv[u]));
            xmx = max(xmx, xy_x(pv[u])); ymx = max(ymx, xy_y(pv[u]));
        }
    }
    xmn = wave_min_i32(xmn); ymn = wave_min_i32(ymn);  // DPP
    xmx = wave_max_i32(xmx); ymx = wave_max_i32(ymx);
    if (lane == 0) {
        red[4 * wave + 0] = xmn; red[4 * wave + 1] = ymn;
        red[4 * wave + 2] = xmx; red[4 * wave + 3] = ymx;
    }
    for (int c = tid; c <= kCells; c += kNT) cend[c] = 0u;
    __syncthreads();
    xmn = red[0]; ymn = red[1]; xmx = red[2]; ymx = red[3];
#pragma unroll
    for (int w = 1; w < kW; ++w) {
        xmn = min(xmn, red[4 * w]); ymn = min(ymn, red[4 * w + 1]);
        xmx = max(xmx, red[4 * w + 2]); ymx = max(ymx, red[4 * w + 3]);
    }
    if (m == 0) { xmn = ymn = 0; xmx = ymx = 0; }
    // coarse: cell > eps, 3x3; fine: cell ~ (eps + 1) / 3
    int cs = fine ? max(1, (e_int + 3) / 3) : e_int + 1;
    while ((int64_t)((xmx - xmn) / cs + 1) * ((ymx - ymn) / cs + 1) > kCells) cs *= 2;
    CellGrid g;
    g.xmn = xmn; g.ymn = ymn; g.cs = cs;
    g.gx = (xmx - xmn) / cs + 1; g.gy = (ymx - ymn) / cs + 1;
    g.narrow = xmx - xmn <= 32767 && ymx - ymn <= 32767;
    g.R = (e_int + cs - 1) / cs;  // |dy| <= e_int  =>  |dyc| <= ceil(e_int / cs) <= 3
#pragma unroll
    for (int r = 0; r <= 2 * kMaxR; ++r) {
        const int dyc = r - kMaxR, ady = abs(dyc);
        // smallest |dy| between points whose cell rows differ by dyc; then the widest |dx| left
        const int64_t dymin = ady == 0 ? 0 : (int64_t)(ady - 1) * cs + 1;
        const int64_t rem = (int64_t)r2i - dymin * dymin;
        int kx = -1;
        if (ady <= g.R && rem >= 0) {
            kx = 0;
            while (kx < g.R && ((int64_t)kx * cs + 1) * ((int64_t)kx * cs + 1) <= rem) ++kx;
        }
        g.kx[r] = kx;
    }
    __syncthreads();  // red reusable
#pragma unroll
    for (int u = 0; u < kHold; ++u)
        if (u * kNT + tid < m) atomicAdd(&cend[cell_y(g, pv[u]) * g.gx + cell_x(g, pv[u])], 1u);
    __syncthreads();
    {  // exclusive scan of the cell counts in place (kCells / kNT per thread)
        constexpr int per = kCells / kNT;
        uint32_t loc[per], sum = 0;
#pragma unroll
        for (int k = 0; k < per; ++k) { loc[k] = cend[tid * per + k]; sum += loc[k]; }
        const uint32_t inc = (uint32_t)wave_incl_scan((int)sum);  // DPP
        if (lane == 63) red[wave] = (int)inc;
        __syncthreads();
        uint32_t off = inc - sum;
        for (int w = 0; w < wave; ++w) off += (uint32_t)red[w];
#pragma unroll
        for (int k = 0; k < per; ++k) { cend[tid * per + k] = off; off += loc[k]; }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kHold; ++u) {  // afterwards cend[c] = end of cell c
        if (u * kNT + tid >= m) continue;
        const uint32_t at = atomicAdd(&cend[cell_y(g, pv[u]) * g.gx + cell_x(g, pv[u])], 1u);
        spt[at] = pv[u];
        sidx[at] = (uint16_t)(u * kNT + tid);
    }
    __syncthreads();
    if (ascending) {
        for (int c = tid; c < g.gx * g.gy; c += kNT) {
            const int lo = c == 0 ? 0 : (int)cend[c - 1], hi = (int)cend[c];
            for (int a = lo + 1; a < hi; ++a) {
                const uint16_t key = sidx[a];
                const uint32_t kv = spt[a];
                int b = a - 1;
                while (b >= lo && sidx[b] > key) {
                    sidx[b + 1] = sidx[b];
                    spt[b + 1] = spt[b];
                    --b;
                }
                sidx[b + 1] = key;
                spt[b + 1] = kv;
            }
        }
        __syncthreads();
    }
    return g;
}

// Calls f(a, w, ok) for the cell-order positions a of the cells around point v that can hold a
// point within eps (the candidates; w = spt[a]; f applies the eps test and must ignore ok ==
// false).  Each cell row's columns are one contiguous run, walked four positions at a time with
// the four LDS reads issued together (a tail slot reads a stale in-allocation word, ok == false).
template <class F>
__device__ __forceinline__ void for_candidates(const CellGrid &g, const uint32_t *cend, const uint32_t *spt,
                                               uint32_t v, F &&f) {
    const int cx = cell_x(g, v), cy = cell_y(g, v);
#pragma unroll
    for (int r = 0; r <= 2 * kMaxR; ++r) {
        const int ry = cy + r - kMaxR, kx = g.kx[r];
        if (kx < 0 || ry < 0 || ry >= g.gy) continue;
        const int cl = ry * g.gx + max(cx - kx, 0), ch = ry * g.gx + min(cx + kx, g.gx - 1);
        const int hi = (int)cend[ch];
        for (int a = cl == 0 ? 0 : (int)cend[cl - 1]; a < hi; a += 4) {
            uint32_t w[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) w[k] = spt[a + k];
#pragma unroll
            for (int k = 0; k < 4; ++k) f(a + k, w[k], a + k < hi);
        }
    }
}

}  // namespace epsg
}  // namespace ecc
