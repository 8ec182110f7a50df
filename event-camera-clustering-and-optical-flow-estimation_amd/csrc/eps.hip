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
// coalesced (no 4/8-B scatter).  The list kernel builds each query's neighbour set as a bitmap
// over the segment (one wave per query) and emits it in ascending segment-local index order (the
// order of DBSCAN_precomp's adjacency lists), at offsets from a device exclusive scan of the counts.
// Algorithmic bytes: 4 B/point in + 4 B/point (count) [+ 8 B core distance] out; lists: + 4 B
// per neighbour out.
#include "eps_grid.hpp"

namespace {

using ecc::epsg::CellGrid;
using ecc::epsg::kCells;
using ecc::epsg::kNT;
using ecc::buffer_load_u32;
using ecc::buffer_view;
using ecc::xy_x;
using ecc::xy_y;
constexpr int kMaxPts = 16384;
constexpr int kLeftWord = 9;  // ctx->flags[9]: segments the row-run counts left to the candidate walk

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
// `left` (row-run leftovers mode): only the segments eps_run_counts_kernel marked
// (counts[base] == -1; *left = how many) are processed.
template <int K, bool kStage>
__global__ void __launch_bounds__(kNT)
eps_counts_kernel(const uint32_t *__restrict__ xy, SegView sv, int e_int, uint32_t r2i, int min_pts,
                  int32_t *__restrict__ counts, double *__restrict__ core, const int32_t *__restrict__ left) {
    extern __shared__ uint32_t lds_c[];
    uint32_t *cend = lds_c;
    uint32_t *spt = cend + kCells + 1;
    uint16_t *sidx = reinterpret_cast<uint16_t *>(spt + sv.stride);
    uint16_t *st_cnt = sidx + sv.stride;
    uint32_t *st_d2 = reinterpret_cast<uint32_t *>(st_cnt + ((sv.stride + 1) & ~1ll));
    __shared__ int red[64];
    const int tid = threadIdx.x;
    if (left && *left == 0) return;  // uniform: no leftovers
    for (int64_t s = blockIdx.x; s < sv.n_segs; s += gridDim.x) {
        const int m = seg_points(sv, s);
        const int64_t base = s * sv.stride;
        if (left && (m == 0 || counts[base] != -1)) continue;  // uniform: done by the row-run kernel
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

// Row-run form.  A segment's points are distinct pixels whenever it is a downsample window (one
// representative per hash bucket, and a pixel always hashes to the same bucket), so the segment is
// an occupancy bitmap over its bounding box, one bit per pixel, 32 pixels a word, each word paired
// with the number of points in the words before it (row-major).  The points of row y in [xl, xh)
// then number prefix(y, xh) - prefix(y, xl), with prefix(y, x) = base[word] + popc(bits[word]
// below x): a query's count is a sum over the 2*eps + 1 rows of the disk (half-width w(dy) =
// floor(sqrt(floor(eps^2) - dy^2)), the same integer test d^2 <= floor(eps^2) as the candidate
// walk), two LDS reads per row, no candidate loop and no test.  (Core distances by walking each
// row's run bit by bit measured 0.68 -> 0.92 ms at OPTICS eps 10; see K > 0 below.)  The bitmap
// of a 346 x 260
// sensor is 3120 words (25 KB): four 8-wave workgroups per CU share the CU's LDS, so one
// segment's set-up barriers overlap the others' queries.  A segment whose bitmap exceeds
// kRunWords or that repeats a pixel is left to eps_counts_kernel (marked by counts[base] = -1,
// counted in *left).
constexpr int kRT = 512;
constexpr int kRunWords = 4864;  // (bits, prefix) pairs: 38 KB, four workgroups per CU
constexpr int kHwTab = 512;      // eps < 512 (larger eps: the candidate walk)

// K > 0 (core distances, eps < 32): a disk row's chord lies inside the three bitmap words around
// the query's column, so the row is two 64-bit masks — the pixels at or left of x within the
// chord, and those right of it — whose popcounts give the count and whose K nearest set bits per
// side (leading / trailing zero counts, no per-bit loop) feed the K-smallest insertion network:
// a row holds at most K of the K nearest points on each side of x.
template <int K>
__global__ void __launch_bounds__(kRT)
eps_run_counts_kernel(const uint32_t *__restrict__ xy, SegView sv, int e_int, uint32_t r2i, int min_pts,
                      int32_t *__restrict__ counts, double *__restrict__ core, int32_t *__restrict__ left) {
    __shared__ uint2 wd[kRunWords + 1];  // [kRunWords]: a zero word for rows outside the box
    __shared__ int box[kRT / 64][4];
    __shared__ int wsum[kRT / 64];
    __shared__ int dup[2];  // by segment parity: reset one segment ahead, behind two barriers
    __shared__ uint16_t hwt[kHwTab];  // disk half-widths floor(sqrt(floor(eps^2) - a^2)), a < kHwTab
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int kW = kRT / 64;
    if (tid == 0) {
        wd[kRunWords] = make_uint2(0u, 0u);
        dup[0] = dup[1] = 0;
    }
    for (int a = tid; a < kHwTab && a <= e_int; a += kRT) {  // exact integer square roots
        const uint32_t v = r2i - (uint32_t)(a * a);
        uint32_t h = (uint32_t)sqrtf((float)v);
        while (h * h > v) --h;
        while ((h + 1) * (h + 1) <= v) ++h;
        hwt[a] = (uint16_t)h;
    }
    int par = 0;
    for (int64_t s = blockIdx.x; s < sv.n_segs; s += gridDim.x, par ^= 1) {
        if (tid == 0) dup[par ^ 1] = 0;  // last read in the previous segment, before its barrier 6
        const int m = seg_points(sv, s);
        const int64_t base = s * sv.stride;
        const __amdgpu_buffer_rsrc_t seg = buffer_view(xy + base, (uint32_t)m * 4u);
        int xmn = 0x7fffffff, ymn = 0x7fffffff, xmx = -1, ymx = -1;
        for (int q = tid; q < m; q += kRT) {
            const uint32_t v = buffer_load_u32(seg, (uint32_t)q * 4u);
            xmn = min(xmn, xy_x(v)); ymn = min(ymn, xy_y(v));
            xmx = max(xmx, xy_x(v)); ymx = max(ymx, xy_y(v));
        }
        xmn = ecc::wave_min_i32(xmn); ymn = ecc::wave_min_i32(ymn);  // DPP
        xmx = ecc::wave_max_i32(xmx); ymx = ecc::wave_max_i32(ymx);
        if (lane == 0) {
            box[wave][0] = xmn; box[wave][1] = ymn;
            box[wave][2] = xmx; box[wave][3] = ymx;
        }
        __syncthreads();  // 1
        xmn = box[0][0]; ymn = box[0][1]; xmx = box[0][2]; ymx = box[0][3];
#pragma unroll
        for (int w = 1; w < kW; ++w) {
            xmn = min(xmn, box[w][0]); ymn = min(ymn, box[w][1]);
            xmx = max(xmx, box[w][2]); ymx = max(ymx, box[w][3]);
        }
        const int Wb = m ? xmx - xmn + 1 : 1, H = m ? ymx - ymn + 1 : 1;
        const int WW = (Wb >> 5) + 1;  // words per row: x == Wb (a run's end) still has a word
        const int64_t words = (int64_t)H * WW;
        bool leftover = words > kRunWords;  // uniform
        if (!leftover) {
            for (int w = tid; w < words; w += kRT) wd[w] = make_uint2(0u, 0u);
        }
        __syncthreads();  // 2
        if (!leftover) {
            for (int q = tid; q < m; q += kRT) {
                const uint32_t v = buffer_load_u32(seg, (uint32_t)q * 4u);
                const int x = xy_x(v) - xmn, y = xy_y(v) - ymn;
                const uint32_t bit = 1u << (x & 31);
                const uint32_t old = atomicOr(&wd[y * WW + (x >> 5)].x, bit);
                if (old & bit) dup[par] = 1;
            }
        }
        __syncthreads();  // 3
        leftover = leftover || dup[par];  // uniform
        if (leftover) {
            if (tid == 0 && m > 0) {
                counts[base] = -1;
                atomicAdd(left, 1);
            }
        } else {
            if (K == 0) {  // prefix of the word popcounts: thread t takes words [t * per, t * per + per)
                const int per = (int)((words + kRT - 1) / kRT);
                const int w0 = tid * per, w1 = min(w0 + per, (int)words);
                int loc = 0;
                for (int w = w0; w < w1; ++w) loc += __popc(wd[w].x);
                const int inc = ecc::wave_incl_scan(loc);
                if (lane == 63) wsum[wave] = inc;
                __syncthreads();  // 4
                int off = inc - loc;
                for (int w = 0; w < wave; ++w) off += wsum[w];
                for (int w = w0; w < w1; ++w) {
                    wd[w].y = (uint32_t)off;
                    off += __popc(wd[w].x);
                }
                __syncthreads();  // 5
            }
            // queries in segment order: lane q's results at base + q (coalesced)
            const int amax = min(e_int, H - 1);  // rows beyond the box hold nothing
            for (int q = tid; q < sv.stride; q += kRT) {
                int cnt = 0;
                int best[K > 0 ? K : 1];
#pragma unroll
                for (int k = 0; k < (K > 0 ? K : 1); ++k) best[k] = 0x7fffffff;
                if (K > 0 && q < m) {
                    const uint32_t v = buffer_load_u32(seg, (uint32_t)q * 4u);
                    const int x = xy_x(v) - xmn, y = xy_y(v) - ymn;
                    const int wx = x >> 5, xb = x & 31;
                    for (int a = 0; a <= amax; ++a) {
                        const int hw = hwt[a];  // <= 31
                        const uint64_t lmask = ((2ull << (32 + xb)) - 1ull) & ~((1ull << (32 + xb - hw)) - 1ull);
                        const uint64_t rmask = (1ull << hw) - 1ull;
                        const int a2 = a * a;
#pragma unroll
                        for (int sgn = 0; sgn < 2; ++sgn) {
                            if (sgn && a == 0) break;
                            const int yy = sgn ? y - a : y + a;
                            const bool ok = (unsigned)yy < (unsigned)H;
                            const int rb = yy * WW;
                            const uint32_t w0 = wd[ok && wx > 0 ? rb + wx - 1 : kRunWords].x;
                            const uint32_t w1 = wd[ok ? rb + wx : kRunWords].x;
                            const uint32_t w2 = wd[ok && wx + 1 < WW ? rb + wx + 1 : kRunWords].x;
                            // bit 32 + xb of Lm is x itself; bit i of Rm is x + 1 + i
                            uint64_t Lm = (((uint64_t)w1 << 32) | w0) & lmask;
                            uint64_t Rm = ((((uint64_t)w2 << 32) | w1) >> (xb + 1)) & rmask;
                            cnt += __popcll(Lm) + __popcll(Rm);
#pragma unroll
                            for (int t = 0; t < K; ++t) {
                                const int pl = 63 - __clzll(Lm | 1ull);  // bit 0 is never in Lm
                                const int dl = 32 + xb - pl;
                                int vl = Lm ? dl * dl + a2 : 0x7fffffff;
                                Lm &= ~(1ull << pl);
                                const int dr = __ffsll((long long)Rm);  // 1-based: dx of the nearest
                                int vr = Rm ? dr * dr + a2 : 0x7fffffff;
                                Rm &= Rm - 1ull;
#pragma unroll
                                for (int k = 0; k < (K > 0 ? K : 1); ++k) {
                                    const int l1 = min(best[k], vl);
                                    vl = max(best[k], vl);
                                    best[k] = l1;
                                }
#pragma unroll
                                for (int k = 0; k < (K > 0 ? K : 1); ++k) {
                                    const int l1 = min(best[k], vr);
                                    vr = max(best[k], vr);
                                    best[k] = l1;
                                }
                            }
                        }
                    }
                } else if (q < m) {
                    const uint32_t v = buffer_load_u32(seg, (uint32_t)q * 4u);
                    const int x = xy_x(v) - xmn, y = xy_y(v) - ymn;
#pragma unroll 4
                    for (int a = 0; a <= amax; ++a) {
                        const int hw = hwt[a];  // a broadcast read; no loop-carried state
                        const int xl = max(x - hw, 0), xh = min(x + hw + 1, Wb);
                        const uint32_t ml = (1u << (xl & 31)) - 1u, mh = (1u << (xh & 31)) - 1u;
                        const int cl = xl >> 5, ch = xh >> 5;
#pragma unroll
                        for (int sgn = 0; sgn < 2; ++sgn) {
                            if (sgn && a == 0) break;
                            const int yy = sgn ? y - a : y + a;
                            const bool ok = (unsigned)yy < (unsigned)H;
                            const int rb = yy * WW;
                            const uint2 lo = wd[ok ? rb + cl : kRunWords], hi = wd[ok ? rb + ch : kRunWords];
                            cnt += (int)(hi.y - lo.y) + __popc(hi.x & mh) - __popc(lo.x & ml);
                        }
                    }
                }
                counts[base + q] = cnt;
                if (K > 0) {
                    uint32_t sel = 0xffffffffu;  // not a core point (or padding)
                    if (cnt >= min_pts) {
#pragma unroll
                        for (int k = 0; k < (K > 0 ? K : 1); ++k) sel = (k == min_pts - 1) ? (uint32_t)best[k] : sel;
                    }
                    core[base + q] = sel == 0xffffffffu ? -1.0 : sqrt((double)sel);  // correctly rounded
                }
            }
        }
        __syncthreads();  // 6: the LDS is reused by the next segment
    }
}

// One query of eps_lists_kernel on the calling wave (all 64 lanes; v is wave-uniform): sets the
// bitmap bits of its neighbours, then writes them ascending to nbr[out0, end) and clears the
// bitmap words it used.  Branch-free row setup (all 14 cell-bound reads in flight together), two
// candidates per lane per trip with their point and index read together, DPP prefix of the
// per-lane counts: a handful of dependent LDS round trips per query.
template <bool kN>
__device__ __forceinline__ void emit_list(const CellGrid &g, const uint32_t *cend, const uint32_t *spt,
                                          const uint16_t *sidx, unsigned long long *bits, uint32_t v, int e_int,
                                          uint32_t r2i, int words, int wpl, int64_t out0, int64_t end,
                                          int32_t *__restrict__ nbr, int64_t nbr_cap, int32_t *__restrict__ err) {
    constexpr int kRows = 2 * ecc::epsg::kMaxR + 1;
    const int lane = threadIdx.x & 63;
    const int cx = ecc::epsg::cell_x(g, v), cy = ecc::epsg::cell_y(g, v);
    // the rows' cell bounds: lane 2r reads row r's start bound, lane 2r + 1 its end (one LDS
    // read per lane, all in flight together), then the wave takes them with readlane
    int idx = 0;
    {
        const int r = lane >> 1, ry = cy + r - ecc::epsg::kMaxR;
        int kx = -1;  // g.kx[r] by selects (a runtime index would put g.kx in scratch memory)
#pragma unroll
        for (int q = 0; q < kRows; ++q) kx = r == q ? g.kx[q] : kx;
        if (kx >= 0 && ry >= 0 && ry < g.gy) {
            const int cl = ry * g.gx + max(cx - kx, 0), ch = ry * g.gx + min(cx + kx, g.gx - 1);
            idx = (lane & 1) ? ch : (cl > 0 ? cl - 1 : -1);
        } else {
            idx = -1;
        }
    }
    const int bound = idx >= 0 ? (int)cend[idx] : 0;  // invalid rows and cell 0's start read as 0
    int pre[kRows + 1], off[kRows];
    pre[0] = 0;
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        const int lo = __builtin_amdgcn_readlane(bound, 2 * r), hi = __builtin_amdgcn_readlane(bound, 2 * r + 1);
        off[r] = lo - pre[r];
        pre[r + 1] = pre[r] + (hi - lo);
    }
    const int total_c = pre[kRows];
    for (int f = lane; f < total_c; f += 128) {
        const int f2 = f + 64, f2c = f2 < total_c ? f2 : f;
        int a0 = f + off[0], a1 = f2c + off[0];
#pragma unroll
        for (int r = 1; r < kRows; ++r) {
            a0 = f >= pre[r] ? f + off[r] : a0;
            a1 = f2c >= pre[r] ? f2c + off[r] : a1;
        }
        const uint32_t w0 = spt[a0], w1 = spt[a1];
        const int j0 = sidx[a0], j1 = sidx[a1];
        asm volatile("" ::"v"(j0), "v"(j1));  // both index reads issued with the point reads
        uint32_t d2;
        if (ecc::epsg::in_eps<kN>(v, w0, e_int, r2i, &d2))
            __hip_atomic_fetch_or(&bits[j0 >> 6], 1ull << (j0 & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        if (f2 < total_c && ecc::epsg::in_eps<kN>(v, w1, e_int, r2i, &d2))
            __hip_atomic_fetch_or(&bits[j1 >> 6], 1ull << (j1 & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    unsigned long long wv[4];
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int w = lane * wpl + k;
        const bool mine = k < wpl && w < words;
        wv[k] = mine ? bits[w] : 0ull;
        cnt += __popcll(wv[k]);
        if (mine) bits[w] = 0ull;
    }
    const int inc = ecc::wave_incl_scan(cnt);
    const int total = __builtin_amdgcn_readlane(inc, 63);
    if (lane == 0 && out0 + total != end) *err = 1;  // counts disagree with the lists
    int64_t out = out0 + (inc - cnt);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        unsigned long long x = wv[k];
        const int jb = (lane * wpl + k) << 6;
        while (x) {
            const int j = jb + __builtin_ctzll(x);
            x &= x - 1;
            if (out < end && out < nbr_cap) nbr[out] = j;
            else *err = 1;
            ++out;
        }
    }
}

// Ascending neighbour lists, one WAVE per query, queries in segment-index order.  Dynamic LDS:
// cend[kCells + 1] | spt[stride] | sidx[stride] (the fine grid) | a neighbour bitmap of
// ceil(stride / 64) u64 words per wave.  The wave walks the query's candidate rows flattened
// (lane f takes candidate f, f + 64, ...), sets bit j of every candidate j within eps (ds_or),
// then each lane takes wpl consecutive bitmap words, and a wave prefix of their popcounts places
// its indices: the list comes out ascending (DBSCAN_precomp's adjacency order) and one query's
// list is written by one wave into its own contiguous range, so consecutive stores of a wave
// land in the same lines (the lane-per-query merge wrote each lane's list one 4-B store at a
// time into its own line: 3x write amplification at the memory side, 8 ms at C4).
__global__ void __launch_bounds__(kNT)
eps_lists_kernel(const uint32_t *__restrict__ xy, SegView sv, int e_int, uint32_t r2i,
                 const int64_t *__restrict__ offsets, int32_t *__restrict__ nbr, int64_t nbr_cap,
                 int32_t *__restrict__ err) {
    extern __shared__ uint32_t lds_l[];
    uint32_t *cend = lds_l;
    uint32_t *spt = cend + kCells + 1;
    uint16_t *sidx = reinterpret_cast<uint16_t *>(spt + sv.stride);
    const int n_words = (int)((sv.stride + 63) >> 6);
    unsigned long long *bits_all =
        reinterpret_cast<unsigned long long *>(lds_l + ((kCells + 1 + sv.stride + (sv.stride + 1) / 2 + 1) & ~1ll));
    __shared__ int red[64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int kW = kNT / 64;
    unsigned long long *bits = bits_all + (int64_t)wave * n_words;
    for (int w = lane; w < n_words; w += 64) bits[w] = 0ull;
    for (int64_t s = blockIdx.x; s < sv.n_segs; s += gridDim.x) {
        const int m = seg_points(sv, s);
        const int64_t base = s * sv.stride;
        const CellGrid g = ecc::epsg::bin_cells(xy, base, m, e_int, r2i, cend, spt, sidx, red, false, true);
        const int words = (m + 63) >> 6, wpl = (words + 63) >> 6;  // bitmap words in use, per lane
        ecc::epsg::with_narrow(g, [&](auto narrow) {
            constexpr bool kN = decltype(narrow)::value;
            // a wave's queries are q = wave + kW * t; lane L prefetches query t0 + L's point and
            // list range for the next 64 (no dependent global load per query)
            for (int t0 = 0; wave + kW * t0 < m; t0 += 64) {
                const int ql = wave + kW * (t0 + lane);
                const uint32_t pv = ql < m ? xy[base + ql] : 0u;
                const int64_t po0 = ql < m ? offsets[base + ql] : 0, po1 = ql < m ? offsets[base + ql + 1] : 0;
                for (int tt = 0; tt < 64; ++tt) {
                    if (wave + kW * (t0 + tt) >= m) break;  // wave-uniform
                    // the query's point and list range: readlane of a wave-uniform lane (no permute)
                    const uint32_t v = (uint32_t)ecc::lane_value((int)pv, tt);
                    const int64_t out0 = ecc::lane_value64(po0, tt), end = ecc::lane_value64(po1, tt);
                    emit_list<kN>(g, cend, spt, sidx, bits, v, e_int, r2i, words, wpl, out0, end, nbr, nbr_cap, err);
                }
            }
        });
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
#define ECC_EPS_PICK(S)                                                                                        \
    (K == 0 ? eps_counts_kernel<0, S> : K <= 1 ? eps_counts_kernel<1, S> : K <= 2 ? eps_counts_kernel<2, S>     \
     : K <= 4 ? eps_counts_kernel<4, S> : K <= 8 ? eps_counts_kernel<8, S> : K <= 16 ? eps_counts_kernel<16, S> \
     : K <= 32 ? eps_counts_kernel<32, S> : eps_counts_kernel<64, S>)
    using Kern = void (*)(const uint32_t *, SegView, int, uint32_t, int, int32_t *, double *, const int32_t *);
    const Kern kern = stage ? (Kern)ECC_EPS_PICK(true) : (Kern)ECC_EPS_PICK(false);
#undef ECC_EPS_PICK
    const size_t lds = grid_lds + (stage ? stage_lds : 0);
    ECC_CHECK_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                  "eps_counts lds");
    hipStream_t s = ecc::as_stream(stream);
    // counts: the row-run kernel (eps < 512); with core distances when min_pts <= 8 and eps < 32.
    // Its leftovers (segments that repeat a pixel or whose bitmap exceeds its LDS) go through the
    // candidate walk, which exits at once without any; other cases take the candidate walk whole.
    const bool run = K == 0 ? e_int < kHwTab : (K <= 8 && e_int < 32);
    if (run) {
        int32_t *left = ctx->flags + kLeftWord;
        ECC_CHECK_HIP(ctx, hipMemsetAsync(left, 0, 4, s), "memset(eps leftovers)");
        {
            using RunKern = void (*)(const uint32_t *, SegView, int, uint32_t, int, int32_t *, double *, int32_t *);
            const RunKern rk = K == 0 ? eps_run_counts_kernel<0> : K <= 1 ? eps_run_counts_kernel<1>
                             : K <= 2 ? eps_run_counts_kernel<2> : K <= 4 ? eps_run_counts_kernel<4>
                             : eps_run_counts_kernel<8>;
            ECC_TIMED(ctx, s, "eps_run_counts_kernel");
            // one workgroup per segment (a resident grid of 4 per CU striding over 2442 segments
            // left its last round 40 % full)
            const unsigned grid = (unsigned)std::min<int64_t>(n_segs, 1 << 20);
            hipLaunchKernelGGL(rk, dim3(grid), dim3(kRT), 0, s, xy, sv, e_int, (uint32_t)r2i, min_pts, counts,
                               core_dist, left);
        }
        ECC_TIMED(ctx, s, "eps_counts_left_kernel");
        const unsigned grid = (unsigned)std::min<int64_t>(n_segs, ctx->n_cu);  // one WG per CU (LDS)
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kNT), lds, s, xy, sv, e_int, (uint32_t)r2i, min_pts, counts,
                           core_dist, (const int32_t *)left);
    } else {
        // segments are grid-strided; enough workgroups for every CU at the occupancy the LDS allows
        ECC_TIMED(ctx, s, "eps_counts_kernel");
        const unsigned grid = (unsigned)std::min<int64_t>(n_segs, 2048);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kNT), lds, s, xy, sv, e_int, (uint32_t)r2i, min_pts, counts,
                           core_dist, (const int32_t *)nullptr);
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
    const size_t grid_words = (size_t)((kCells + 1 + seg_stride + (seg_stride + 1) / 2 + 1) & ~1ll);
    const size_t lds = grid_words * 4 + (size_t)(kNT / 64) * ((seg_stride + 63) / 64) * 8;
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
