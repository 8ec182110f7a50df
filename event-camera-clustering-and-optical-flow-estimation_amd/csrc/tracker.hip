// Corner tracker: damped predictor-corrector with grouping.
//
// Reference: class CornerTracker, FCT/metavision_time_surface_periodic_group_track.cpp:201-537
// (the "Luenberger observer" of the README is this fixed-gain predictor-corrector: direction
// damping 0.8, velocity/direction blend 0.3, group-velocity blend 0.3).  It runs on the CPU
// once per 16384-event slice (:847), O(T*C) matching + O(T^2) grouping.
//
// MI355X design: the whole multi-slice update runs in ONE launch of one workgroup (the
// algorithm is sequential over slices and order-dependent inside one: greedy matching in track
// order, greedy grouping in seed order), so a batch of slices costs one kernel instead of one
// host round trip each.  A slice's working set (detections, predictions, match states, the
// grouping candidates) lives in LDS, so the per-track state is read and written once per
// slice; matching runs as parallel conflict-free rounds that provably reproduce the greedy
// order (see tracker_kernel), update + erase + append is one block-scan pass, and only the
// grouping's ordered sums stay sequential.  Every fp32 expression is written in the
// reference's operation order and compiled without FMA contraction, so positions,
// velocities and directions are bit-identical to oracle/oracle.cpp (std::pow(0.8f, i-1) is a
// host-side table, :254).
#include "ecc_internal.hpp"

#include <cmath>
#include <cstring>
#include <type_traits>
#include <vector>

#ifndef ECC_TRACKER_PROFILE
#define ECC_TRACKER_PROFILE 0
#endif

namespace {

#if ECC_TRACKER_PROFILE
// wall-clock ticks per phase (thread 0, after the phase's barrier) + matching rounds
__device__ unsigned long long g_trk_prof[16];
#define TRK_MARK(k)                                                  \
    do {                                                             \
        const unsigned long long now_ = wall_clock64();              \
        prof[k] += now_ - last_;                                     \
        last_ = now_;                                                \
    } while (0)
#else
#define TRK_MARK(k) do { } while (0)
#endif

constexpr int kNT = 512;                         // one workgroup of 8 waves (2 per SIMD)
constexpr int kH = ECC_TRACK_HIST_MAX;
constexpr int kMaxTrk = ECC_TRACKER_MAX_TRACKS;  // active tracks of a slice held in LDS
constexpr int kMaxDet = ECC_TRACKER_MAX_DETECTIONS;

struct DevTrack {
    int x, y, label, frame_count, is_matched, fsld, hist_len;
    int hx[kH], hy[kH];
    float vx, vy, dcx, dcy, dtx, dty;
    int group_id;
};

struct DevGroup {
    int id, n_labels, first_label_offset;
    float avx, avy, cx, cy, radius;
};

struct TrackerCounters {
    int32_t n_tracks, next_label, cur, n_groups, n_group_labels, err;
    int32_t resume;  // first slice of the launch left to tracker_kernel (tracker_fast_kernel stopped there)
    int32_t pad1;
};

struct TrackerParams {
    float max_distance, damping, smoothing, group_radius;
    int max_frames, history, frames_to_skip;
    float pow_tab[kH + 1];
    // Squared-distance thresholds equivalent to the reference's sqrt comparisons (sqrt_rn is
    // monotone): sqrt_rn(s) < max_distance <=> s < s_match, sqrt_rn(s) <= group_radius <=>
    // s <= s_group, for s = dx*dx + dy*dy rounded as in dist().
    float s_match, s_group;
};

// Host: smallest float s >= 0 with pred(sqrtf(s)) false, by bisection over the (monotone)
// bit patterns of [0, +inf]; sqrtf is correctly rounded on the host, like sqrt_rn.
template <class Pred>
static float first_false(Pred pred) {
    uint32_t lo = 0u, hi = 0x7F800000u;  // pred(sqrt(+0)) .. +inf
    if (!pred(0.0f)) return 0.0f;
    float inf;
    std::memcpy(&inf, &hi, 4);
    if (pred(std::sqrt(inf))) return inf;
    while (hi - lo > 1u) {  // pred(sqrt(lo)) true, pred(sqrt(hi)) false
        const uint32_t mid = lo + (hi - lo) / 2;
        float f;
        std::memcpy(&f, &mid, 4);
        (pred(std::sqrt(f)) ? lo : hi) = mid;
    }
    float r;
    std::memcpy(&r, &hi, 4);
    return r;
}

struct F2 { float x, y; };
__device__ __forceinline__ F2 add(F2 a, F2 b) { return F2{__fadd_rn(a.x, b.x), __fadd_rn(a.y, b.y)}; }
__device__ __forceinline__ F2 mul(F2 a, float s) { return F2{__fmul_rn(a.x, s), __fmul_rn(a.y, s)}; }
__device__ __forceinline__ float dist(F2 a, F2 b) {  // :217-222
    const float dx = __fsub_rn(a.x, b.x), dy = __fsub_rn(a.y, b.y);
    return ecc::sqrt_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)));
}
__device__ __forceinline__ float dist2(F2 a, F2 b) {  // dist()'s radicand, same rounding
    const float dx = __fsub_rn(a.x, b.x), dy = __fsub_rn(a.y, b.y);
    return __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy));
}
__device__ __forceinline__ float norm(F2 a) {
    return ecc::sqrt_rn(__fadd_rn(__fmul_rn(a.x, a.x), __fmul_rn(a.y, a.y)));
}

__device__ __forceinline__ void push_hist(DevTrack &t, int history) {  // :224-231
#pragma unroll
    for (int k = kH - 1; k > 0; --k) { t.hx[k] = t.hx[k - 1]; t.hy[k] = t.hy[k - 1]; }
    t.hx[0] = t.x;
    t.hy[0] = t.y;
    t.hist_len = min(t.hist_len + 1, history);
}

__device__ __forceinline__ F2 calc_direction(const DevTrack &t, const TrackerParams &p) {  // :233-271
    if (t.hist_len < 2) return F2{0.f, 0.f};
    F2 w{0.f, 0.f};
    float total = 0.f;
#pragma unroll
    for (int i = 1; i < kH; ++i) {
        if (i < t.hist_len) {
            F2 d{(float)(t.hx[i - 1] - t.hx[i]), (float)(t.hy[i - 1] - t.hy[i])};
            const float mag = norm(d);
            if (mag > 0.f) {
                d = mul(d, __fdiv_rn(1.0f, mag));
                const float wt = p.pow_tab[i - 1];
                w = add(w, mul(d, wt));
                total = __fadd_rn(total, wt);
            }
        }
    }
    if (total > 0.f) {
        w = mul(w, __fdiv_rn(1.0f, total));
        const float mag = norm(w);
        if (mag > 0.f) w = mul(w, __fdiv_rn(1.0f, mag));
    }
    return w;
}

__device__ __forceinline__ F2 estimate_velocity(const DevTrack &t, const TrackerParams &p) {  // :273-302
    if (t.hist_len < 2) return F2{0.f, 0.f};
    F2 tot{0.f, 0.f};
    int count = 0;
#pragma unroll
    for (int i = 1; i < kH; ++i) {
        if (i < t.hist_len) {
            tot = add(tot, F2{(float)(t.hx[i - 1] - t.hx[i]), (float)(t.hy[i - 1] - t.hy[i])});
            count++;
        }
    }
    const F2 avg = count > 0 ? mul(tot, __fdiv_rn(1.0f, (float)count)) : F2{0.f, 0.f};
    const float speed = norm(avg);
    if (speed > 0.f) {
        const F2 dv = mul(F2{t.dcx, t.dcy}, speed);
        return add(mul(avg, __fsub_rn(1.0f, p.smoothing)), mul(dv, p.smoothing));
    }
    return avg;
}

__device__ __forceinline__ F2 predict(const DevTrack &t, const TrackerParams &p) {  // :304-319
    const F2 pos{(float)t.x, (float)t.y};
    F2 pred = add(pos, F2{t.vx, t.vy});
    if (t.fsld > 0) {
        const float conf = fmaxf(0.0f, __fsub_rn(1.0f, __fdiv_rn((float)t.fsld, (float)p.frames_to_skip)));
        const F2 dp = add(pos, mul(F2{t.dcx, t.dcy}, norm(F2{t.vx, t.vy})));
        pred = add(mul(pred, __fsub_rn(1.0f, conf)), mul(dp, conf));
    }
    return pred;
}

// ---- LDS plan.  A slice's working set lives in LDS, in distinct __shared__ arrays (so the
// compiler can keep loads of one in flight across atomics on another); an array is reused once
// its phase is over (P0 detections, P1 predictions, P2 matching rounds, P3 update/erase/append,
// P4 grouping).  Candidates (tracks with fsld == 0 after P3) each own a distinct detection, so
// there are at most C of them.
static_assert(kMaxTrk == kMaxDet, "ck_x/ck_y overlay the prediction arrays");
static_assert(kMaxTrk <= 4096, "track index packs into 12 bits of the matching tag");
static_assert(64 * 16 <= 2 * kMaxTrk, "member staging fits the st array");

// Detection grid for the matching scans: cells of kCell >= 2 * (max_distance + 1) + 2 pixels
// hashed into kBuckets buckets, so every detection a prediction can reach lies in at most 3 x 3
// cells.  Collisions only add candidates (the argmin is taken over (dist, index) explicitly).
constexpr int kBuckets = 512;
constexpr int kBrute = 384;
constexpr int kLaneList = 4;  // in-range detections a matching lane keeps in registers
constexpr int kTailCap = 1024; // candidate entries of the one-wave matching tail  // up to this many detections a scan walks all of them (uniform, no grid)  // per-track candidate list held in registers during the matching rounds
__device__ __forceinline__ int floor_div(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
__device__ __forceinline__ int cell_bucket(int cx, int cy) {
    return (int)(((uint32_t)cx * 0x9E3779B1u ^ (uint32_t)cy * 0x85EBCA77u) >> (32 - 9));
}
static_assert(kBuckets == 1 << 9, "bucket hash takes the top 9 bits");

// Exclusive scan of v[0..kBuckets) in place (one entry per thread); v[kBuckets] = total.
__device__ __forceinline__ void block_scan_buckets(int *v, int *ws) {
    static_assert(kBuckets == kNT, "one bucket per thread");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int a = v[threadIdx.x];
    int inc = a;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(inc, d);
        if (lane >= d) inc += o;
    }
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    int pre = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kNT / 64; ++w) {
        pre += w < wave ? ws[w] : 0;
        all += ws[w];
    }
    v[threadIdx.x] = pre + inc - a;
    if (threadIdx.x == 0) v[kBuckets] = all;
    __syncthreads();
}

// Compiler-only ordering point for wave-synchronous LDS exchanges (no hardware wait needed:
// one wave's LDS instructions execute in issue order).
__device__ __forceinline__ void wave_sync() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ uint64_t lanes_below() {
    const int lane = threadIdx.x & 63;
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Exclusive block-wide ranks of two per-thread flags (thread order); totals through *t0, *t1.
__device__ __forceinline__ void block_rank2(bool f0, bool f1, int *ws, int &r0, int &r1, int &t0, int &t1) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t m0 = __ballot(f0), m1 = __ballot(f1);
    if (lane == 0) {
        ws[wave] = __popcll(m0);
        ws[16 + wave] = __popcll(m1);
    }
    __syncthreads();
    int p0 = 0, p1 = 0;
    t0 = 0;
    t1 = 0;
#pragma unroll
    for (int w = 0; w < kNT / 64; ++w) {
        const int c0 = ws[w], c1 = ws[16 + w];
        p0 += w < wave ? c0 : 0;
        p1 += w < wave ? c1 : 0;
        t0 += c0;
        t1 += c1;
    }
    __syncthreads();  // ws reusable
    r0 = p0 + __popcll(m0 & lanes_below());
    r1 = p1 + __popcll(m1 & lanes_below());
}

// Track stores: a grouping candidate's vx, vy and group_id are written once, after grouping.
__device__ __forceinline__ void store_track(DevTrack *dst, const DevTrack &t, bool cand) {
    dst->x = t.x; dst->y = t.y; dst->label = t.label; dst->frame_count = t.frame_count;
    dst->is_matched = t.is_matched; dst->fsld = t.fsld; dst->hist_len = t.hist_len;
#pragma unroll
    for (int k = 0; k < kH; ++k) { dst->hx[k] = t.hx[k]; dst->hy[k] = t.hy[k]; }
    dst->dcx = t.dcx; dst->dcy = t.dcy; dst->dtx = t.dtx; dst->dty = t.dty;
    if (!cand) { dst->vx = t.vx; dst->vy = t.vy; dst->group_id = t.group_id; }
}

// P4 of one slice (wave 0 of the caller's workgroup; wave-synchronous: a wave's LDS operations
// execute in issue order, so only compiler reordering is fenced): greedy grouping in seed order
// over the G candidates staged in LDS (:321-398), then the velocity blend with the group
// average (:388-397) written to the candidates' tracks.  Only the average velocities feed the
// next slice; centroids, radii and the label lists (the getCornerGroups() view) are formed when
// `last` (the launch's last slice), since every slice overwrites them.
struct GroupLds {
    const int *ck_x, *ck_y, *ck_label;
    const int16_t *ck_tidx;
    const float *ck_vx, *ck_vy;
    int *ck_gid;
    uint8_t *ck_proc;
    float2 *gav;
    uint64_t *gmem;
    int *goff;
    float4 *stage;
    unsigned *rad;
};

// `put(new_index, vx, vy, group_id)` stores a candidate's blended velocity and group id: into the
// next global track list (tracker_kernel) or into the LDS-resident list (tracker_fast_kernel).
template <class Put>
__device__ __forceinline__ void group_slice(const GroupLds L, int G, bool last, const TrackerParams p, int max_tracks,
                                         Put &&put, DevGroup *__restrict__ groups, int *__restrict__ group_labels,
                                         int *n_groups_out, int *n_glabels_out, unsigned long long *gprof = nullptr) {
    const int lane = threadIdx.x & 63;
#if ECC_TRACKER_PROFILE
    unsigned long long g_last = wall_clock64();
#define GRP_MARK(k) do { if (gprof) { const unsigned long long n_ = wall_clock64(); gprof[k] += n_ - g_last; g_last = n_; } } while (0)
#else
#define GRP_MARK(k) do { } while (0)
#endif
    int n_groups = 0, n_glabels = 0;
    if (G <= 64) {
        // one candidate per lane, in registers: seed search and membership are ballots
        const bool valid = lane < G;
        const int mx = valid ? L.ck_x[lane] : 0, my = valid ? L.ck_y[lane] : 0;
        const float mvx = valid ? L.ck_vx[lane] : 0.f, mvy = valid ? L.ck_vy[lane] : 0.f;
        const int mtidx = valid ? L.ck_tidx[lane] : 0;
        int mgid = valid ? L.ck_gid[lane] : -1;
        bool proc = !valid;
        int next = 0;
        // phase A: seeds in order, each group's members (ballot) and label range
        for (;;) {
            const uint64_t open_ = __ballot(!proc && lane >= next);
            if (!open_) break;
            const int sl = __ffsll((unsigned long long)open_) - 1;
            next = sl + 1;
            const F2 pi{(float)__builtin_amdgcn_readlane(mx, sl), (float)__builtin_amdgcn_readlane(my, sl)};
            const bool mem = !proc && dist2(pi, F2{(float)mx, (float)my}) <= p.s_group;
            const uint64_t m = __ballot(mem);
            if (!m) continue;
            if (mem) {
                proc = true;
                mgid = n_groups;
                const int r = __popcll(m & lanes_below());
                if (last && n_glabels + r < max_tracks) group_labels[n_glabels + r] = L.ck_label[lane];
                // members in label order = candidate order: staged contiguously for phase B
                L.stage[n_glabels + r] = make_float4((float)mx, (float)my, mvx, mvy);
            }
            if (lane == 0) {
                L.gmem[n_groups] = m;
                L.goff[n_groups] = n_glabels;
            }
            n_glabels += __popcll(m);
            n_groups++;
        }
        wave_sync();
        GRP_MARK(0);
        // phase B: one lane per group (<= 64 groups): ordered fp32 sums over its members
        // (candidate order), streamed from their contiguous staging, eight loads ahead
        if (lane < n_groups) {
            const uint64_t m = L.gmem[lane];
            const int cnt = __popcll(m), off = L.goff[lane];
            F2 sp{0.f, 0.f}, sv{0.f, 0.f};
            for (int q = 0; q < cnt; q += 8) {
                float4 v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = L.stage[off + min(q + u, cnt - 1)];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    if (q + u >= cnt) break;
                    sv = add(sv, F2{v[u].z, v[u].w});
                    if (last) sp = add(sp, F2{v[u].x, v[u].y});
                }
            }
            const float inv = __fdiv_rn(1.0f, (float)cnt);
            const F2 av = mul(sv, inv);
            if (last) {
                const F2 cen = mul(sp, inv);
                float smax = 0.f;  // max over members of sqrt_rn(s) == sqrt_rn(max s) (monotone)
                for (uint64_t m2 = m; m2; m2 &= m2 - 1) {
                    const int k = __ffsll((unsigned long long)m2) - 1;
                    smax = fmaxf(smax, dist2(F2{(float)L.ck_x[k], (float)L.ck_y[k]}, cen));
                }
                if (lane < max_tracks)
                    groups[lane] = DevGroup{lane, cnt, L.goff[lane], av.x, av.y, cen.x, cen.y, ecc::sqrt_rn(smax)};
            }
            L.gav[lane] = make_float2(av.x, av.y);
        }
        wave_sync();
        GRP_MARK(1);
        // velocity blend with the group average (:388-397); candidates' last fields.  With
        // group_radius >= 0 every candidate joins a group this slice; otherwise none forms.
        if (valid) {
            float vx = mvx, vy = mvy;
            if (mgid >= 0 && mgid < n_groups) {
                const float2 g = L.gav[mgid];
                vx = __fadd_rn(__fmul_rn(vx, 0.7f), __fmul_rn(g.x, 0.3f));
                vy = __fadd_rn(__fmul_rn(vy, 0.7f), __fmul_rn(g.y, 0.3f));
            }
            put(mtidx, vx, vy, mgid);
        }
        GRP_MARK(2);
    } else {
        for (int k = lane; k < G; k += 64) L.ck_proc[k] = 0;
        wave_sync();
        int next = 0;
        for (;;) {
            int seed = -1;
            for (int b0 = next; b0 < G; b0 += 64) {
                const int k = b0 + lane;
                const uint64_t m = __ballot(k < G && !L.ck_proc[k]);
                if (m) {
                    seed = b0 + __ffsll((unsigned long long)m) - 1;
                    break;
                }
            }
            if (seed < 0) break;
            next = seed + 1;
            const F2 pi{(float)L.ck_x[seed], (float)L.ck_y[seed]};
            const int gid = n_groups;
            int cnt = 0;
            uint64_t mine = 0;  // bit c: this lane is a member in chunk c
            F2 sp{0.f, 0.f}, sv{0.f, 0.f};
            for (int b0 = 0, c = 0; b0 < G; b0 += 64, ++c) {
                const int k = b0 + lane;
                bool mem = false;
                if (k < G && !L.ck_proc[k]) mem = dist(pi, F2{(float)L.ck_x[k], (float)L.ck_y[k]}) <= p.group_radius;
                const uint64_t m = __ballot(mem);
                if (!m) continue;
                const int r = __popcll(m & lanes_below());
                if (mem) {
                    mine |= 1ull << c;
                    L.ck_proc[k] = 1;
                    L.ck_gid[k] = gid;
                    if (last && n_glabels + cnt + r < max_tracks) group_labels[n_glabels + cnt + r] = L.ck_label[k];
                    L.stage[r] = make_float4((float)L.ck_x[k], (float)L.ck_y[k], L.ck_vx[k], L.ck_vy[k]);
                }
                wave_sync();
                // ordered fp32 sums over the members (k ascending), evaluated by every lane
                const int nm = __popcll(m);
                int q = 0;
                for (; q + 4 <= nm; q += 4) {
                    const float4 v0 = L.stage[q], v1 = L.stage[q + 1], v2 = L.stage[q + 2], v3 = L.stage[q + 3];
                    sp = add(add(add(add(sp, F2{v0.x, v0.y}), F2{v1.x, v1.y}), F2{v2.x, v2.y}), F2{v3.x, v3.y});
                    sv = add(add(add(add(sv, F2{v0.z, v0.w}), F2{v1.z, v1.w}), F2{v2.z, v2.w}), F2{v3.z, v3.w});
                }
                for (; q < nm; ++q) {
                    const float4 v = L.stage[q];
                    sp = add(sp, F2{v.x, v.y});
                    sv = add(sv, F2{v.z, v.w});
                }
                cnt += nm;
                wave_sync();
            }
            if (cnt > 0) {
                const F2 av = mul(sv, __fdiv_rn(1.0f, (float)cnt));
                if (last) {
                    const F2 cen = mul(sp, __fdiv_rn(1.0f, (float)cnt));
                    // radius = max distance of the group's members to the centroid (fp32 >= 0
                    // orders like its bit pattern)
                    if (lane == 0) *L.rad = 0u;
                    wave_sync();
                    for (uint64_t mm = mine; mm; mm &= mm - 1) {
                        const int k = (__ffsll((unsigned long long)mm) - 1) * 64 + lane;
                        atomicMax(L.rad, __float_as_uint(dist(F2{(float)L.ck_x[k], (float)L.ck_y[k]}, cen)));
                    }
                    wave_sync();
                    const float mr = __uint_as_float(*L.rad);
                    if (lane == 0 && gid < max_tracks)
                        groups[gid] = DevGroup{gid, cnt, n_glabels, av.x, av.y, cen.x, cen.y, mr};
                }
                if (lane == 0) L.gav[gid] = make_float2(av.x, av.y);
                n_glabels += cnt;
                n_groups++;
            }
            wave_sync();
        }
        // velocity blend with the group average (:388-397); candidates' last fields
        for (int k = lane; k < G; k += 64) {
            const int gid = L.ck_gid[k];
            float vx = L.ck_vx[k], vy = L.ck_vy[k];
            if (gid >= 0 && gid < n_groups) {
                const float2 g = L.gav[gid];
                vx = __fadd_rn(__fmul_rn(vx, 0.7f), __fmul_rn(g.x, 0.3f));
                vy = __fadd_rn(__fmul_rn(vy, 0.7f), __fmul_rn(g.y, 0.3f));
            }
            put((int)L.ck_tidx[k], vx, vy, gid);
        }
    }
    *n_groups_out = n_groups;
    *n_glabels_out = n_glabels;
}

// One workgroup processes the slices in order (the algorithm is sequential over slices); inside
// a slice every phase is parallel over tracks / detections / candidates except the greedy
// grouping (wave 0).
//   P1  prediction per track (:451), is_matched reset (:438-441).
//   P2  greedy matching in track order (:446-487) as conflict-free rounds: every unresolved
//       track takes its nearest unclaimed detection with dist < max_distance (first minimum),
//       and keeps it iff no earlier unresolved track has that detection in range (the
//       smallest such track index per detection is an LDS atomicMin of a round-tagged key).
//       Earlier tracks can then never claim it, and the argmin over a shrinking set that
//       still holds it is unchanged, so the result equals the sequential loop; the first
//       unresolved track always resolves, so rounds terminate.
//   P3  matched / missed update (:471-497), new tracks for unmatched detections in detection
//       order (:501-514) and the stable erase (:517-526) in one pass: kept tracks are written
//       to the other buffer at their block-scan rank; candidates (fsld == 0) are listed in LDS.
//   P4  greedy grouping in seed order over the candidates (:321-398) with ordered fp32 sums,
//       then the group-velocity blend (:388-397).
__global__ void __launch_bounds__(kNT)
tracker_kernel(DevTrack *buf0, DevTrack *buf1, int max_tracks, DevGroup *__restrict__ groups,
               int *__restrict__ group_labels, TrackerCounters *__restrict__ ctr, TrackerParams p,
               const ecc_corner *__restrict__ corners, const int64_t *__restrict__ starts,
               const int32_t *__restrict__ counts, int n_slices, int cap) {
    __shared__ int2 s_det[kMaxDet + 4];              // P0-P3 detections; P4 group average velocity
    __shared__ uint32_t s_claim[kMaxDet / 32];       // P0-P3 claimed detections (bits)
    __shared__ int s_want[kMaxDet];                  // P2 matching tags; P3-P4 candidate label
    __shared__ float s_px[kMaxTrk], s_py[kMaxTrk];   // P1-P2 predictions; P3-P4 candidate x, y
    __shared__ __attribute__((aligned(16))) int16_t s_st[kMaxTrk];  // P1-P3 match state; P4 member staging
    __shared__ __attribute__((aligned(16))) float s_cv[2 * kMaxDet];  // P3-P4 candidate velocity; P0-P2 grid entries
    __shared__ __attribute__((aligned(16))) int16_t s_ctidx[kMaxDet];  // candidate's index in the new list; P0-P2 bucket ends
    __shared__ int s_cgid[kMaxDet];                  // candidate's group id (stale until grouped)
    __shared__ uint8_t s_cproc[kMaxDet];             // grouped
    __shared__ int s_ws[32];                         // wave counts
    __shared__ unsigned s_rad;                       // group radius (fp32 bits, >= 0)
    __shared__ int s_tail[2];                        // matching tail: list cursor, overflow
    __shared__ uint64_t s_gmem[64];                  // grouping (<= 64 candidates): member masks
    __shared__ int s_goff[64];                       //   and first label offsets
    __shared__ int16_t t_trk[64], t_off[64], t_n[64];
    __shared__ int16_t t_d[kTailCap];
    __shared__ float t_dd[kTailCap];
    int2 *const det = s_det;
    float2 *const gav = reinterpret_cast<float2 *>(s_det);
    uint32_t *const claim = s_claim;
    int *const want = s_want, *const ck_label = s_want;
    float *const px = s_px, *const py = s_py;
    int *const ck_x = reinterpret_cast<int *>(s_px), *const ck_y = reinterpret_cast<int *>(s_py);
    int16_t *const st = s_st;
    float4 *const stage = reinterpret_cast<float4 *>(s_st);
    float *const ck_vx = s_cv, *const ck_vy = s_cv + kMaxDet;
    int16_t *const ck_tidx = s_ctidx;
    int *const ck_gid = s_cgid;
    uint8_t *const ck_proc = s_cproc;
    int *const ws = s_ws;
    // grid entries {x | y << 16 (int16 each), index} by bucket; g_end[b] = end of bucket b
    uint2 *const g_ent = reinterpret_cast<uint2 *>(s_cv);
    int *const g_end = reinterpret_cast<int *>(s_ctidx);
    static_assert(sizeof(uint2) * kMaxDet <= sizeof(s_cv), "grid entries fit s_cv");
    static_assert((kBuckets + 1) * sizeof(int) <= sizeof(s_ctidx), "bucket ends fit s_ctidx");

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // |dx| or |dy| above max_distance + 1 cannot give dist < max_distance (for sane radii)
    const float reach = __fadd_rn(p.max_distance, 1.0f);
    // grid matching for sane radii; otherwise every scan walks all detections
    const bool grid_ok = p.max_distance >= 0.0f && p.max_distance < 1.0e5f;
    const int cell = grid_ok ? (int)ceilf(reach) + 1 : 1;
    const int s0 = ctr->resume;  // slices before it were processed by tracker_fast_kernel
    if (s0 >= n_slices) return;
    int T = ctr->n_tracks, next_label = ctr->next_label, cur = ctr->cur, err = ctr->err;
    int n_groups = 0, n_glabels = 0;
#if ECC_TRACKER_PROFILE
    unsigned long long prof[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, last_ = wall_clock64();
    const unsigned long long c0_ = clock64(), w0_ = last_;
#endif
    for (int s = s0; s < n_slices; ++s) {
        DevTrack *A = cur ? buf1 : buf0;   // active tracks
        DevTrack *Bf = cur ? buf0 : buf1;  // next active list
        int C = counts[s];
        if (C > cap) { C = cap; err = ECC_ERR_CAPACITY; }  // beyond max_detections: dropped, reported
        if (C < 0) C = 0;
        const int64_t first = starts ? starts[s] : (int64_t)s * cap;  // slice s = corners[first, first + C)
        // P0: detections
        bool wide = false;  // a coordinate outside int16: this slice scans without the grid
        for (int d = tid; d < C; d += kNT) {
            const ecc_corner c = corners[first + d];
            det[d] = make_int2(c.x, c.y);
            want[d] = 0x7fffffff;
            wide |= c.x < -32768 || c.x > 32767 || c.y < -32768 || c.y > 32767;
        }
        for (int w = tid; w < (C + 31) / 32; w += kNT) claim[w] = 0u;
        const bool any_wide = __syncthreads_or(wide);
        const bool use_grid = grid_ok && C > kBrute && !any_wide;
        if (use_grid) {
            for (int b = tid; b <= kBuckets; b += kNT) g_end[b] = 0;
            __syncthreads();
            for (int d = tid; d < C; d += kNT) {
                const int2 q = det[d];
                atomicAdd(&g_end[cell_bucket(floor_div(q.x, cell), floor_div(q.y, cell))], 1);
            }
        }
        // P1: predictions
        bool open = false;
        for (int i = tid; i < T; i += kNT) {
            const DevTrack &t = A[i];
            DevTrack q;
            q.x = t.x; q.y = t.y; q.vx = t.vx; q.vy = t.vy; q.dcx = t.dcx; q.dcy = t.dcy; q.fsld = t.fsld;
            const F2 pp = predict(q, p);
            px[i] = pp.x;
            py[i] = pp.y;
            const bool skip = q.fsld > p.frames_to_skip;
            st[i] = skip ? (int16_t)-2 : (int16_t)-3;
            open |= !skip;
        }
        // P2: matching rounds
        int round = 0;
        bool pending = __syncthreads_or(open) && C > 0;
        if (use_grid && pending) {
            TRK_MARK(0);
            block_scan_buckets(g_end, ws);  // bucket starts
            for (int d = tid; d < C; d += kNT) {  // scatter; afterwards g_end[b] = end of bucket b
                const int2 q = det[d];
                const int at = atomicAdd(&g_end[cell_bucket(floor_div(q.x, cell), floor_div(q.y, cell))], 1);
                g_ent[at] = make_uint2(((uint32_t)q.x & 0xFFFFu) | ((uint32_t)q.y << 16), (uint32_t)d);
            }
            __syncthreads();
        }
        TRK_MARK(7);
        if (C == 0)
            for (int i = tid; i < T; i += kNT)
                if (st[i] == -3) st[i] = -1;
        // Grid visitor (large C, one lane per track): f(d, dd) for every unclaimed detection with
        // dist < max_distance from the prediction pp.
        auto visit_grid = [&](const F2 pp, bool check_claims, auto &&f) {
            // the cells of the integer box [pp - reach, pp + reach]: at most 3 x 3
            const int cx0 = floor_div((int)floorf(__fsub_rn(pp.x, reach)), cell);
            const int cx1 = floor_div((int)ceilf(__fadd_rn(pp.x, reach)), cell);
            const int cy0 = floor_div((int)floorf(__fsub_rn(pp.y, reach)), cell);
            const int cy1 = floor_div((int)ceilf(__fadd_rn(pp.y, reach)), cell);
            int seen[9], ns = 0;
            for (int cy = cy0; cy <= cy1; ++cy)
                for (int cx = cx0; cx <= cx1; ++cx) {
                    const int b = cell_bucket(cx, cy);
                    bool dup = false;
                    for (int k = 0; k < ns; ++k) dup |= seen[k] == b;  // hash collision
                    if (dup) continue;
                    seen[ns++] = b;
                    const int e1 = g_end[b];
                    for (int e = b ? g_end[b - 1] : 0; e < e1; ++e) {
                        const uint2 g = g_ent[e];
                        const F2 dq{(float)(int16_t)(g.x & 0xFFFFu), (float)(int16_t)(g.x >> 16)};
                        if (!(dist2(pp, dq) < p.s_match)) continue;
                        const int d = (int)g.y;
                        if (check_claims && ((claim[d >> 5] >> (d & 31)) & 1u)) continue;
                        f(d, dist(pp, dq));
                    }
                }
        };
        // L lanes per track (a power of two, T * L <= kNT): lane jl of a track's group scans
        // detections jl, jl + L, ...; the group combines its (dist, index) minima with shuffles.
        int L = 1;
        if (!use_grid)
            while (L < 64 && T * L * 2 <= kNT) L <<= 1;
        const int jl = tid & (L - 1);
        // Each lane's in-range detections of the first round stay in registers (the lane owns one
        // track when T * L <= kNT), so later rounds only re-check claims; a lane with more than
        // kLaneList of them rescans its share instead.
        const bool lists_ok = T <= kNT / L;
        float l_d[kLaneList];
        int l_i[kLaneList];
        int l_n = 0;
        bool l_ovf = false;
        while (pending) {
            const int tag = (8191 - round) << 12;
            for (int i = tid / L; i < T; i += kNT / L) {
                if (st[i] != -3) continue;  // uniform over the lane group
                float bd = p.max_distance;
                int bi = -1;
                auto take = [&](int d, float dd) {
                    atomicMin(&want[d], tag | i);
                    // first minimum in detection order == smallest (dist, index)
                    if (bi < 0 || dd < bd || (dd == bd && d < bi)) { bd = dd; bi = d; }
                };
                if (lists_ok && round > 0 && !l_ovf) {
#pragma unroll
                    for (int k = 0; k < kLaneList; ++k)
                        if (k < l_n && !((claim[l_i[k] >> 5] >> (l_i[k] & 31)) & 1u)) take(l_i[k], l_d[k]);
                } else {
                    const F2 pp{px[i], py[i]};
                    const bool record = lists_ok && round == 0;
                    auto take_rec = [&](int d, float dd) {
                        take(d, dd);
                        if (record) {
#pragma unroll
                            for (int k = 0; k < kLaneList; ++k)
                                if (k == l_n) { l_d[k] = dd; l_i[k] = d; }
                            l_ovf |= l_n == kLaneList;
                            l_n += l_n < kLaneList ? 1 : 0;
                        }
                    };
                    if (use_grid && fabsf(pp.x) < 1.0e9f && fabsf(pp.y) < 1.0e9f) {
                        visit_grid(pp, round > 0, take_rec);
                    } else {
                        for (int d = jl; d < C; d += L) {
                            if (round > 0 && ((claim[d >> 5] >> (d & 31)) & 1u)) continue;
                            const int2 q = det[d];
                            const F2 dq{(float)q.x, (float)q.y};
                            // in range iff the squared distance is below s_match; sqrt only then
                            if (dist2(pp, dq) < p.s_match) take_rec(d, dist(pp, dq));
                        }
                    }
                }
                for (int o = L >> 1; o > 0; o >>= 1) {
                    const float od = __shfl_xor(bd, o);
                    const int oi = __shfl_xor(bi, o);
                    if (oi >= 0 && (bi < 0 || od < bd || (od == bd && oi < bi))) { bd = od; bi = oi; }
                }
                if (jl == 0) st[i] = bi < 0 ? (int16_t)-1 : (int16_t)(-4 - bi);
            }
            __syncthreads();
            if (round == 0) TRK_MARK(8); else TRK_MARK(1);
            bool again = false;
            for (int i = tid; i < T; i += kNT) {
                const int sv = st[i];
                if (sv > -4) continue;
                const int b = -4 - sv;
                if (want[b] == (tag | i)) {
                    st[i] = (int16_t)b;
                    atomicOr(&claim[b >> 5], 1u << (b & 31));
                } else {
                    st[i] = -3;
                    again = true;
                }
            }
            ++round;
            pending = __syncthreads_or(again);
            TRK_MARK(5);
            if (pending && round == 1 && lists_ok) {
                // Tail: the tracks still unresolved (typically few) finish in one wave, without
                // workgroup barriers.  Each track's lane group moves its register lists to LDS.
                const int i = tid / L;
                const bool unres = i < T && st[i] == -3;
                int gn = unres ? l_n : 0, ex = gn;
                int govf = unres && l_ovf ? 1 : 0;
                for (int o = 1; o < L; o <<= 1) {  // inclusive prefix of the list sizes in the group
                    const int v = __shfl_up(ex, o, L);
                    if (jl >= o) ex += v;
                }
                const int gtot = __shfl(ex, (lane & ~(L - 1)) + L - 1);
                ex -= gn;
                for (int o = L >> 1; o > 0; o >>= 1) govf |= __shfl_xor(govf, o);
                const bool head = unres && jl == 0;
                if (tid == 0) { s_tail[0] = 0; s_tail[1] = 0; }
                int u, u_unused, n_unres, n_unused;
                block_rank2(head, false, ws, u, u_unused, n_unres, n_unused);  // also orders the reset
                int off = 0;
                if (head) {
                    off = atomicAdd(&s_tail[0], gtot);
                    if (govf) atomicOr(&s_tail[1], 1);
                }
                off = __shfl(off, lane & ~(L - 1));
                __syncthreads();
                const bool tail_ok = n_unres <= 64 && s_tail[1] == 0 && s_tail[0] <= kTailCap;
                if (tail_ok) {
                    if (head) {
                        t_trk[u] = (int16_t)i;
                        t_off[u] = (int16_t)off;
                        t_n[u] = (int16_t)gtot;
                    }
                    if (unres) {
#pragma unroll
                        for (int k = 0; k < kLaneList; ++k)
                            if (k < l_n) {
                                t_d[off + ex + k] = (int16_t)l_i[k];
                                t_dd[off + ex + k] = l_d[k];
                            }
                    }
                    __syncthreads();
                    if (wave == 0) {
                        const bool act = lane < n_unres;
                        const int ti = act ? t_trk[lane] : 0, to = act ? t_off[lane] : 0, tn = act ? t_n[lane] : 0;
                        bool done = !act;
                        int r = round;
                        while (__ballot(!done)) {
                            const int tag = (8191 - r) << 12;
                            float bd = 0.f;
                            int bi = -1;
                            if (!done)
                                for (int k = 0; k < tn; ++k) {
                                    const int d = t_d[to + k];
                                    if ((claim[d >> 5] >> (d & 31)) & 1u) continue;
                                    atomicMin(&want[d], tag | ti);
                                    const float dd = t_dd[to + k];
                                    if (bi < 0 || dd < bd || (dd == bd && d < bi)) { bd = dd; bi = d; }
                                }
                            wave_sync();
                            if (!done) {
                                if (bi < 0) {
                                    st[ti] = -1;
                                    done = true;
                                } else if (want[bi] == (tag | ti)) {
                                    st[ti] = (int16_t)bi;
                                    atomicOr(&claim[bi >> 5], 1u << (bi & 31));
                                    done = true;
                                }
                            }
                            wave_sync();
                            ++r;
                        }
#if ECC_TRACKER_PROFILE
                        prof[9] += r - round;
#endif
                    }
                    pending = false;
                }
            }
        }
        __syncthreads();
        TRK_MARK(1);
#if ECC_TRACKER_PROFILE
        prof[6] += round;
#endif
        // P3: update, erase, append
        int T2 = 0, G = 0;
        for (int base = 0; base < T; base += kNT) {
            const int i = base + tid;
            DevTrack t;
            bool keep = false, cand = false;
            if (i < T) {
                t = A[i];
                const int sv = st[i];
                t.is_matched = 0;
                if (sv >= 0) {  // matched (:471-485)
                    t.x = det[sv].x;
                    t.y = det[sv].y;
                    t.is_matched = 1;
                    t.fsld = 0;
                    t.frame_count++;
                    push_hist(t, p.history);
                    const F2 nd = calc_direction(t, p);
                    t.dtx = nd.x;                                          // DirectionVector::update
                    t.dty = nd.y;
                    t.dcx = __fadd_rn(__fmul_rn(t.dcx, p.damping), __fmul_rn(t.dtx, __fsub_rn(1.0f, p.damping)));
                    t.dcy = __fadd_rn(__fmul_rn(t.dcy, p.damping), __fmul_rn(t.dty, __fsub_rn(1.0f, p.damping)));
                    const F2 v = estimate_velocity(t, p);
                    t.vx = v.x;
                    t.vy = v.y;
                } else if (sv == -1) {  // missed (:488-497): move to the prediction
                    const F2 pp = predict(t, p);
                    t.x = (int)pp.x;                                       // Q16 truncation
                    t.y = (int)pp.y;
                    t.fsld++;
                    push_hist(t, p.history);
                    const F2 v = estimate_velocity(t, p);
                    t.vx = v.x;
                    t.vy = v.y;
                }
                keep = !(t.fsld > p.frames_to_skip || t.frame_count > p.max_frames);
                cand = keep && t.fsld == 0;
            }
            int rk, rc, tk, tc;
            block_rank2(keep, cand, ws, rk, rc, tk, tc);
            if (keep) store_track(Bf + T2 + rk, t, cand);
            if (cand) {
                const int k = G + rc;
                ck_x[k] = t.x;
                ck_y[k] = t.y;
                ck_vx[k] = t.vx;
                ck_vy[k] = t.vy;
                ck_label[k] = t.label;
                ck_tidx[k] = (int16_t)(T2 + rk);
                ck_gid[k] = t.group_id;
            }
            T2 += tk;
            G += tc;
        }
        TRK_MARK(2);
        // new tracks for the unmatched detections, in detection order; slots past max_tracks
        // (counted before the erase, like the reference's append-then-erase) are dropped
        const int room = max_tracks - T;
        const bool keep_new = !(0 > p.frames_to_skip || 1 > p.max_frames);
        int n_unm = 0;
        for (int base = 0; base < C; base += kNT) {
            const int d = base + tid;
            const bool un = d < C && !((claim[d >> 5] >> (d & 31)) & 1u);
            int r, r_unused, tot, tot_unused;
            block_rank2(un, false, ws, r, r_unused, tot, tot_unused);
            r += n_unm;
            if (un) {
                if (r < room) {
                    if (keep_new) {
                        DevTrack t;
                        t.x = det[d].x;
                        t.y = det[d].y;
                        t.label = next_label + r;
                        t.frame_count = 1;
                        t.is_matched = 0;
                        t.fsld = 0;
                        t.hist_len = 0;
#pragma unroll
                        for (int k = 0; k < kH; ++k) { t.hx[k] = 0; t.hy[k] = 0; }
                        push_hist(t, p.history);
                        t.vx = t.vy = 0.f;
                        t.dcx = t.dcy = t.dtx = t.dty = 0.f;
                        t.group_id = -1;                                   // Q17
                        store_track(Bf + T2 + r, t, true);
                        const int k = G + r;
                        ck_x[k] = t.x;
                        ck_y[k] = t.y;
                        ck_vx[k] = 0.f;
                        ck_vy[k] = 0.f;
                        ck_label[k] = t.label;
                        ck_tidx[k] = (int16_t)(T2 + r);
                        ck_gid[k] = -1;
                    }
                } else {
                    err = ECC_ERR_CAPACITY;
                }
            }
            n_unm += tot;
        }
        next_label += n_unm;
        const int added = room > 0 ? min(n_unm, room) : 0;
        if (keep_new) {
            T2 += added;
            G += added;
        }
        T = T2;
        cur ^= 1;
        __syncthreads();
        TRK_MARK(3);
        // P4: greedy grouping in seed order over the candidates, then the velocity blend (wave 0)
        if (wave == 0)
            group_slice(GroupLds{ck_x, ck_y, ck_label, ck_tidx, ck_vx, ck_vy, ck_gid, ck_proc, gav,
                                 s_gmem, s_goff, stage, &s_rad},
                        G, s == n_slices - 1, p, max_tracks,
                        [Bf](int k, float vx, float vy, int gid) {
                            DevTrack *dst = Bf + k;
                            dst->vx = vx;
                            dst->vy = vy;
                            dst->group_id = gid;
                        },
                        groups, group_labels, &n_groups, &n_glabels
                        );
        __syncthreads();
        TRK_MARK(4);
    }
#if ECC_TRACKER_PROFILE
    prof[10] = clock64() - c0_;
    prof[11] = wall_clock64() - w0_;
    if (tid == 0)
        for (int k = 0; k < 12; ++k) g_trk_prof[k] = prof[k];
#endif
    const bool any_err = __syncthreads_or(err != 0);
    if (tid == 0) {
        if (any_err && err == 0) err = ECC_ERR_CAPACITY;
        ctr->n_tracks = T;
        ctr->next_label = next_label;
        ctr->cur = cur;
        ctr->n_groups = n_groups;
        ctr->n_group_labels = n_glabels;
        ctr->err = err;
    }
}


// ---- tracker_fast_kernel: the slice loop with every track in a register file --------------------
// The common regime (tens of tracks and detections per slice) is bound by latency, not work: the
// 512-lane kernel above spends most of a slice on global round trips (its track list lives in
// HBM between phases) and on workgroup barriers.  Here one 256-lane workgroup (one wave per
// SIMD) keeps track i in the registers of thread i for the whole launch; a slice moves the list
// through LDS only to apply the stable erase, detections are prefetched one slice ahead, and the
// matching rounds read the in-range detections each track found in its first scan from
// registers.  The arithmetic, the matching rule and the grouping are tracker_kernel's (same
// helpers, same operation order), so the state is bit-identical.  A slice with T + C > 256
// (tracks + detections) hands the rest of the launch to tracker_kernel: the list is written to
// the current buffer and ctr->resume = that slice.
// Quad permutes by DPP (quad_perm: lane i of each quad reads lane sel[i] of it).
template <int kCtrl>
__device__ __forceinline__ int qperm(int v) { return __builtin_amdgcn_mov_dpp(v, kCtrl, 0xf, 0xf, false); }
template <int kCtrl>
__device__ __forceinline__ float qperm_f(float v) { return __int_as_float(qperm<kCtrl>(__float_as_int(v))); }

constexpr int kFT = 256;    // the largest T + C of a slice handled here (LDS arrays)
constexpr int kFThreads = 512;  // 8 waves: the round-0 scan runs 2-4 lanes per track
constexpr int kFW = kFThreads / 64;
constexpr int kFList = 8;   // in-range detections a track keeps in registers (more: it rescans)
constexpr int kFTagTop = (1 << 23) - 1;  // round tags: ((kFTagTop - round) << 8) | track
static_assert(kFT <= 256, "track index packs into 8 bits of the matching tag");

struct FastList {  // the track list, structure of arrays (conflict-free LDS)
    int x[kFT], y[kFT], label[kFT], frame_count[kFT], is_matched[kFT], fsld[kFT], hist_len[kFT];
    int hx[kH][kFT], hy[kH][kFT];
    float vx[kFT], vy[kFT], dcx[kFT], dcy[kFT], dtx[kFT], dty[kFT];
    int group_id[kFT];
    float ux[kH][kFT], uy[kH][kFT];  // direction cache (FastTrack)
    uint32_t um[kFT];
};

// A track plus its direction cache: u[i] = the normalised step h[i-1] - h[i] of its history and
// bit i of um = that step is non-zero (calc_direction's `magnitude > 0`, :250).  A step's unit
// vector depends only on its integer difference, so after push_hist the old u[i-1] is the new
// u[i] bit for bit and only u[1] is computed; calc_direction then sums the cached terms in its
// own order (one sqrt + one divide per slice instead of one per history step).
struct FastTrack {
    DevTrack t;
    float ux[kH], uy[kH];
    uint32_t um;
};

__device__ __forceinline__ void unit_step(const DevTrack &t, int i, float &ux, float &uy, bool &nz) {  // :244-252
    F2 d{(float)(t.hx[i - 1] - t.hx[i]), (float)(t.hy[i - 1] - t.hy[i])};
    const float mag = norm(d);
    nz = mag > 0.f;
    d = mul(d, __fdiv_rn(1.0f, mag));
    ux = d.x;
    uy = d.y;
}

__device__ __forceinline__ void cache_all(FastTrack &f) {
    f.um = 0u;
    f.ux[0] = f.uy[0] = 0.f;
#pragma unroll
    for (int i = 1; i < kH; ++i) {
        bool nz;
        unit_step(f.t, i, f.ux[i], f.uy[i], nz);
        f.um |= nz ? (1u << i) : 0u;
    }
}

// push_hist + the cache shift + the new step u[1]
__device__ __forceinline__ void push_hist_cached(FastTrack &f, int history) {
    push_hist(f.t, history);
#pragma unroll
    for (int i = kH - 1; i > 1; --i) { f.ux[i] = f.ux[i - 1]; f.uy[i] = f.uy[i - 1]; }
    bool nz;
    unit_step(f.t, 1, f.ux[1], f.uy[1], nz);
    f.um = ((f.um << 1) & ~3u) | (nz ? 2u : 0u);
}

__device__ __forceinline__ F2 calc_direction_cached(const FastTrack &f, const TrackerParams &p) {  // :233-271
    if (f.t.hist_len < 2) return F2{0.f, 0.f};
    F2 w{0.f, 0.f};
    float total = 0.f;
#pragma unroll
    for (int i = 1; i < kH; ++i) {
        if (i < f.t.hist_len && ((f.um >> i) & 1u)) {
            const float wt = p.pow_tab[i - 1];
            w = add(w, mul(F2{f.ux[i], f.uy[i]}, wt));
            total = __fadd_rn(total, wt);
        }
    }
    if (total > 0.f) {
        w = mul(w, __fdiv_rn(1.0f, total));
        const float mag = norm(w);
        if (mag > 0.f) w = mul(w, __fdiv_rn(1.0f, mag));
    }
    return w;
}

__device__ __forceinline__ void fast_put(FastList &L, int k, const FastTrack &f) {
    const DevTrack &t = f.t;
#pragma unroll
    for (int h = 0; h < kH; ++h) { L.ux[h][k] = f.ux[h]; L.uy[h][k] = f.uy[h]; }
    L.um[k] = f.um;
    L.x[k] = t.x; L.y[k] = t.y; L.label[k] = t.label; L.frame_count[k] = t.frame_count;
    L.is_matched[k] = t.is_matched; L.fsld[k] = t.fsld; L.hist_len[k] = t.hist_len;
#pragma unroll
    for (int h = 0; h < kH; ++h) { L.hx[h][k] = t.hx[h]; L.hy[h][k] = t.hy[h]; }
    L.vx[k] = t.vx; L.vy[k] = t.vy; L.dcx[k] = t.dcx; L.dcy[k] = t.dcy; L.dtx[k] = t.dtx; L.dty[k] = t.dty;
    L.group_id[k] = t.group_id;
}

__device__ __forceinline__ FastTrack fast_get(const FastList &L, int k) {
    FastTrack f;
#pragma unroll
    for (int h = 0; h < kH; ++h) { f.ux[h] = L.ux[h][k]; f.uy[h] = L.uy[h][k]; }
    f.um = L.um[k];
    DevTrack &t = f.t;
    t.x = L.x[k]; t.y = L.y[k]; t.label = L.label[k]; t.frame_count = L.frame_count[k];
    t.is_matched = L.is_matched[k]; t.fsld = L.fsld[k]; t.hist_len = L.hist_len[k];
#pragma unroll
    for (int h = 0; h < kH; ++h) { t.hx[h] = L.hx[h][k]; t.hy[h] = L.hy[h][k]; }
    t.vx = L.vx[k]; t.vy = L.vy[k]; t.dcx = L.dcx[k]; t.dcy = L.dcy[k]; t.dtx = L.dtx[k]; t.dty = L.dty[k];
    t.group_id = L.group_id[k];
    return f;
}

__global__ void __launch_bounds__(kFThreads)
tracker_fast_kernel(DevTrack *buf0, DevTrack *buf1, int max_tracks, DevGroup *__restrict__ groups,
                    int *__restrict__ group_labels, TrackerCounters *__restrict__ ctr, TrackerParams p,
                    const ecc_corner *__restrict__ corners, const int64_t *__restrict__ starts,
                    const int32_t *__restrict__ counts, int n_slices, int cap) {
    __shared__ FastList L;                     // next track list (P3), velocities blended in P4
    FastList *const Lp = &L;
    __shared__ int2 f_det[kFT];
    __shared__ float2 f_detf[kFT + 32];         // as floats (+32: a scan chunk never reads past it)
    __shared__ int16_t f_li[kFList][kFThreads];  // a round-0 lane's in-range detections
    __shared__ float f_ld[kFList][kFThreads];    // and their distances
    __shared__ int16_t f_mi[kFList][kFT];       // a track's in-range detections (merged over its lanes)
    __shared__ float f_md[kFList][kFT];
    __shared__ int8_t f_mn[kFT];                // their number (-1: more than kFList, rescan)
    __shared__ int16_t f_best[kFT];             // round 0's choice of track i
    __shared__ float2 f_pp[kFT];                // predictions
    __shared__ int8_t f_st[kFT];                // P1 states
    __shared__ int16_t f_tail[64];              // matching tail: the unresolved tracks, in order
    __shared__ int16_t f_res[kFT];              //   and their results
    __shared__ int f_want[kFT + 1];             // [kFT]: sink of the tail's masked-off atomics
    __shared__ uint8_t f_claim[kFT + 1];        // [kFT]: always claimed
    __shared__ int f_ws[3 * kFW];
    __shared__ int ck_x[kFT], ck_y[kFT], ck_label[kFT], ck_gid[kFT];
    __shared__ int16_t ck_tidx[kFT];
    __shared__ float ck_vx[kFT], ck_vy[kFT];
    __shared__ uint8_t ck_proc[kFT];
    __shared__ float2 gav[kFT];
    __shared__ uint64_t gmem[64];
    __shared__ int goff[64];
    __shared__ float4 gstage[64];
    __shared__ unsigned grad;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int T = ctr->n_tracks, next_label = ctr->next_label, err = ctr->err;
    DevTrack *A = ctr->cur ? buf1 : buf0;
    int n_groups = 0, n_glabels = 0;
    if (T > kFT) {  // uniform: the whole launch is tracker_kernel's
        if (tid == 0) ctr->resume = 0;
        return;
    }
    FastTrack me;
    if (tid < T) {
        me.t = A[tid];
        cache_all(me);
    }
    if (tid == 0) f_claim[kFT] = 1;
    const int cload = min(cap, kFT);  // detections a slice handled here can have
    auto first_of = [&](int s) -> int64_t { return starts ? starts[s] : (int64_t)s * cap; };
    // detection prefetch: slice s's corner in (dnx, dny) of thread d; counts/starts of s + 1
    int dnx = 0, dny = 0;
    int c_cur = counts[0];
    {
        const int64_t f0 = first_of(0);
        if (tid < min(max(c_cur, 0), cload)) { dnx = corners[f0 + tid].x; dny = corners[f0 + tid].y; }
    }
    int c_nxt = n_slices > 1 ? counts[1] : 0;
    int64_t f_nxt = n_slices > 1 ? first_of(1) : 0;
    const bool keep_new = !(0 > p.frames_to_skip || 1 > p.max_frames);
    int stop = n_slices;
#if ECC_TRACKER_PROFILE
    unsigned long long prof[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, last_ = wall_clock64();
    const unsigned long long c0_ = clock64(), w0_ = last_;
#endif
    for (int s = 0; s < n_slices; ++s) {
        int C = c_cur;
        const bool over_cap = C > cap;
        if (over_cap) C = cap;
        if (C < 0) C = 0;
        if (T + C > kFT) { stop = s; break; }  // uniform
        if (over_cap) err = ECC_ERR_CAPACITY;   // beyond max_detections: dropped, reported
        // P0: detections, claims, matching tags; prefetch of the next slice
        if (tid < C) {
            f_det[tid] = make_int2(dnx, dny);
            f_detf[tid] = make_float2((float)dnx, (float)dny);
            f_want[tid] = 0x7fffffff;
            f_claim[tid] = 0;
        }
        int pnx = 0, pny = 0, c_nn = 0;
        int64_t f_nn = 0;
        if (s + 1 < n_slices && tid < min(max(c_nxt, 0), cload)) { pnx = corners[f_nxt + tid].x; pny = corners[f_nxt + tid].y; }
        if (s + 2 < n_slices) { c_nn = counts[s + 2]; f_nn = first_of(s + 2); }
        // P1: prediction (:451) of track tid; -2 skipped (or no track), -3 unresolved, -1 missed,
        // >= 0 matched
        int st = -2;
        F2 pp{0.f, 0.f};
        if (tid < T) {
            pp = predict(me.t, p);
            st = me.t.fsld > p.frames_to_skip ? -2 : (C == 0 ? -1 : -3);
            f_pp[tid] = make_float2(pp.x, pp.y);
            f_st[tid] = (int8_t)st;
        }
        __syncthreads();
        TRK_MARK(7);
        // P2 round 0 with L lanes per track: sub-lane tj scans the 32-detection chunks tj,
        // tj + L, ... as an unrolled in-range bit mask, then the mask's set bits four at a time
        // (their loads batched).  A track's choice, the first minimum of dist in detection
        // order, is the minimum of (dist, index) over its lanes; its in-range detections are
        // merged into one list (order irrelevant) for the later rounds.
        {
            const int lsh = T <= 128 ? 2 : 1;  // uniform: L = 1 << lsh, T * L <= kFThreads
            const int L = 1 << lsh;
            const int ti = tid >> lsh, tj = tid & (L - 1);
            const bool act = ti < T && f_st[ti] == -3;
            const float2 pq = ti < T ? f_pp[ti] : make_float2(0.f, 0.f);
            const F2 tp{pq.x, pq.y};
            const int tag0 = (kFTagTop << 8) | ti;
            int l_n = 0;
            bool l_ovf = false;
            int bi = -1;
            float bd = 0.f;
            auto scan = [&](auto width) {
                constexpr int CW = decltype(width)::value;  // detections per chunk
                for (int c0 = tj * CW; c0 < C; c0 += L * CW) {
                    const int nc = C - c0;
                    uint32_t m = 0u;
#pragma unroll
                    for (int k = 0; k < CW; ++k) {
                        const float2 q = f_detf[c0 + k];
                        m |= (k < nc && dist2(tp, F2{q.x, q.y}) < p.s_match) ? (1u << k) : 0u;
                    }
                    while (m) {  // dist < max_distance; dist = sqrt_rn(s2) as dist() rounds it
                        int d4[4];
                        bool v4[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            v4[u] = m != 0u;
                            d4[u] = v4[u] ? c0 + __ffs(m) - 1 : 0;
                            m &= m - 1u;
                        }
                        float dd4[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const float2 q = f_detf[d4[u]];
                            dd4[u] = ecc::sqrt_rn(dist2(tp, F2{q.x, q.y}));
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            if (!v4[u]) continue;
                            const int d = d4[u];
                            atomicMin(&f_want[d], tag0);
                            if (bi < 0 || dd4[u] < bd || (dd4[u] == bd && d < bi)) { bd = dd4[u]; bi = d; }
                            if (l_n < kFList) {
                                f_li[l_n][tid] = (int16_t)d;
                                f_ld[l_n][tid] = dd4[u];
                                ++l_n;
                            } else {
                                l_ovf = true;
                            }
                        }
                    }
                }
            };
            if (act) {
                if (C <= 16 * L)
                    scan(std::integral_constant<int, 16>{});
                else
                    scan(std::integral_constant<int, 32>{});
            }
            // the track's lanes: minimum, list sizes -> merged list offsets
            // (quad DPP permutes: L = 2 or 4 lanes of a track lie in one quad; the lane shuffles
            // were LDS permutes on the slice's serial chain.  Every permute runs in all lanes:
            // one under a lane condition would read a disabled source lane.)
            int cnt = l_ovf ? kFList + 1 : l_n, incl = cnt;
            auto take = [&](float od, int oi) {
                if (oi >= 0 && (bi < 0 || od < bd || (od == bd && oi < bi))) { bd = od; bi = oi; }
            };
            int total;
            if (L == 4) {  // uniform
                take(qperm_f<0xB1>(bd), qperm<0xB1>(bi));  // lane ^ 1
                const int u1 = qperm<0x90>(incl);             // lane - 1
                incl += tj >= 1 ? u1 : 0;
                take(qperm_f<0x4E>(bd), qperm<0x4E>(bi));  // lane ^ 2
                const int u2 = qperm<0x44>(incl);             // lane - 2
                incl += tj >= 2 ? u2 : 0;
                total = qperm<0xFF>(incl);                   // lane 3 of the quad
            } else {
                take(qperm_f<0xB1>(bd), qperm<0xB1>(bi));  // lane ^ 1
                const int u1 = qperm<0xA0>(incl);             // lane - 1 within the pair
                incl += tj >= 1 ? u1 : 0;
                total = qperm<0xF5>(incl);                   // lane 1 of the pair
            }
            if (act && total <= kFList) {
                const int off = incl - cnt;
                for (int k = 0; k < l_n; ++k) {
                    f_mi[off + k][ti] = f_li[k][tid];
                    f_md[off + k][ti] = f_ld[k][tid];
                }
            }
            if (act && tj == 0) {
                f_mn[ti] = (int8_t)(total <= kFList ? total : -1);
                f_best[ti] = (int16_t)bi;
            }
        }
        __syncthreads();
        if (st == -3) {  // round 0 resolves (owner thread)
            const int b0 = f_best[tid];
            if (b0 < 0) {
                st = -1;
            } else if (f_want[b0] == ((kFTagTop << 8) | tid)) {
                st = b0;
                f_claim[b0] = 1;
            }
        }
        TRK_MARK(8);
        const int my_n = st == -3 ? f_mn[tid] : 0;  // -1: more than kFList in range (rescan)
        {
            // Tail: with <= 64 unresolved tracks and no list overflow, one wave finishes the
            // rounds with no workgroup barrier (a wave's LDS instructions execute in order);
            // each round reads the claims of a track's whole list at once (branch-free: a
            // past-the-list slot reads the always-claimed slot kFT).
            const bool unres = st == -3;
            const uint64_t mu = __ballot(unres), mo = __ballot(unres && my_n < 0);
            if (lane == 0) {
                f_ws[wave] = __popcll(mu);
                f_ws[kFW + wave] = __popcll(mo);
            }
            __syncthreads();
            int u = __popcll(mu & lanes_below()), n_unres = 0, n_ovf = 0;
#pragma unroll
            for (int w = 0; w < kFW; ++w) {
                u += w < wave ? f_ws[w] : 0;
                n_unres += f_ws[w];
                n_ovf += f_ws[kFW + w];
            }
            if (n_unres > 0 && n_unres <= 64 && n_ovf == 0) {
                if (unres) f_tail[u] = (int16_t)tid;
                __syncthreads();
                if (wave == 0) {
                    const bool act = lane < n_unres;
                    const int ti = act ? f_tail[lane] : 0;
                    const int ln = act ? f_mn[ti] : 0;
                    int li[kFList];
                    float ld[kFList];
#pragma unroll
                    for (int k = 0; k < kFList; ++k) {
                        li[k] = k < ln ? f_mi[k][ti] : kFT;
                        ld[k] = f_md[k][ti];
                    }
                    int res = act ? -3 : -2;
                    for (int r = 1; __ballot(res == -3); ++r) {
                        const int tg = ((kFTagTop - r) << 8) | ti;
                        uint8_t cl[kFList];
#pragma unroll
                        for (int k = 0; k < kFList; ++k) cl[k] = f_claim[li[k]];
                        int bi = -1;
                        float bd = 0.f;
#pragma unroll
                        for (int k = 0; k < kFList; ++k) {
                            if (res != -3 || cl[k]) continue;
                            atomicMin(&f_want[li[k]], tg);
                            if (bi < 0 || ld[k] < bd || (ld[k] == bd && li[k] < bi)) { bd = ld[k]; bi = li[k]; }
                        }
                        if (res == -3 && bi < 0) res = -1;
                        wave_sync();
                        if (res == -3 && f_want[bi] == tg) {
                            res = bi;
                            f_claim[bi] = 1;
                        }
                        wave_sync();
#if ECC_TRACKER_PROFILE
                        prof[9] += 1;
#endif
                    }
                    if (act) f_res[ti] = (int16_t)res;
                }
                __syncthreads();
                if (unres) st = f_res[tid];
            }
        }
        // P2 rounds 1.. across the workgroup (many unresolved tracks, or a list overflow)
        int round = 1;
        for (; __syncthreads_or(st == -3); ++round) {
            const int tag = ((kFTagTop - round) << 8) | tid;
            int best = -1;
            if (st == -3) {
                float bd = 0.f;
                if (my_n >= 0) {
#pragma unroll
                    for (int k = 0; k < kFList; ++k) {
                        if (k >= my_n) break;
                        const int d = f_mi[k][tid];
                        if (f_claim[d]) continue;
                        const float dd = f_md[k][tid];
                        atomicMin(&f_want[d], tag);
                        if (best < 0 || dd < bd || (dd == bd && d < best)) { bd = dd; best = d; }
                    }
                } else {
                    for (int d = 0; d < C; ++d) {
                        if (f_claim[d]) continue;
                        const float2 q = f_detf[d];
                        const float s2 = dist2(pp, F2{q.x, q.y});
                        if (!(s2 < p.s_match)) continue;
                        const float dd = ecc::sqrt_rn(s2);
                        atomicMin(&f_want[d], tag);
                        if (best < 0 || dd < bd) { bd = dd; best = d; }
                    }
                }
                if (best < 0) st = -1;
            }
            __syncthreads();
            if (st == -3 && f_want[best] == tag) {
                st = best;
                f_claim[best] = 1;
            }
        }
        TRK_MARK(1);
#if ECC_TRACKER_PROFILE
        prof[6] += round;
#endif
        // P3: update (:471-497); kept tracks at their rank, then new tracks for the unmatched
        // detections in detection order (:501-514); candidates (fsld == 0) listed for P4
        FastTrack ft = me;
        DevTrack &t = ft.t;
        bool keep = false, cand = false;
        if (tid < T) {
            t.is_matched = 0;
            const bool matched = st >= 0;
            if (matched || st == -1) {
                if (matched) {  // :471-485
                    const int2 q = f_det[st];
                    t.x = q.x;
                    t.y = q.y;
                    t.is_matched = 1;
                    t.fsld = 0;
                    t.frame_count++;
                } else {  // missed (:488-497): move to the prediction of P1 (same state)
                    t.x = (int)pp.x;  // Q16 truncation
                    t.y = (int)pp.y;
                    t.fsld++;
                }
                push_hist_cached(ft, p.history);
                if (matched) {
                    const F2 nd = calc_direction_cached(ft, p);
                    t.dtx = nd.x;  // DirectionVector::update
                    t.dty = nd.y;
                    t.dcx = __fadd_rn(__fmul_rn(t.dcx, p.damping), __fmul_rn(t.dtx, __fsub_rn(1.0f, p.damping)));
                    t.dcy = __fadd_rn(__fmul_rn(t.dcy, p.damping), __fmul_rn(t.dty, __fsub_rn(1.0f, p.damping)));
                }
                const F2 v = estimate_velocity(t, p);
                t.vx = v.x;
                t.vy = v.y;
            }
            keep = !(t.fsld > p.frames_to_skip || t.frame_count > p.max_frames);
            cand = keep && t.fsld == 0;
        }
        TRK_MARK(2);
        const bool un = tid < C && !f_claim[tid];
        const uint64_t mk = __ballot(keep), mc = __ballot(cand), mu = __ballot(un);
        if (lane == 0) {
            f_ws[wave] = __popcll(mk);
            f_ws[kFW + wave] = __popcll(mc);
            f_ws[2 * kFW + wave] = __popcll(mu);
        }
        __syncthreads();
        int rk = __popcll(mk & lanes_below()), rc = __popcll(mc & lanes_below()), ru = __popcll(mu & lanes_below());
        int T2 = 0, G0 = 0, n_unm = 0;
#pragma unroll
        for (int w = 0; w < kFW; ++w) {
            const int a = f_ws[w], b = f_ws[kFW + w], c = f_ws[2 * kFW + w];
            rk += w < wave ? a : 0;
            rc += w < wave ? b : 0;
            ru += w < wave ? c : 0;
            T2 += a;
            G0 += b;
            n_unm += c;
        }
        if (keep) fast_put(L, rk, ft);
        if (cand) {
            ck_x[rc] = t.x;
            ck_y[rc] = t.y;
            ck_vx[rc] = t.vx;
            ck_vy[rc] = t.vy;
            ck_label[rc] = t.label;
            ck_tidx[rc] = (int16_t)rk;
            ck_gid[rc] = t.group_id;
        }
        const int room = max_tracks - T;  // counted before the erase, like append-then-erase
        if (un) {
            if (ru < room) {
                if (keep_new) {
                    FastTrack nf;
                    DevTrack &nt = nf.t;
                    nt.x = dnx;
                    nt.y = dny;
                    nt.label = next_label + ru;
                    nt.frame_count = 1;
                    nt.is_matched = 0;
                    nt.fsld = 0;
                    nt.hist_len = 0;
#pragma unroll
                    for (int h = 0; h < kH; ++h) { nt.hx[h] = 0; nt.hy[h] = 0; }
                    push_hist(nt, p.history);
                    nt.vx = nt.vy = 0.f;
                    nt.dcx = nt.dcy = nt.dtx = nt.dty = 0.f;
                    nt.group_id = -1;  // Q17
                    // hist_len 1: no step is read before push_hist_cached computes it (the
                    // entry a push shifts in always sits at index hist_len, past the sum)
#pragma unroll
                    for (int h = 0; h < kH; ++h) { nf.ux[h] = 0.f; nf.uy[h] = 0.f; }
                    nf.um = 0u;
                    fast_put(L, T2 + ru, nf);
                    const int k = G0 + ru;
                    ck_x[k] = nt.x;
                    ck_y[k] = nt.y;
                    ck_vx[k] = 0.f;
                    ck_vy[k] = 0.f;
                    ck_label[k] = nt.label;
                    ck_tidx[k] = (int16_t)(T2 + ru);
                    ck_gid[k] = -1;
                }
            } else {
                err = ECC_ERR_CAPACITY;
            }
        }
        next_label += n_unm;
        const int added = (keep_new && room > 0) ? min(n_unm, room) : 0;
        const int G = G0 + added;
        __syncthreads();
        TRK_MARK(3);
        // P4: greedy grouping in seed order, group-velocity blend into the LDS list (wave 0)
        if (wave == 0)
            group_slice(GroupLds{ck_x, ck_y, ck_label, ck_tidx, ck_vx, ck_vy, ck_gid, ck_proc, gav, gmem, goff,
                                 gstage, &grad},
                        G, s == n_slices - 1, p, max_tracks,
                        [Lp](int k, float vx, float vy, int gid) {
                            Lp->vx[k] = vx;
                            Lp->vy[k] = vy;
                            Lp->group_id[k] = gid;
                        },
                        groups, group_labels, &n_groups, &n_glabels
#if ECC_TRACKER_PROFILE
                        , prof + 12
#endif
                        );
        __syncthreads();
        TRK_MARK(4);
        T = T2 + added;
        if (tid < T) me = fast_get(L, tid);
        TRK_MARK(5);
        dnx = pnx;
        dny = pny;
        c_cur = c_nxt;
        c_nxt = c_nn;
        f_nxt = f_nn;
    }
#if ECC_TRACKER_PROFILE
    prof[10] = clock64() - c0_;
    prof[11] = wall_clock64() - w0_;
    if (tid == 0 && stop > 0)
        for (int k = 0; k < 16; ++k) g_trk_prof[k] = prof[k];
#endif
    if (tid < T) A[tid] = me.t;
    const bool any_err = __syncthreads_or(err != 0);
    if (tid == 0) {
        if (any_err && err == 0) err = ECC_ERR_CAPACITY;
        ctr->n_tracks = T;
        ctr->next_label = next_label;
        ctr->err = err;
        ctr->resume = stop;
        if (stop == n_slices) {
            ctr->n_groups = n_groups;
            ctr->n_group_labels = n_glabels;
        }
    }
}

}  // namespace

struct ecc_tracker {
    ecc_ctx *ctx = nullptr;
    TrackerParams params{};
    int max_tracks = 0, max_det = 0;
    DevTrack *buf[2] = {nullptr, nullptr};
    DevGroup *groups = nullptr;
    int *group_labels = nullptr;
    TrackerCounters *ctr = nullptr;
};

ECC_API void ecc_tracker_cfg_default(ecc_tracker_cfg *cfg) {
    if (!cfg) return;
    // CornerTracker tracker(30.0f, 30, 10, 5, 0.8f, 0.3f, 100.0f), FCT/…group_track.cpp:805-813
    cfg->max_distance = 30.f;
    cfg->max_frames = 30;
    cfg->history_size = 10;
    cfg->frames_to_skip = 5;
    cfg->damping = 0.8f;
    cfg->smoothing = 0.3f;
    cfg->group_radius = 100.f;
}

ECC_API int ecc_tracker_create(ecc_ctx *ctx, const ecc_tracker_cfg *cfg, int32_t max_tracks,
                               int32_t max_detections, ecc_tracker **out) {
    if (!ctx || !cfg || !out || max_tracks < 1 || max_detections < 1 ||
        max_tracks > kMaxTrk || max_detections > kMaxDet || cfg->history_size < 1 || cfg->history_size > kH ||
        cfg->frames_to_skip < 1)
        return ECC_ERR_INVALID;
    *out = nullptr;
    ecc_tracker *tr = new (std::nothrow) ecc_tracker();
    if (!tr) return ECC_ERR_NOMEM;
    tr->ctx = ctx;
    tr->max_tracks = max_tracks;
    tr->max_det = max_detections;
    TrackerParams &p = tr->params;
    p.max_distance = cfg->max_distance;
    p.damping = cfg->damping;
    p.smoothing = cfg->smoothing;
    p.group_radius = cfg->group_radius;
    p.max_frames = cfg->max_frames;
    p.history = cfg->history_size;
    p.frames_to_skip = cfg->frames_to_skip;
    for (int k = 0; k <= kH; ++k) p.pow_tab[k] = (float)std::pow((double)0.8f, (double)k);  // :254
    {
        const float md = p.max_distance, gr = p.group_radius;
        // s < s_match <=> sqrt(s) < md;  s <= s_group <=> sqrt(s) <= gr (NaN radii: never)
        p.s_match = md == md ? first_false([md](float r) { return r < md; }) : -1.0f;
        if (gr == gr) {
            const float above = first_false([gr](float r) { return r <= gr; });
            uint32_t b;
            std::memcpy(&b, &above, 4);
            if (above == 0.0f) {
                p.s_group = -1.0f;
            } else if (b == 0x7F800000u) {
                p.s_group = above;  // every finite s
            } else {
                --b;
                std::memcpy(&p.s_group, &b, 4);
            }
        } else {
            p.s_group = -1.0f;
        }
    }
    hipSetDevice(ctx->device);
    const size_t tb = sizeof(DevTrack) * (size_t)max_tracks;
    bool ok = hipMalloc(&tr->buf[0], tb) == hipSuccess && hipMalloc(&tr->buf[1], tb) == hipSuccess &&
              hipMalloc(&tr->groups, sizeof(DevGroup) * (size_t)max_tracks) == hipSuccess &&
              hipMalloc(&tr->group_labels, sizeof(int) * (size_t)max_tracks) == hipSuccess &&
              hipMalloc(&tr->ctr, sizeof(TrackerCounters)) == hipSuccess &&
              hipMemset(tr->ctr, 0, sizeof(TrackerCounters)) == hipSuccess;
    if (!ok) {
        ecc_tracker_destroy(tr);
        return ECC_ERR_NOMEM;
    }
    *out = tr;
    return ECC_OK;
}

ECC_API int ecc_tracker_destroy(ecc_tracker *tr) {
    if (!tr) return ECC_ERR_INVALID;
    hipSetDevice(tr->ctx->device);
    hipDeviceSynchronize();
    hipFree(tr->buf[0]);
    hipFree(tr->buf[1]);
    hipFree(tr->groups);
    hipFree(tr->group_labels);
    hipFree(tr->ctr);
    delete tr;
    return ECC_OK;
}

static int tracker_launch(ecc_tracker *tr, const ecc_corner *corners, const int64_t *starts, const int32_t *counts,
                          int32_t n_slices, int32_t cap, ecc_stream_t stream) {
    ecc_ctx *ctx = tr->ctx;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    const int cap_eff = cap < tr->max_det ? cap : tr->max_det;
    {
        ECC_TIMED(ctx, ecc::as_stream(stream), "tracker_fast_kernel");
        hipLaunchKernelGGL(tracker_fast_kernel, dim3(1), dim3(kFThreads), 0, ecc::as_stream(stream),
                           tr->buf[0], tr->buf[1], tr->max_tracks, tr->groups, tr->group_labels,
                           tr->ctr, tr->params, corners, starts, counts, n_slices, cap_eff);
    }
    ECC_CHECK_LAUNCH(ctx, "tracker_fast_kernel");
    {  // the slices from ctr->resume on (none when the fast kernel finished the launch)
        ECC_TIMED(ctx, ecc::as_stream(stream), "tracker_kernel");
        hipLaunchKernelGGL(tracker_kernel, dim3(1), dim3(kNT), 0, ecc::as_stream(stream),
                           tr->buf[0], tr->buf[1], tr->max_tracks, tr->groups, tr->group_labels,
                           tr->ctr, tr->params, corners, starts, counts, n_slices, cap_eff);
    }
    ECC_CHECK_LAUNCH(ctx, "tracker_kernel");
    return ECC_OK;
}

ECC_API int ecc_tracker_update(ecc_tracker *tr, const ecc_corner *corners, const int32_t *counts,
                               int32_t n_slices, int32_t cap, ecc_stream_t stream) {
    if (!tr || n_slices < 0 || cap < 0) return ECC_ERR_INVALID;
    if (n_slices == 0) return ECC_OK;
    if (!counts || (cap > 0 && !corners)) return ECC_ERR_INVALID;
    return tracker_launch(tr, corners, nullptr, counts, n_slices, cap, stream);
}

ECC_API int ecc_tracker_update_lists(ecc_tracker *tr, const ecc_corner *corners, const int64_t *starts,
                                     const int32_t *counts, int32_t n_slices, ecc_stream_t stream) {
    if (!tr || n_slices < 0) return ECC_ERR_INVALID;
    if (n_slices == 0) return ECC_OK;
    if (!counts || !starts || !corners) return ECC_ERR_INVALID;
    return tracker_launch(tr, corners, starts, counts, n_slices, tr->max_det, stream);
}

#if ECC_TRACKER_PROFILE
// Profiling builds only (make TRACKER_PROFILE=1): wall-clock ticks of the last update's phases
// (P0+P1, P2, P3 update, P3 append, P4) and the matching rounds; ticks_per_us from the device.
ECC_API int ecc_tracker_profile(unsigned long long *out8, double *ticks_per_us) {
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_trk_prof), 16 * sizeof(unsigned long long)) != hipSuccess) return ECC_ERR_HIP;
    int khz = 0;
    hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    *ticks_per_us = khz / 1000.0;
    return ECC_OK;
}
#endif

ECC_API int ecc_tracker_status(ecc_tracker *tr, ecc_stream_t stream) {
    if (!tr) return ECC_ERR_INVALID;
    TrackerCounters c{};
    ECC_CHECK_HIP(tr->ctx, hipMemcpyAsync(&c, tr->ctr, sizeof(c), hipMemcpyDeviceToHost, ecc::as_stream(stream)), "read ctr");
    ECC_CHECK_HIP(tr->ctx, hipStreamSynchronize(ecc::as_stream(stream)), "sync");
    return c.err;
}

ECC_API int ecc_tracker_get_tracks(ecc_tracker *tr, ecc_track *out, int32_t cap, int32_t *n_out,
                                   ecc_stream_t stream) {
    if (!tr || (cap > 0 && !out)) return ECC_ERR_INVALID;
    hipStream_t s = ecc::as_stream(stream);
    TrackerCounters c{};
    ECC_CHECK_HIP(tr->ctx, hipMemcpyAsync(&c, tr->ctr, sizeof(c), hipMemcpyDeviceToHost, s), "read ctr");
    ECC_CHECK_HIP(tr->ctx, hipStreamSynchronize(s), "sync");
    if (n_out) *n_out = c.n_tracks;
    const int n = c.n_tracks < cap ? c.n_tracks : cap;
    if (n <= 0) return ECC_OK;
    std::vector<DevTrack> h(n);
    ECC_CHECK_HIP(tr->ctx, hipMemcpy(h.data(), tr->buf[c.cur], sizeof(DevTrack) * n, hipMemcpyDeviceToHost), "read tracks");
    for (int i = 0; i < n; ++i) {
        const DevTrack &t = h[i];
        ecc_track &o = out[i];
        std::memset(&o, 0, sizeof(o));
        o.x = t.x; o.y = t.y; o.label = t.label; o.frame_count = t.frame_count;
        o.is_matched = t.is_matched; o.frames_since_last_detection = t.fsld;
        o.hist_len = t.hist_len;
        for (int k = 0; k < t.hist_len && k < kH; ++k) { o.hist_x[k] = t.hx[k]; o.hist_y[k] = t.hy[k]; }
        o.vx = t.vx; o.vy = t.vy;
        o.dir_cur_x = t.dcx; o.dir_cur_y = t.dcy; o.dir_tgt_x = t.dtx; o.dir_tgt_y = t.dty;
        o.group_id = t.fsld == 0 ? t.group_id : -1;
    }
    return c.n_tracks > cap ? ECC_ERR_CAPACITY : ECC_OK;
}

ECC_API int ecc_tracker_get_groups(ecc_tracker *tr, ecc_group *out, int32_t cap, int32_t *n_out,
                                   int32_t *labels, int32_t labels_cap, ecc_stream_t stream) {
    if (!tr || (cap > 0 && !out) || (labels_cap > 0 && !labels)) return ECC_ERR_INVALID;
    hipStream_t s = ecc::as_stream(stream);
    TrackerCounters c{};
    ECC_CHECK_HIP(tr->ctx, hipMemcpyAsync(&c, tr->ctr, sizeof(c), hipMemcpyDeviceToHost, s), "read ctr");
    ECC_CHECK_HIP(tr->ctx, hipStreamSynchronize(s), "sync");
    if (n_out) *n_out = c.n_groups;
    const int n = c.n_groups < cap ? c.n_groups : cap;
    if (n > 0) {
        std::vector<DevGroup> h(n);
        ECC_CHECK_HIP(tr->ctx, hipMemcpy(h.data(), tr->groups, sizeof(DevGroup) * n, hipMemcpyDeviceToHost), "read groups");
        for (int i = 0; i < n; ++i)
            out[i] = ecc_group{h[i].id, h[i].n_labels, h[i].first_label_offset, h[i].avx, h[i].avy,
                               h[i].cx, h[i].cy, h[i].radius};
    }
    const int nl = c.n_group_labels < labels_cap ? c.n_group_labels : labels_cap;
    if (nl > 0)
        ECC_CHECK_HIP(tr->ctx, hipMemcpy(labels, tr->group_labels, sizeof(int) * nl, hipMemcpyDeviceToHost), "read labels");
    return (c.n_groups > cap || c.n_group_labels > labels_cap) ? ECC_ERR_CAPACITY : ECC_OK;
}

// Checkpoint / hand-over (SURVEY §5, §8e "track state handed rank->rank"): the reference's
// CornerTracker is a value (FCT/…group_track.cpp:163-199: the track list plus next_label); this
// replaces the device tracker's list by a host copy, e.g. one ecc_tracker_get_tracks returned.
// The groups are derived state (updateCornerGroups rebuilds them on every update, :321-398) and
// read as empty until the next update.
ECC_API int ecc_tracker_set_tracks(ecc_tracker *tr, const ecc_track *tracks, int32_t n, int32_t next_label,
                                   ecc_stream_t stream) {
    if (!tr || n < 0 || (n > 0 && !tracks)) return ECC_ERR_INVALID;
    if (n > tr->max_tracks) return ECC_ERR_CAPACITY;
    for (int i = 0; i < n; ++i)
        if (tracks[i].hist_len < 0 || tracks[i].hist_len > kH) return ECC_ERR_INVALID;
    hipStream_t s = ecc::as_stream(stream);
    ECC_CHECK_HIP(tr->ctx, hipSetDevice(tr->ctx->device), "hipSetDevice");
    std::vector<DevTrack> h((size_t)n);
    for (int i = 0; i < n; ++i) {
        const ecc_track &t = tracks[i];
        DevTrack &o = h[i];
        std::memset(&o, 0, sizeof(o));
        o.x = t.x; o.y = t.y; o.label = t.label; o.frame_count = t.frame_count;
        o.is_matched = t.is_matched; o.fsld = t.frames_since_last_detection;
        o.hist_len = t.hist_len;
        for (int k = 0; k < t.hist_len; ++k) { o.hx[k] = t.hist_x[k]; o.hy[k] = t.hist_y[k]; }
        o.vx = t.vx; o.vy = t.vy;
        o.dcx = t.dir_cur_x; o.dcy = t.dir_cur_y; o.dtx = t.dir_tgt_x; o.dty = t.dir_tgt_y;
        o.group_id = t.group_id;
    }
    TrackerCounters c{};
    c.n_tracks = n;
    c.next_label = next_label;
    // the copies are staged in pageable memory: synchronous with respect to the host
    ECC_CHECK_HIP(tr->ctx, hipStreamSynchronize(s), "sync");
    if (n > 0)
        ECC_CHECK_HIP(tr->ctx, hipMemcpy(tr->buf[0], h.data(), sizeof(DevTrack) * (size_t)n, hipMemcpyHostToDevice),
                      "write tracks");
    ECC_CHECK_HIP(tr->ctx, hipMemcpy(tr->ctr, &c, sizeof(c), hipMemcpyHostToDevice), "write ctr");
    return ECC_OK;
}

ECC_API int ecc_tracker_next_label(ecc_tracker *tr, int32_t *next_label, ecc_stream_t stream) {
    if (!tr || !next_label) return ECC_ERR_INVALID;
    TrackerCounters c{};
    ECC_CHECK_HIP(tr->ctx, hipMemcpyAsync(&c, tr->ctr, sizeof(c), hipMemcpyDeviceToHost, ecc::as_stream(stream)), "read ctr");
    ECC_CHECK_HIP(tr->ctx, hipStreamSynchronize(ecc::as_stream(stream)), "sync");
    *next_label = c.next_label;
    return ECC_OK;
}
