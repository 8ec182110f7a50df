// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference's hot-path algorithms (LogicTronixInc/Event-Camera-
// Clustering-and-Optical-Flow-Estimation).  Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may load this library, and only as the checker / the CPU
// baseline — never as the product path.  Each function cites the reference file:line it
// restates.  Paths are relative to the reference root; aliases as in SURVEY.md:
//   SMP = event-cam-pre-processing-opencl/event-cam-sampling
//   KM  = event-cam-clustering-accel/event-cam-k-means-clustering
//   FCT = event-cam-tracking/event-cam-fast-corner-tracker
//   PCC = event-cam-clustering/point-cloud-clustering
//   OPT = event-cam-clustering/optics-clustering
//
// Pinning:
//   * downsample counts + k-means assignment: pinned against the reference's own OpenCL kernels
//     (compiled from /root/reference by oracle/ref/Makefile, run on the GPU box through
//     oracle/ref/ref_harness.c) — tests/test_ref_opencl.py;
//   * OPTICS / kd-tree / epsilon estimation: pinned by the reference's assert KATs
//     (OPT/test/test_main.cpp) transcribed into tests/golden/optics_kat.json;
//   * SAE/arc test, NMS, tracker, DBSCAN: the reference code is embedded in Metavision/OpenCV/PCL
//     programs that cannot be built here without stand-in headers -> "parity unpinned" beyond
//     hand-derived known-answer cases (tests/test_oracle_kat.py).
//
// Built with -O2 -ffp-contract=off so fp32 expressions round exactly as written (as the
// reference's gcc build does on x86-64 without FMA).

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <set>
#include <vector>

#include "../include/ecc.h"

#define ORC_API extern "C" __attribute__((visibility("default")))

// ------------------------------------------------------------------------------------------
// a1-a2: hash downsample.  SMP/build/coordinate_processor.cl:3-14 (hash_coordinate),
// :16-89 (process_coordinates).  Executed sequentially in event order, so the racy
// `prev_value == 0` winner (Q2) becomes the lowest event index.
// ------------------------------------------------------------------------------------------
ORC_API int orc_downsample_hash(const uint32_t *xy, int64_t n, int window, int x_max, int y_max,
                                int mult_x, int mult_y, int n_buckets, uint32_t *rep_xy,
                                uint32_t *rep_idx, int32_t *win_unique, int32_t *win_repeated) {
    if (window <= 0 || n_buckets <= 0 || n < 0) return -1;
    std::vector<int> map(n_buckets);
    const int64_t n_win = (n + window - 1) / window;
    for (int64_t w = 0; w < n_win; ++w) {
        std::fill(map.begin(), map.end(), 0);                  // :35-44
        int unique = 0, repeated = 0;
        const int64_t lo = w * window, hi = std::min<int64_t>(n, lo + window);
        for (int64_t i = lo; i < hi; ++i) {                    // :50
            const int x = (int)(xy[i] & 0xffffu), y = (int)(xy[i] >> 16);
            if (x >= 0 && x <= x_max && y >= 0 && y <= y_max) { // :56
                const int h = (x * mult_x + y * mult_y) % n_buckets;  // :11
                const int prev = map[h]++;                     // :62 atomic_inc
                if (prev == 0) {                               // :65-71
                    if (rep_xy) rep_xy[w * window + unique] = xy[i];
                    if (rep_idx) rep_idx[w * window + unique] = (uint32_t)i;
                    ++unique;
                } else if (prev == 1) {                        // :73-75
                    ++repeated;
                }
            }
        }
        if (win_unique) win_unique[w] = unique;
        if (win_repeated) win_repeated[w] = repeated;
    }
    return 0;
}

// ------------------------------------------------------------------------------------------
// a4: analyzeCoordinates / findCoordinate, FCT/metavision_time_surface_periodic.cpp:56-120 — per
// window of `window` pairs, a linear search of the unique list (:56-66) appending new
// coordinates with count 1 or bumping an existing count (:75-95); uniqueCount (:98).
// ------------------------------------------------------------------------------------------
ORC_API int orc_dedup_exact(const uint32_t *xy, int64_t n, int window, uint32_t *uniq_idx, int32_t *uniq_cnt,
                            int32_t *n_unique) {
    if (window <= 0 || n < 0) return -1;
    struct CoordinateInfo { int x, y, count; int64_t first; };
    std::vector<CoordinateInfo> coords;
    const int64_t n_win = (n + window - 1) / window;
    for (int64_t w = 0; w < n_win; ++w) {
        coords.clear();
        const int64_t lo = w * window, hi = std::min<int64_t>(n, lo + window);
        for (int64_t i = lo; i < hi; ++i) {
            const int x = (int)(xy[i] & 0xffffu), y = (int)(xy[i] >> 16);
            int found = -1;
            for (int k = 0; k < (int)coords.size(); k++)  // findCoordinate :56-66
                if (coords[k].x == x && coords[k].y == y) { found = k; break; }
            if (found != -1) coords[found].count++;
            else coords.push_back({x, y, 1, i});
        }
        for (size_t k = 0; k < coords.size(); ++k) {
            if (uniq_idx) uniq_idx[lo + k] = (uint32_t)coords[k].first;
            if (uniq_cnt) uniq_cnt[lo + k] = coords[k].count;
        }
        if (n_unique) n_unique[w] = (int32_t)coords.size();
    }
    return 0;
}

// ------------------------------------------------------------------------------------------
// a5: assign_to_centers, KM/assign_to_centers.cl:1-34.  length((cx-x, cy-y, 0)) < threshold,
// first minimum wins (strict <), indMin = 255 when nothing is closer than the threshold.
// Labels here are centre indices (the kernel stores the even float offset 2c, :26).
// ------------------------------------------------------------------------------------------
static inline uint8_t assign_one(float px, float py, const float *c, int k, float thr) {
    float best = thr;                                   // :11 threshold_dd = 50
    int ind = 255;                                      // :12 uchar indMin = -1
    for (int i = 0; i < k; ++i) {                       // :14 i = 0,2,..,14 over 8 centres
        const float dx = c[2 * i] - px;                 // :15
        const float dy = c[2 * i + 1] - py;             // :16
        const float d = std::sqrt(dx * dx + dy * dy);   // :17-18 length(float3(dx,dy,0))
        if (d < best) { ind = i; best = d; }            // :21-25
    }
    return (uint8_t)ind;
}

ORC_API int orc_kmeans_assign_f32(const float *xy, int64_t n, const float *c, int k, float thr,
                                  uint8_t *labels) {
    for (int64_t i = 0; i < n; ++i) labels[i] = assign_one(xy[2 * i], xy[2 * i + 1], c, k, thr);
    return 0;
}

// a6-a8, "fixed" mode (Appendix A Q7-Q9): Lloyd update = per-cluster mean of the assigned
// points (the reference's intent at KM/assign_to_centers2.c:509-512 without the ss[j+1] index
// bug), sums in fp64 (exact for integer pixel coordinates), unchanged when empty; stop after
// max_iters updates or when the largest per-coordinate shift <= tol (tol < 0: never).
ORC_API int orc_kmeans_run_f32(const float *xy, int64_t n, float *c, int k, int max_iters, float thr,
                               float tol, uint8_t *labels, int32_t *iters_out) {
    std::vector<double> sx(k), sy(k);
    std::vector<int64_t> cnt(k);
    int it = 0;
    for (; it < max_iters;) {
        std::fill(sx.begin(), sx.end(), 0.0);
        std::fill(sy.begin(), sy.end(), 0.0);
        std::fill(cnt.begin(), cnt.end(), 0);
        for (int64_t i = 0; i < n; ++i) {
            const uint8_t a = assign_one(xy[2 * i], xy[2 * i + 1], c, k, thr);
            if (a == 255) continue;                      // assign_data_cluster drops 255/2=127
            sx[a] += xy[2 * i];
            sy[a] += xy[2 * i + 1];
            cnt[a] += 1;
        }
        float shift = 0.f;
        for (int j = 0; j < k; ++j) {
            if (cnt[j] == 0) continue;
            const float nx = (float)(sx[j] / (double)cnt[j]);
            const float ny = (float)(sy[j] / (double)cnt[j]);
            shift = std::max(shift, std::max(std::fabs(nx - c[2 * j]), std::fabs(ny - c[2 * j + 1])));
            c[2 * j] = nx;
            c[2 * j + 1] = ny;
        }
        ++it;
        if (tol >= 0.f && shift <= tol) break;
    }
    if (labels)
        for (int64_t i = 0; i < n; ++i) labels[i] = assign_one(xy[2 * i], xy[2 * i + 1], c, k, thr);
    if (iters_out) *iters_out = it;
    return 0;
}

ORC_API int orc_kmeans_run_xy16(const uint32_t *xy, int64_t n, float *c, int k, int max_iters,
                                float thr, float tol, uint8_t *labels, int32_t *iters_out) {
    std::vector<float> f((size_t)n * 2);
    for (int64_t i = 0; i < n; ++i) {
        f[2 * i] = (float)(xy[i] & 0xffffu);
        f[2 * i + 1] = (float)(xy[i] >> 16);
    }
    return orc_kmeans_run_f32(f.data(), n, c, k, max_iters, thr, tol, labels, iters_out);
}

// "ref_compat" k-means host loop, KM/assign_to_centers2.c:184-548 with its quirks:
// Q7 (ss[j],ss[j+1],ss[j+2],ss[j+3] indexing of the per-1024 partial sums of the 8x4096 bin
// buffer), Q8 (bins re-seeded with the previous readback, never cleared), Q9 (C `abs` on float
// truncates, selective per-coordinate update only while |err| exceeds the running max,
// restart while error_max > 10).  8 centres, bins of 2048.  Returns the number of passes.
// Float reduction order follows reduction_scalar (:121-140): 1024-wide pairwise tree.
static float tree_sum_1024(const float *v) {
    float buf[1024];
    std::memcpy(buf, v, sizeof(buf));
    for (int s = 512; s > 0; s >>= 1)
        for (int l = 0; l < s; ++l) buf[l] += buf[l + s];
    return buf[0];
}

// One pass of the loop above from a given bin buffer (output[8*4096], in/out: the previous
// pass's readback with its stale tails, Q8): the bins' first cluster_index[c] slots are this
// pass's points (index order), the rest keeps the input; sums, update.  Returns 1 when the
// reference would restart (error_max > 10).
// The reference's `abs(new - old)` on a float (assign_to_centers2.c:526-527) is C's int abs(int)
// of the float converted to int.  An empty bin divides by zero (:509-512), and the conversion of
// the resulting inf/NaN is undefined in C; on the reference's x86-64 target cvttss2si yields
// INT_MIN and abs(INT_MIN) stays INT_MIN.  Restated without the UB (the sanitizer build checks).
static float ref_int_abs(float d) {
    if (!(d > -2147483648.f && d < 2147483648.f)) return -2147483648.f;
    return (float)std::abs((int)d);
}

ORC_API int orc_kmeans_refcompat_pass(const float *xy, int64_t n, float *c16, float *output, int32_t *bin_counts_out,
                                      float *partial_sums_out) {
    if (n > 2048 * 8) return -1;
    int cluster_index[8] = {0};
    for (int64_t g = 0; g < n; ++g) {
        const uint8_t a = assign_one(xy[2 * g], xy[2 * g + 1], c16, 8, 50.f);
        const unsigned cl = (a == 255) ? 127u : (unsigned)a;
        if (cl < 8) {
            const int idx = cluster_index[cl]++;
            if (idx < 2048) {
                output[cl * 4096 + idx] = xy[2 * g];
                output[cl * 4096 + 2048 + idx] = xy[2 * g + 1];
            }
        }
    }
    float ss[32];
    for (int gidx = 0; gidx < 32; ++gidx) ss[gidx] = tree_sum_1024(&output[gidx * 1024]);
    float nc[16];
    for (int j = 0; j < 16; j += 2) {
        nc[j] = (ss[j] + ss[j + 1]) / (float)cluster_index[j / 2];
        nc[j + 1] = (ss[j + 2] + ss[j + 3]) / (float)cluster_index[j / 2];
    }
    float error_max = 0.f;
    for (int j = 0; j < 16; ++j) {
        const float a = ref_int_abs(nc[j] - c16[j]);
        if (a > error_max) { error_max = a; c16[j] = nc[j]; }
    }
    if (bin_counts_out) std::memcpy(bin_counts_out, cluster_index, sizeof(cluster_index));
    if (partial_sums_out) std::memcpy(partial_sums_out, ss, sizeof(ss));
    return error_max > 10.f ? 1 : 0;
}

ORC_API int orc_kmeans_refcompat(const float *xy, int64_t n, float *c16, int max_passes,
                                 int32_t *bin_counts_out, float *partial_sums_out) {
    if (n > 2048 * 8) return -1;
    std::vector<float> output(8 * 4096, 0.f);            // :133-137 zero once
    int passes = 0;
    for (;;) {
        int cluster_index[8] = {0};                      // :186-188
        for (int64_t g = 0; g < n; ++g) {                // assign + scatter, in index order
            const uint8_t a = assign_one(xy[2 * g], xy[2 * g + 1], c16, 8, 50.f);
            const unsigned cl = (a == 255) ? 127u : (unsigned)a;  // (2c)/2, 255/2 = 127
            if (cl < 8) {
                const int idx = cluster_index[cl]++;
                if (idx < 2048) {                        // no overflow check in the kernel
                    output[cl * 4096 + idx] = xy[2 * g];
                    output[cl * 4096 + 2048 + idx] = xy[2 * g + 1];
                }
            }
        }
        float ss[32];
        for (int gidx = 0; gidx < 32; ++gidx) ss[gidx] = tree_sum_1024(&output[gidx * 1024]);
        float nc[16];
        for (int j = 0; j < 16; j += 2) {                // :509-512 (Q7)
            nc[j] = (ss[j] + ss[j + 1]) / (float)cluster_index[j / 2];
            nc[j + 1] = (ss[j + 2] + ss[j + 3]) / (float)cluster_index[j / 2];
        }
        float err[16], error_max = 0.f;
        for (int j = 0; j < 16; ++j) err[j] = nc[j] - c16[j];
        for (int j = 0; j < 16; ++j) {                   // :525-532 (Q9)
            const float a = ref_int_abs(err[j]);
            if (a > error_max) { error_max = a; c16[j] = nc[j]; }
        }
        ++passes;
        if (bin_counts_out) std::memcpy(bin_counts_out, cluster_index, sizeof(cluster_index));
        if (partial_sums_out) std::memcpy(partial_sums_out, ss, sizeof(ss));
        if (!(error_max > 10.f) || passes >= max_passes) break;  // :545-548
    }
    return passes;
}

// ------------------------------------------------------------------------------------------
// a16-a17: batch SAE update + arc test.  FCT/metavision_time_surface_periodic_group_track.cpp
// circles :44-45 ({dy,dx} pairs: at(y + c[0], x + c[1])), SAE write :900-923, arc test
// :948-1063.  Slices of `slice` events (make_n_events(16384), :772-774); detection only for
// slices with index >= first_detect (time_surface_flag, :797/:878/:926).
// ------------------------------------------------------------------------------------------
static const int kCircle3[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},  {3, 0},  {3, -1},
                                    {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                    {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};
static const int kCircle4[20][2] = {{0, 4},   {1, 4},   {2, 3},   {3, 2},   {4, 1},
                                    {4, 0},   {4, -1},  {3, -2},  {2, -3},  {1, -4},
                                    {0, -4},  {-1, -4}, {-2, -3}, {-3, -2}, {-4, -1},
                                    {-4, 0},  {-4, 1},  {-3, 2},  {-2, 3},  {-1, 4}};

template <int N, int SMIN, int SMAX>
static bool streak_test(const int64_t *sae, int W, int x, int y, const int (*circ)[2]) {
    auto T = [&](int k) -> int64_t {
        const int kk = ((k % N) + N) % N;
        return sae[(int64_t)(y + circ[kk][0]) * W + (x + circ[kk][1])];
    };
    for (int i = 0; i < N; i++) {                                     // :962 / :1012
        for (int s = SMIN; s <= SMAX; s++) {                          // :964 / :1014
            if (T(i) < T(i - 1 + N)) continue;                        // :968 / :1017
            if (T(i + s - 1) < T(i + s)) continue;                    // :972 / :1021
            double min_t = (double)T(i);                              // :977 / :1024
            for (int j = 1; j < s; j++) {                             // :978-983
                const double tj = (double)T(i + j);
                if (tj < min_t) min_t = tj;
            }
            bool did_break = false;
            for (int j = s; j < N; j++) {                             // :986-995
                const double tj = (double)T(i + j);
                if (tj >= min_t) { did_break = true; break; }
            }
            if (!did_break) return true;                              // :997-1001
        }
    }
    return false;
}

ORC_API int orc_arc_test(const int64_t *sae, int W, int x, int y) {
    if (!streak_test<16, 3, 6>(sae, W, x, y, kCircle3)) return 0;
    return streak_test<20, 4, 8>(sae, W, x, y, kCircle4) ? 1 : 0;
}

ORC_API int orc_fast_detect(const uint32_t *xy, const int64_t *t, int64_t n, int W, int H,
                            int slice, int margin, int border_mode, int first_detect, int64_t *sae,
                            uint8_t *flags) {
    if (slice <= 0 || W <= 2 * margin || H <= 2 * margin) return -1;
    const int64_t n_slices = (n + slice - 1) / slice;
    for (int64_t s = 0; s < n_slices; ++s) {
        const int64_t lo = s * slice, hi = std::min<int64_t>(n, lo + slice);
        for (int64_t e = lo; e < hi; ++e) {                             // :900-923
            const int x = (int)(xy[e] & 0xffffu), y = (int)(xy[e] >> 16);
            if (x < W && y < H) sae[(int64_t)y * W + x] = t[e];
            flags[e] = 0;
        }
        if (s < first_detect) continue;                                 // :926
        for (int64_t e = lo; e < hi; ++e) {                             // :932
            const int x = (int)(xy[e] & 0xffffu), y = (int)(xy[e] >> 16);
            if (x < margin || x >= W - margin || y < margin || y >= H - margin) {  // :951-953
                if (border_mode == 1) break;                            // :957 (Q11)
                continue;
            }
            flags[e] = (uint8_t)orc_arc_test(sae, W, x, y);             // :960-1063
        }
    }
    return 0;
}

// ------------------------------------------------------------------------------------------
// a18: CornerFilter::filterCorners, FCT/…group_track.cpp:81-152.  The candidate corners of a
// slice are its flagged events in event order (corners.push_back at :1061).
// ------------------------------------------------------------------------------------------
ORC_API int orc_filter_corners(const ecc_corner *in, int n_in, int W, int H, int box,
                               ecc_corner *out, int cap) {
    if (n_in <= 0) return 0;                                            // :88-89
    std::vector<uint8_t> mask((size_t)W * H, 0);                        // :99
    const int half = box / 2;                                           // :102
    int n_out = 0;
    for (int c = 0; c < n_in; ++c) {                                    // :105
        const ecc_corner &cr = in[c];
        const int sx = std::max(0, cr.x - half), ex = std::min(W - 1, cr.x + half);  // :114-117
        const int sy = std::max(0, cr.y - half), ey = std::min(H - 1, cr.y + half);
        bool local_max = true;
        for (int y = sy; y <= ey && local_max; y++)                     // :120-132
            for (int x = sx; x <= ex; x++)
                if (mask[(size_t)y * W + x] > 0) { local_max = false; break; }
        if (!local_max) continue;
        if (n_out < cap) out[n_out] = ecc_corner{cr.x, cr.y, n_out};   // :137-142
        ++n_out;
        for (int y = sy; y <= ey; y++)                                  // :144-147 filled rect
            for (int x = sx; x <= ex; x++) mask[(size_t)y * W + x] = 255;
    }
    return n_out;
}

ORC_API int orc_corner_nms(const uint32_t *xy, const uint8_t *flags, int64_t n, int slice, int W,
                           int H, int box, int cap, ecc_corner *out, int32_t *counts) {
    const int64_t n_slices = (n + slice - 1) / slice;
    std::vector<ecc_corner> cand;
    int rc = 0;
    for (int64_t s = 0; s < n_slices; ++s) {
        cand.clear();
        const int64_t lo = s * slice, hi = std::min<int64_t>(n, lo + slice);
        for (int64_t e = lo; e < hi; ++e)
            if (flags[e]) cand.push_back(ecc_corner{(int)(xy[e] & 0xffffu), (int)(xy[e] >> 16), 0});
        int k = orc_filter_corners(cand.data(), (int)cand.size(), W, H, box, out + s * cap, cap);
        if (k > cap) { k = cap; rc = -4; }
        counts[s] = k;
    }
    return rc;
}

// ------------------------------------------------------------------------------------------
// a19-a21: CornerTracker, FCT/…group_track.cpp:163-537.  cv::Point2f arithmetic is restated
// with an fp32 pair whose operators round exactly like OpenCV's (one rounding per * and +).
// ------------------------------------------------------------------------------------------
namespace {
struct P2 {
    float x, y;
};
static inline P2 operator+(P2 a, P2 b) { return P2{a.x + b.x, a.y + b.y}; }
static inline P2 operator*(P2 a, float s) { return P2{a.x * s, a.y * s}; }
static inline P2 &operator+=(P2 &a, P2 b) { a.x += b.x; a.y += b.y; return a; }
static inline P2 &operator*=(P2 &a, float s) { a.x *= s; a.y *= s; return a; }

struct Dir { P2 current, target; float damping, smoothing; };       // :163-175
struct Track {                                                       // :177-190
    int x, y, label, frame_count;
    bool is_matched;
    int fsld;
    std::deque<std::pair<int, int>> hist;
    P2 velocity;
    Dir dir;
    int group_id;
};
struct Group { std::vector<int> labels; P2 avg_vel, centroid; float radius; };  // :193-199

struct OrcTracker {
    ecc_tracker_cfg cfg;
    int next_label = 0;
    std::vector<Track> tracks;
    std::map<int, Group> groups;
    float pow_tab[ECC_TRACK_HIST_MAX + 1];

    explicit OrcTracker(const ecc_tracker_cfg &c) : cfg(c) {
        for (int k = 0; k <= ECC_TRACK_HIST_MAX; ++k)   // std::pow(0.8f, i-1): double pow, :254
            pow_tab[k] = (float)std::pow((double)0.8f, (double)k);
    }
    static float dist(P2 a, P2 b) {                                   // :217-222
        const float dx = a.x - b.x, dy = a.y - b.y;
        return std::sqrt(dx * dx + dy * dy);
    }
    void push_hist(Track &t) {                                        // :224-231
        t.hist.push_front({t.x, t.y});
        if ((int)t.hist.size() > cfg.history_size) t.hist.pop_back();
    }
    P2 direction(const Track &t) {                                    // :233-271
        if (t.hist.size() < 2) return P2{0, 0};
        P2 w{0, 0};
        float total = 0;
        for (size_t i = 1; i < t.hist.size(); ++i) {
            P2 d{(float)(t.hist[i - 1].first - t.hist[i].first),
                 (float)(t.hist[i - 1].second - t.hist[i].second)};
            const float mag = std::sqrt(d.x * d.x + d.y * d.y);
            if (mag > 0) {
                d *= 1.0f / mag;
                const float wt = pow_tab[i - 1];
                w += d * wt;
                total += wt;
            }
        }
        if (total > 0) {
            w *= 1.0f / total;
            const float mag = std::sqrt(w.x * w.x + w.y * w.y);
            if (mag > 0) w *= 1.0f / mag;
        }
        return w;
    }
    P2 velocity(const Track &t) {                                     // :273-302
        if (t.hist.size() < 2) return P2{0, 0};
        P2 tot{0, 0};
        int count = 0;
        for (size_t i = 1; i < t.hist.size(); ++i) {
            tot += P2{(float)(t.hist[i - 1].first - t.hist[i].first),
                      (float)(t.hist[i - 1].second - t.hist[i].second)};
            count++;
        }
        const P2 avg = count > 0 ? tot * (1.0f / count) : P2{0, 0};
        const float speed = std::sqrt(avg.x * avg.x + avg.y * avg.y);
        if (speed > 0) {
            const P2 dv = t.dir.current * speed;
            return avg * (1.0f - cfg.smoothing) + dv * cfg.smoothing;
        }
        return avg;
    }
    P2 predict(const Track &t) {                                      // :304-319
        P2 pred = P2{(float)t.x, (float)t.y} + t.velocity;
        if (t.fsld > 0) {
            const float conf = std::max(0.0f, 1.0f - t.fsld / (float)cfg.frames_to_skip);
            const P2 dp = P2{(float)t.x, (float)t.y} +
                          t.dir.current * std::sqrt(t.velocity.x * t.velocity.x +
                                                    t.velocity.y * t.velocity.y);
            pred = pred * (1.0f - conf) + dp * conf;
        }
        return pred;
    }
    void update_groups() {                                            // :321-398
        groups.clear();
        int next_gid = 0;
        std::vector<bool> processed(tracks.size(), false);
        for (size_t i = 0; i < tracks.size(); i++) {
            if (processed[i] || tracks[i].fsld > 0) continue;
            Group g;
            P2 sp{0, 0}, sv{0, 0};
            int count = 0;
            for (size_t j = 0; j < tracks.size(); j++) {
                if (processed[j] || tracks[j].fsld > 0) continue;
                const float d = dist(P2{(float)tracks[i].x, (float)tracks[i].y},
                                     P2{(float)tracks[j].x, (float)tracks[j].y});
                if (d <= cfg.group_radius) {
                    processed[j] = true;
                    g.labels.push_back(tracks[j].label);
                    tracks[j].group_id = next_gid;
                    sp += P2{(float)tracks[j].x, (float)tracks[j].y};
                    sv += tracks[j].velocity;
                    count++;
                }
            }
            if (count > 0) {
                g.centroid = sp * (1.0f / count);
                g.avg_vel = sv * (1.0f / count);
                float mr = 0;
                for (int lab : g.labels) {
                    for (const Track &t : tracks) {
                        if (t.label == lab) {
                            mr = std::max(mr, dist(P2{(float)t.x, (float)t.y}, g.centroid));
                            break;
                        }
                    }
                }
                g.radius = mr;
                groups[next_gid] = g;
                next_gid++;
            }
        }
        for (Track &t : tracks) {
            if (t.fsld == 0 && groups.count(t.group_id)) {
                const Group &g = groups[t.group_id];
                t.velocity = t.velocity * 0.7f + g.avg_vel * 0.3f;
            }
        }
    }
    void update(const ecc_corner *cs, int n) {                        // :421-530
        std::vector<Track> det;
        for (int i = 0; i < n; ++i) {
            Track t{};
            t.x = cs[i].x; t.y = cs[i].y; t.label = -1; t.frame_count = 0; t.is_matched = false;
            t.fsld = 0; t.velocity = P2{0, 0};
            t.dir = Dir{P2{0, 0}, P2{0, 0}, cfg.damping, cfg.smoothing};
            t.group_id = -1;                                          // Q17
            det.push_back(t);
        }
        for (Track &t : tracks) t.is_matched = false;
        std::vector<bool> matched(det.size(), false);
        for (Track &t : tracks) {
            if (t.fsld > cfg.frames_to_skip) continue;
            const P2 pp = predict(t);
            float md = cfg.max_distance;
            int best = -1;
            for (size_t i = 0; i < det.size(); ++i) {
                if (matched[i]) continue;
                const float d = dist(pp, P2{(float)det[i].x, (float)det[i].y});
                if (d < md) { md = d; best = (int)i; }
            }
            if (best >= 0) {
                t.x = det[best].x; t.y = det[best].y;
                t.is_matched = true; t.fsld = 0; t.frame_count++;
                push_hist(t);
                const P2 nd = direction(t);
                t.dir.target = nd;                                     // DirectionVector::update
                t.dir.current = t.dir.current * t.dir.damping + t.dir.target * (1.0f - t.dir.damping);
                t.velocity = velocity(t);
                matched[best] = true;
            } else {
                const P2 pr = predict(t);
                t.x = (int)pr.x; t.y = (int)pr.y;                     // Q16 truncation
                t.fsld++;
                push_hist(t);
                t.velocity = velocity(t);
            }
        }
        for (size_t i = 0; i < det.size(); ++i) {
            if (matched[i]) continue;
            Track nt = det[i];
            nt.label = next_label++;
            nt.frame_count = 1;
            nt.fsld = 0;
            nt.velocity = P2{0, 0};
            nt.dir = Dir{P2{0, 0}, P2{0, 0}, cfg.damping, cfg.smoothing};
            push_hist(nt);
            tracks.push_back(nt);
        }
        tracks.erase(std::remove_if(tracks.begin(), tracks.end(),
                                    [this](const Track &c) {
                                        return c.fsld > cfg.frames_to_skip ||
                                               c.frame_count > cfg.max_frames;
                                    }),
                     tracks.end());
        update_groups();
    }
};
}  // namespace

ORC_API void *orc_tracker_create(const ecc_tracker_cfg *cfg) { return new OrcTracker(*cfg); }
ORC_API void orc_tracker_destroy(void *tr) { delete static_cast<OrcTracker *>(tr); }
ORC_API int orc_tracker_update(void *tr, const ecc_corner *cs, int n) {
    static_cast<OrcTracker *>(tr)->update(cs, n);
    return 0;
}
ORC_API int orc_tracker_get_tracks(void *trp, ecc_track *out, int cap) {
    OrcTracker *tr = static_cast<OrcTracker *>(trp);
    const int n = (int)tr->tracks.size();
    for (int i = 0; i < n && i < cap; ++i) {
        const Track &t = tr->tracks[i];
        ecc_track &o = out[i];
        std::memset(&o, 0, sizeof(o));
        o.x = t.x; o.y = t.y; o.label = t.label; o.frame_count = t.frame_count;
        o.is_matched = t.is_matched; o.frames_since_last_detection = t.fsld;
        o.hist_len = (int)t.hist.size();
        for (size_t h = 0; h < t.hist.size() && h < ECC_TRACK_HIST_MAX; ++h) {
            o.hist_x[h] = t.hist[h].first;
            o.hist_y[h] = t.hist[h].second;
        }
        o.vx = t.velocity.x; o.vy = t.velocity.y;
        o.dir_cur_x = t.dir.current.x; o.dir_cur_y = t.dir.current.y;
        o.dir_tgt_x = t.dir.target.x; o.dir_tgt_y = t.dir.target.y;
        o.group_id = t.fsld == 0 ? t.group_id : -1;
    }
    return n;
}
ORC_API int orc_tracker_get_groups(void *trp, ecc_group *out, int cap, int32_t *labels,
                                   int labels_cap) {
    OrcTracker *tr = static_cast<OrcTracker *>(trp);
    int n = 0, off = 0;
    for (const auto &kv : tr->groups) {
        if (n < cap) {
            ecc_group &g = out[n];
            g.id = kv.first;
            g.n_labels = (int)kv.second.labels.size();
            g.first_label_offset = off;
            g.avg_vx = kv.second.avg_vel.x; g.avg_vy = kv.second.avg_vel.y;
            g.cx = kv.second.centroid.x; g.cy = kv.second.centroid.y;
            g.radius = kv.second.radius;
        }
        for (int lab : kv.second.labels) {
            if (off < labels_cap) labels[off] = lab;
            ++off;
        }
        ++n;
    }
    return n;
}

// ------------------------------------------------------------------------------------------
// a10-a12: eps-neighbourhood (brute force, DBSCAN_simple.h:118-142: d^2 <= eps^2 in double,
// self included) and core distance (optics.hpp:286-299: (min_pts-1)-th smallest distance of the
// neighbourhood incl. self, via nth_element on squared distance).  Points are segmented like the
// library (segment s point j at s*stride+j, j < seg_counts[s]); lists hold segment-local
// indices in ascending order.
// ------------------------------------------------------------------------------------------
ORC_API int orc_eps_neighbours(const uint32_t *xy, int64_t n_segs, int64_t stride,
                               const int32_t *seg_counts, double eps, int min_pts, int32_t *counts,
                               double *core_dist, int64_t *offsets, int32_t *nbr, int64_t nbr_cap) {
    const double r2 = eps * eps;
    int64_t off = 0;
    std::vector<double> d2s;
    for (int64_t s = 0; s < n_segs; ++s) {
        const int64_t base = s * stride;
        const int m = seg_counts ? seg_counts[s] : (int)stride;
        for (int i = 0; i < m; ++i) {
            const double xi = (double)(xy[base + i] & 0xffffu), yi = (double)(xy[base + i] >> 16);
            d2s.clear();
            if (offsets) offsets[base + i] = off;
            for (int j = 0; j < m; ++j) {
                const double dx = (double)(xy[base + j] & 0xffffu) - xi;
                const double dy = (double)(xy[base + j] >> 16) - yi;
                const double d2 = dx * dx + dy * dy;
                if (d2 <= r2) {
                    d2s.push_back(d2);
                    if (nbr && off < nbr_cap) nbr[off] = j;
                    ++off;
                }
            }
            if (counts) counts[base + i] = (int32_t)d2s.size();
            if (core_dist) {
                if ((int)d2s.size() < min_pts || min_pts < 1) {
                    core_dist[base + i] = -1.0;
                } else {
                    std::nth_element(d2s.begin(), d2s.begin() + (min_pts - 1), d2s.end());
                    core_dist[base + i] = std::sqrt(d2s[min_pts - 1]);
                }
            }
        }
        if (offsets && m < stride) {
            for (int64_t i = m; i < stride; ++i) offsets[base + i] = off;
        }
    }
    if (offsets) offsets[n_segs * stride] = off;
    return off > nbr_cap && nbr ? -4 : 0;
}

// a9-a10: DBSCANSimpleCluster::extract, PCC/DBSCAN_simple.h:27-90, literally (seed queue, types,
// noise flags), with the brute-force radiusSearch (:118-142) over a cloud of n points of `dim`
// coordinates of type T.  pcl::PointXYZ's fields are float, so `double distance_x =
// points[i].x - points[index].x` subtracts in FLOAT and widens the difference (:132-134);
// distance_square = dx*dx + dy*dy + dz*dz in double (:135) <= radius*radius (:127).  The
// index itself is pushed first with distance 0 (:124-125).  Output: the clusters in output order
// (size descending :89, ties by smallest member — std::sort is unstable, Q23 — then creation),
// each sorted + unique (:82-83), as CSR (offs[c]..offs[c+1]); labels[i] = the last output
// cluster containing i, or -1.  Returns the number of clusters.
template <typename T>
static int dbscan_cloud(const T *pts, int n, int dim, double eps, int min_pts, int min_size, int max_size,
                        int32_t *labels, int64_t *offs, int32_t *members, int64_t cap) {
    enum { UNP = 0, PROC = 1, DONE = 2 };
    const double r2 = eps * eps;
    auto radius = [&](int idx, std::vector<int> &out) {
        out.clear();
        out.push_back(idx);
        for (int i = 0; i < n; i++) {
            if (i == idx) continue;
            double d2 = 0.0;
            for (int d = 0; d < dim; ++d) {
                const T diff = pts[(int64_t)i * dim + d] - pts[(int64_t)idx * dim + d];  // in the point type
                const double dd = (double)diff;
                d2 = d == 0 ? dd * dd : d2 + dd * dd;
            }
            if (d2 <= r2) out.push_back(i);
        }
        return (int)out.size();
    };
    std::vector<int> nn, types(n, UNP);
    std::vector<bool> noise(n, false);
    std::vector<std::vector<int>> clusters;
    for (int i = 0; i < n; i++) {
        if (types[i] == DONE) continue;
        int sz = radius(i, nn);
        if (sz < min_pts) { noise[i] = true; continue; }
        std::vector<int> q{i};
        types[i] = DONE;
        for (int j = 0; j < sz; j++)
            if (nn[j] != i) { q.push_back(nn[j]); types[nn[j]] = PROC; }
        size_t qi = 1;
        while (qi < q.size()) {
            const int ci = q[qi];
            if (noise[ci] || types[ci] == DONE) { types[ci] = DONE; qi++; continue; }
            sz = radius(ci, nn);
            if (sz >= min_pts)
                for (int j = 0; j < sz; j++)
                    if (types[nn[j]] == UNP) { q.push_back(nn[j]); types[nn[j]] = PROC; }
            types[ci] = DONE;
            qi++;
        }
        if ((int64_t)q.size() >= min_size && (int64_t)q.size() <= max_size) {
            std::sort(q.begin(), q.end());
            q.erase(std::unique(q.begin(), q.end()), q.end());
            clusters.push_back(q);
        }
    }
    std::stable_sort(clusters.begin(), clusters.end(),
                     [](const std::vector<int> &a, const std::vector<int> &b) {
                         if (a.size() != b.size()) return a.size() > b.size();
                         return a.front() < b.front();
                     });
    if (labels) {  // a point in several clusters keeps the last one in output order
        for (int i = 0; i < n; ++i) labels[i] = -1;
        for (size_t c = 0; c < clusters.size(); ++c)
            for (int idx : clusters[c]) labels[idx] = (int32_t)c;
    }
    if (offs) {
        int64_t k = 0;
        offs[0] = 0;
        for (size_t c = 0; c < clusters.size(); ++c) {
            for (int v : clusters[c]) { if (members && k < cap) members[k] = v; ++k; }
            offs[c + 1] = k;
        }
    }
    return (int)clusters.size();
}

// 3-D float points (x, y, z per point); labels = the LAST output cluster holding the point (the
// shared body above overwrites in output order).  The GPU label is the first-claim cluster's rank,
// so where border points have duplicate memberships compare cluster lists, not labels.
ORC_API int orc_dbscan(const float *pts, int n, double eps, int min_pts, int min_size, int max_size,
                       int32_t *labels) {
    return dbscan_cloud<float>(pts, n, 3, eps, min_pts, min_size, max_size, labels, nullptr, nullptr, 0);
}

ORC_API int orc_dbscan_cloud_f32(const float *pts, int n, int dim, double eps, int min_pts, int min_size, int max_size,
                                 int32_t *labels, int64_t *offs, int32_t *members, int64_t cap) {
    return dbscan_cloud<float>(pts, n, dim, eps, min_pts, min_size, max_size, labels, offs, members, cap);
}

ORC_API int orc_dbscan_cloud_f64(const double *pts, int n, int dim, double eps, int min_pts, int min_size,
                                 int max_size, int32_t *labels, int64_t *offs, int32_t *members, int64_t cap) {
    return dbscan_cloud<double>(pts, n, dim, eps, min_pts, min_size, max_size, labels, offs, members, cap);
}

// a10 (DBSCAN_precomp.h:22-44 for float clouds): counts, core distances (optics.hpp:286-299 on
// the same d^2) and adjacency rows in ascending index order, brute force over all pairs.
ORC_API int orc_radius_f32(const float *pts, int n, int dim, double eps, int min_pts, int32_t *counts,
                           double *core_dist, int64_t *offsets, int32_t *nbr, int64_t cap) {
    const double r2 = eps * eps;
    int64_t off = 0;
    std::vector<double> d2s;
    for (int i = 0; i < n; ++i) {
        d2s.clear();
        if (offsets) offsets[i] = off;
        for (int j = 0; j < n; ++j) {
            double d2 = 0.0;
            for (int d = 0; d < dim; ++d) {
                const float diff = pts[(int64_t)j * dim + d] - pts[(int64_t)i * dim + d];
                const double dd = (double)diff;
                d2 = d == 0 ? dd * dd : d2 + dd * dd;
            }
            if (d2 <= r2) {
                d2s.push_back(d2);
                if (nbr && off < cap) nbr[off] = j;
                ++off;
            }
        }
        if (counts) counts[i] = (int32_t)d2s.size();
        if (core_dist) {
            if ((int)d2s.size() < min_pts || min_pts < 1) {
                core_dist[i] = -1.0;
            } else {
                std::nth_element(d2s.begin(), d2s.begin() + (min_pts - 1), d2s.end());
                core_dist[i] = std::sqrt(d2s[min_pts - 1]);
            }
        }
    }
    if (offsets) offsets[n] = off;
    return off > cap && nbr ? -4 : 0;
}

// a13: optics::compute_reachability_dists, OPT/include/optics/optics.hpp:413-565 with exact
// eps-balls (the KDTREE back end's radius_search, kdTree.hpp:407-422, equals the exact ball
// except for the tie case documented as quirk Q21).  Points are D-dim doubles (D <= 3).
// Output: order[i] = point index, reach[i] = reachability (-1 undefined).
namespace {
struct RD {
    size_t idx;
    double r;
};
struct RDLess {  // optics.hpp:67-69
    bool operator()(const RD &a, const RD &b) const {
        return (a.r <= b.r && a.r >= b.r) ? (a.idx < b.idx) : (a.r < b.r);
    }
};
}  // namespace

static double dist_d(const double *a, const double *b, int D) {
    double s = 0;
    for (int i = 0; i < D; ++i) { const double d = a[i] - b[i]; s += d * d; }
    return std::sqrt(s);
}

// §8f rank 3 checker: the same seed-queue restatement (DBSCAN_simple.h:27-90) over 2-D integer
// points, returning the full cluster lists in output order (CSR: offs[c]..offs[c+1] indices
// ascending); a point may appear in several clusters, as in the reference.  Returns clusters.
ORC_API int orc_dbscan_lists(const int32_t *xy, int n, double eps, int min_pts, int min_size, int max_size,
                             int64_t *offs, int32_t *members, int64_t cap) {
    enum { UNP = 0, PROC = 1, DONE = 2 };
    const double r2 = eps * eps;
    // neighbour lists (self included, ascending) — radiusSearch :118-142
    std::vector<std::vector<int>> nl(n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            const double dx = (double)xy[2 * j] - xy[2 * i], dy = (double)xy[2 * j + 1] - xy[2 * i + 1];
            if (dx * dx + dy * dy <= r2) nl[i].push_back(j);
        }
    std::vector<int> types(n, UNP);
    std::vector<bool> noise(n, false);
    std::vector<std::vector<int>> clusters;
    for (int i = 0; i < n; i++) {
        if (types[i] == DONE) continue;
        if ((int)nl[i].size() < min_pts) { noise[i] = true; continue; }
        std::vector<int> q{i};
        types[i] = DONE;
        for (int v : nl[i])
            if (v != i) { q.push_back(v); types[v] = PROC; }
        for (size_t qi = 1; qi < q.size(); ++qi) {
            const int ci = q[qi];
            if (noise[ci] || types[ci] == DONE) { types[ci] = DONE; continue; }
            if ((int)nl[ci].size() >= min_pts)
                for (int v : nl[ci])
                    if (types[v] == UNP) { q.push_back(v); types[v] = PROC; }
            types[ci] = DONE;
        }
        if ((int)q.size() >= min_size && (int)q.size() <= max_size) {
            std::sort(q.begin(), q.end());
            q.erase(std::unique(q.begin(), q.end()), q.end());
            clusters.push_back(q);
        }
    }
    std::stable_sort(clusters.begin(), clusters.end(), [](const std::vector<int> &a, const std::vector<int> &b) {
        if (a.size() != b.size()) return a.size() > b.size();
        return a.front() < b.front();
    });
    int64_t k = 0;
    offs[0] = 0;
    for (size_t c = 0; c < clusters.size(); ++c) {
        for (int v : clusters[c]) { if (k < cap) members[k] = v; ++k; }
        offs[c + 1] = k;
    }
    return (int)clusters.size();
}

ORC_API double orc_epsilon_estimation(const double *pts, int n, int D, int min_pts) {
    // optics.hpp:340-387 (bounding_box initialises max from points[1], Q20)
    if (n <= 1) return 0;
    double mn[3], mx[3];
    for (int i = 0; i < D; ++i) { mn[i] = pts[i]; mx[i] = pts[D + i]; }
    for (int p = 0; p < n; ++p)
        for (int i = 0; i < D; ++i) {
            if (pts[p * D + i] < mn[i]) mn[i] = pts[p * D + i];
            if (pts[p * D + i] > mx[i]) mx[i] = pts[p * D + i];
        }
    double vol = 1;
    for (int i = 0; i < D; ++i) vol *= std::abs(mx[i] - mn[i]);
    const double d = (double)D;
    const double space = (vol / (double)n) * (double)min_pts;
    const double ball = std::sqrt(std::pow(M_PI, d)) / std::tgamma(d / 2.0 + 1.0);
    return std::pow(space / ball, 1.0 / d);
}

ORC_API int orc_optics(const double *pts, int n, int D, int min_pts, double eps, int64_t *order,
                       double *reach_out) {
    if (n < 1) return 0;
    if (eps <= 0.0) eps = orc_epsilon_estimation(pts, n, D, min_pts);
    std::vector<std::vector<size_t>> nb(n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double s = 0;
            for (int k = 0; k < D; ++k) { const double dd = pts[j * D + k] - pts[i * D + k]; s += dd * dd; }
            if (s <= eps * eps) nb[i].push_back(j);
        }
    auto core = [&](int p, double &cd) -> bool {                       // :286-299
        if (nb[p].size() < (size_t)min_pts) return false;
        std::vector<double> d2;
        for (size_t q : nb[p]) {
            double s = 0;
            for (int k = 0; k < D; ++k) { const double dd = pts[p * D + k] - pts[q * D + k]; s += dd * dd; }
            d2.push_back(s);
        }
        std::nth_element(d2.begin(), d2.begin() + (min_pts - 1), d2.end());
        cd = std::sqrt(d2[min_pts - 1]);
        return true;
    };
    std::vector<bool> processed(n, false);
    std::vector<double> reach(n, -1.0);
    std::vector<size_t> ordered;
    auto update = [&](int p, double cd, std::set<RD, RDLess> &seeds) {  // :315-337
        for (size_t o : nb[p]) {
            if (processed[o]) continue;
            const double nr = std::max(cd, dist_d(&pts[p * D], &pts[o * D], D));
            if (reach[o] < 0.0) {
                reach[o] = nr;
                seeds.insert(RD{o, nr});
            } else if (nr < reach[o]) {
                seeds.erase(RD{o, reach[o]});
                reach[o] = nr;
                seeds.insert(RD{o, nr});
            }
        }
    };
    for (int p = 0; p < n; ++p) {                                        // :525-555
        if (processed[p]) continue;
        processed[p] = true;
        ordered.push_back(p);
        std::set<RD, RDLess> seeds;
        double cd;
        if (!core(p, cd)) continue;
        update(p, cd, seeds);
        while (!seeds.empty()) {
            const RD s = *seeds.begin();
            seeds.erase(seeds.begin());
            processed[s.idx] = true;
            ordered.push_back(s.idx);
            double scd;
            if (!core((int)s.idx, scd)) continue;
            update((int)s.idx, scd, seeds);
        }
    }
    for (int i = 0; i < n; ++i) {
        order[i] = (int64_t)ordered[i];
        reach_out[i] = reach[ordered[i]];
    }
    return n;
}

// a14: get_cluster_indices, optics.hpp:674-690.  cluster_of[i] = cluster id of ordered entry i.
ORC_API int orc_get_cluster_indices(const double *reach, int n, double thr, int32_t *cluster_of) {
    int c = -1;
    for (int i = 0; i < n; ++i) {
        if (reach[i] < 0.0 || reach[i] >= thr) ++c;
        cluster_of[i] = c < 0 ? 0 : c;
    }
    return c + 1;
}

// a11: radius search semantics of kdt::KDTree::radius_search (kdTree.hpp:218-226: square_distance
// <= r^2, self included) over D-dim double points, as an exact ball.  Returns the count; indices
// ascending in `out` (capacity cap).
ORC_API int orc_radius_search(const double *pts, int n, int D, const double *q, double r, int64_t *out,
                              int cap) {
    const double r2 = r * r;
    int k = 0;
    for (int i = 0; i < n; ++i) {
        double s = 0;
        for (int d = 0; d < D; ++d) { const double dd = pts[i * D + d] - q[d]; s += dd * dd; }
        if (s <= r2) { if (k < cap) out[k] = i; ++k; }
    }
    return k;
}

// Partial sums of one Lloyd iteration over a shard (for the multi-process tests): acc[3k] +=
// (count, sum x, sum y) of the points assigned to each centre (assign_to_centers semantics).
ORC_API int orc_kmeans_partial_xy16(const uint32_t *xy, int64_t n, const float *c, int k, float thr,
                                    int64_t *acc) {
    for (int64_t i = 0; i < n; ++i) {
        const float px = (float)(xy[i] & 0xffffu), py = (float)(xy[i] >> 16);
        const uint8_t a = assign_one(px, py, c, k, thr);
        if (a == 255) continue;
        acc[3 * a] += 1;
        acc[3 * a + 1] += (int64_t)(xy[i] & 0xffffu);
        acc[3 * a + 2] += (int64_t)(xy[i] >> 16);
    }
    return 0;
}

// ------------------------------------------------------------------------------------------
// §8f rank 1: RAW event ingest.  The reference decodes through Metavision::Camera::from_file
// (FCT/…group_track.cpp:756-760), which is not vendored; these are sequential restatements of
// the published EVT 2.0 / EVT 3.0 word formats (include/ecc.h §8) — parity "unpinned" against
// OpenEB itself — plus stream ENCODERS that build test recordings (vector words, trigger /
// OTHERS / CONTINUED words, redundant TIME_HIGH words, 24-bit time loops).
// ------------------------------------------------------------------------------------------
namespace {
struct Rng {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    int pct(int p) { return (int)(next() % 100) < p; }
};
}  // namespace

ORC_API int64_t orc_evt2_decode(const uint32_t *w, int64_t n, uint32_t *xy, int64_t *t, uint8_t *p, int64_t cap) {
    uint32_t th = 0;
    int64_t k = 0;
    for (int64_t i = 0; i < n; ++i) {
        const uint32_t ty = w[i] >> 28;
        if (ty == 0x0 || ty == 0x1) {  // CD_OFF / CD_ON
            if (k < cap) {
                xy[k] = (w[i] >> 11 & 0x7FFu) | ((w[i] & 0x7FFu) << 16);
                t[k] = ((int64_t)th << 6) | (int64_t)(w[i] >> 22 & 0x3Fu);
                p[k] = (uint8_t)ty;
            }
            ++k;
        } else if (ty == 0x8) {  // EVT_TIME_HIGH
            th = w[i] & 0x0FFFFFFFu;
        }
    }
    return k;
}

ORC_API int64_t orc_evt3_decode(const uint16_t *w, int64_t n, uint32_t *xy, int64_t *t, uint8_t *p, int64_t cap) {
    uint32_t y = 0, tl = 0, th = 0, base = 0, pol = 0;
    int64_t loops = 0, k = 0;
    bool has_th = false;
    auto emit = [&](uint32_t x, uint32_t pp) {
        if (k < cap) {
            xy[k] = (x & 0xFFFFu) | (y << 16);
            t[k] = (loops << 24) | (int64_t)(th << 12 | tl);
            p[k] = (uint8_t)pp;
        }
        ++k;
    };
    for (int64_t i = 0; i < n; ++i) {
        const uint32_t v = w[i];
        switch (v >> 12) {
            case 0x0: y = v & 0x7FFu; break;                         // EVT_ADDR_Y
            case 0x2: emit(v & 0x7FFu, v >> 11 & 1u); break;         // EVT_ADDR_X
            case 0x3: base = v & 0x7FFu; pol = v >> 11 & 1u; break;  // VECT_BASE_X
            case 0x4:                                                // VECT_12
                for (int b = 0; b < 12; ++b)
                    if (v >> b & 1u) emit(base + b, pol);
                base += 12;
                break;
            case 0x5:  // VECT_8
                for (int b = 0; b < 8; ++b)
                    if (v >> b & 1u) emit(base + b, pol);
                base += 8;
                break;
            case 0x6: tl = v & 0xFFFu; break;  // EVT_TIME_LOW
            case 0x8: {                        // EVT_TIME_HIGH
                const uint32_t nt = v & 0xFFFu;
                if (has_th && nt < th) ++loops;
                th = nt;
                has_th = true;
                break;
            }
            default: break;  // 0x7 CONTINUED_4, 0xA EXT_TRIGGER, 0xE OTHERS, 0xF CONTINUED_12
        }
    }
    return k;
}

// Noise words that carry no CD event (EXT_TRIGGER / OTHERS / CONTINUED).
static uint32_t evt2_noise(Rng &r) {
    static const uint32_t ty[3] = {0xA, 0xE, 0xF};
    return (ty[r.next() % 3] << 28) | (uint32_t)(r.next() & 0x0FFFFFFFu);
}
static uint16_t evt3_noise(Rng &r) {
    static const uint32_t ty[4] = {0x7, 0xA, 0xE, 0xF};
    return (uint16_t)((ty[r.next() % 4] << 12) | (uint32_t)(r.next() & 0xFFFu));
}

// EVT 2.0 encoder: TIME_HIGH whenever t >> 6 changes (plus redundant repeats), noise_pct %
// extra noise words.  Events need x, y < 2048, non-decreasing t < 2^34.  Returns words.
ORC_API int64_t orc_evt2_encode(const uint32_t *xy, const int64_t *t, const uint8_t *p, int64_t n, uint64_t seed,
                                int noise_pct, uint32_t *out, int64_t cap) {
    Rng r{seed};
    int64_t k = 0;
    auto put = [&](uint32_t v) { if (k < cap) out[k] = v; ++k; };
    int64_t last_th = -1;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t th = t[i] >> 6;
        if (th != last_th || r.pct(noise_pct / 4)) put(0x80000000u | (uint32_t)(th & 0x0FFFFFFF));
        last_th = th;
        while (r.pct(noise_pct)) put(evt2_noise(r));
        const uint32_t x = xy[i] & 0x7FFu, y = (xy[i] >> 16) & 0x7FFu;
        put(((uint32_t)(p[i] & 1) << 28) | ((uint32_t)(t[i] & 63) << 22) | (x << 11) | y);
    }
    return k;
}

// EVT 3.0 encoder, order-preserving: runs of events with equal (t, y, p) and strictly
// increasing x go out as VECT_BASE_X + VECT_12 / VECT_8 words (chosen at random, zero masks
// allowed) when vect_pct allows; single events as EVT_ADDR_X.  TIME_HIGH on every change of
// t >> 12, with (0xFFF, 0) pairs for every 2^24 loop crossed; TIME_LOW on every change of t.
ORC_API int64_t orc_evt3_encode(const uint32_t *xy, const int64_t *t, const uint8_t *p, int64_t n, uint64_t seed,
                                int noise_pct, int vect_pct, uint16_t *out, int64_t cap) {
    Rng r{seed};
    int64_t k = 0;
    auto put = [&](uint32_t v) { if (k < cap) out[k] = (uint16_t)v; ++k; };
    int64_t last_hi = -1, last_t = -1;  // t >> 12
    int64_t last_y = -1;
    int64_t i = 0;
    while (i < n) {
        const int64_t ti = t[i];
        const int64_t hi = ti >> 12;
        if (hi != last_hi || r.pct(noise_pct / 4)) {
            if (last_hi >= 0)
                for (int64_t L = (last_hi >> 12); L < (hi >> 12); ++L) { put(0x8000u | 0xFFFu); put(0x8000u); }
            put(0x8000u | (uint32_t)(hi & 0xFFF));
            last_hi = hi;
            last_t = -1;
        }
        if (ti != last_t || r.pct(noise_pct / 4)) { put(0x6000u | (uint32_t)(ti & 0xFFF)); last_t = ti; }
        const uint32_t y = (xy[i] >> 16) & 0x7FFu, x0 = xy[i] & 0x7FFu, pi = p[i] & 1u;
        if ((int64_t)y != last_y || r.pct(noise_pct / 4)) { put(0x0000u | y); last_y = y; }
        while (r.pct(noise_pct)) put(evt3_noise(r));
        // run of equal (t, y, p) with strictly increasing x, within 64 px of x0
        int64_t j = i + 1;
        while (j < n && t[j] == ti && ((xy[j] >> 16) & 0x7FFu) == y && (p[j] & 1u) == pi &&
               (xy[j] & 0x7FFu) > (xy[j - 1] & 0x7FFu) && (xy[j] & 0x7FFu) < x0 + 64)
            ++j;
        if (j - i >= 2 && r.pct(vect_pct)) {
            put(0x3000u | (pi << 11) | x0);
            uint32_t base = x0;
            int64_t q = i;
            while (q < j) {
                const int nb = r.pct(50) ? 12 : 8;
                uint32_t m = 0;
                while (q < j && (xy[q] & 0x7FFu) < base + nb) { m |= 1u << ((xy[q] & 0x7FFu) - base); ++q; }
                put((nb == 12 ? 0x4000u : 0x5000u) | m);
                base += nb;
            }
            i = j;
        } else {
            put(0x2000u | (pi << 11) | x0);
            ++i;
        }
    }
    return k;
}

// n-µs reslicer (ecc_reslice_n_us semantics): bounds[k] = first event with t >= t_base + k*T.
ORC_API int64_t orc_reslice_n_us(const int64_t *t, int64_t n, int64_t period, int64_t *bounds, int64_t max_slices) {
    if (n == 0) { bounds[0] = 0; return 0; }
    const int64_t t0 = t[0];
    const int64_t base = (t0 >= 0 ? t0 / period : -((-t0 + period - 1) / period)) * period;
    const int64_t ns = (t[n - 1] - base) / period + 1;
    int64_t i = 0;
    for (int64_t k = 0; k < ns && k < max_slices; ++k) {
        while (i < n && t[i] < base + k * period) ++i;
        bounds[k] = i;
    }
    bounds[ns < max_slices ? ns : max_slices] = n;
    return ns;
}

// ------------------------------------------------------------------------------------------
// §8f ranks 2 + 4: AEClustering (DSA/AEClustering.cpp:20-211, DSA/MyCluster.cpp:5-201) fed by
// the downsample slice path (DSA/…opencl_store.cpp:428-445) and the centroid displacement
// (:470-518).  Literal restatement: Eigen::VectorXd(2) -> double[2]; the unqualified abs() on
// doubles binds to int abs(int) (truncation); merge returns before erasing emptied clusters.
// ------------------------------------------------------------------------------------------
namespace {
struct OrcCluster {
    std::deque<int> datId;
    std::deque<std::array<double, 2>> dat;
    std::deque<double> datT;
    std::deque<bool> datPol;
    double alpha = 0.5;
    double mu[2] = {0, 0};
    int n = 0, kappa = 0, id = 0;
    void add(const double *e, int &eventId, double t0) {
        const double t = e[0] - t0;
        datId.push_back(eventId);
        dat.push_back({e[1], e[2]});
        datT.push_back(t);
        datPol.push_back(e[3] != 0);
        if (n == 0) { mu[0] = e[1]; mu[1] = e[2]; }
        else { mu[0] = (1 - alpha) * mu[0] + alpha * e[1]; mu[1] = (1 - alpha) * mu[1] + alpha * e[2]; }
        n++;
        eventId++;
    }
    void forget(double t) {
        while (n > 0 && datT[0] < t) { dat.pop_front(); datId.pop_front(); datT.pop_front(); if (!datPol.empty()) datPol.pop_front(); n--; }
    }
    static double tabs(double v) { return (double)std::abs((int)v); }
    double manhattan(const double *x) const { return (double)((int)tabs(x[0] - mu[0]) + (int)tabs(x[1] - mu[1])); }
    double sampled(const double *x) const {
        double ma = std::numeric_limits<double>::max();
        if (kappa > n) {
            for (const auto &y : dat) { const double f = (double)((int)tabs(x[0] - y[0]) + (int)tabs(x[1] - y[1])); if (f < ma) ma = f; }
        } else {
            for (int ii = 0; ii < kappa; ++ii) {
                const auto &y = dat[std::rand() % (int)dat.size()];
                const double f = (double)((int)tabs(x[0] - y[0]) + (int)tabs(x[1] - y[1]));
                if (f < ma) ma = f;
            }
        }
        return ma;
    }
};

struct OrcAEC {
    int minN = 10, szBuffer = 800, kappa = 0, eventId = 0, lastUpdated = -1, nextId = 0;
    double tMin = 0, radius = 40, alpha = 0.5, t0 = -1;
    std::deque<double> tBuf;
    std::deque<OrcCluster> clusters;
    void merge(const std::deque<int> &as) {
        const int m = (int)as.size();
        std::vector<int> nn(m), cnt(m, 0);
        int aux_n = 0;
        for (int i = 0; i < m; ++i) { nn[i] = clusters[as[i]].n; aux_n += nn[i]; }
        double amu[2] = {0, 0};
        for (int i = 0; i < m; ++i) {
            const double w = (double)clusters[as[i]].n / (double)aux_n;
            amu[0] += w * clusters[as[i]].mu[0];
            amu[1] += w * clusters[as[i]].mu[1];
        }
        std::vector<OrcCluster> src;
        for (int i = 0; i < m; ++i) src.push_back(clusters[as[i]]);
        OrcCluster &d = clusters[as[0]];
        d.datId.clear(); d.dat.clear(); d.datT.clear(); d.datPol.clear();
        for (int idx = 1; idx >= 0;) {
            idx = -1;
            double tt = std::numeric_limits<double>::max();
            for (int j = 0; j < m; ++j)
                if (cnt[j] < nn[j] && src[j].datT[cnt[j]] < tt) { idx = j; tt = src[j].datT[cnt[j]]; }
            if (idx >= 0) {
                d.datId.push_back(src[idx].datId[cnt[idx]]);
                d.dat.push_back(src[idx].dat[cnt[idx]]);
                d.datT.push_back(src[idx].datT[cnt[idx]]);
                d.datPol.push_back(src[idx].datPol[cnt[idx]]);
                cnt[idx]++;
            }
        }
        d.n = (int)d.dat.size();
        d.mu[0] = amu[0];
        d.mu[1] = amu[1];
        for (int i = m - 1; i > 0; --i) clusters.erase(clusters.begin() + as[i]);
    }
    void update(const double *e) {
        if (t0 < 0) t0 = e[0];
        const double t = e[0] - t0;
        tBuf.push_back(t);
        if ((int)tBuf.size() > szBuffer) tBuf.pop_front();
        tMin = tBuf[0];
        std::deque<int> as, rm;
        const double pix[2] = {e[1], e[2]};
        for (int i = 0; i < (int)clusters.size(); ++i) {
            clusters[i].forget(tMin);
            if (clusters[i].n == 0) rm.push_back(i);
            else if (clusters[i].manhattan(pix) <= radius) as.push_back(i);
            else if (clusters[i].n > minN && clusters[i].sampled(pix) <= radius) as.push_back(i);
        }
        if (as.empty()) {
            OrcCluster c;
            c.alpha = alpha;
            c.kappa = kappa;
            clusters.push_back(c);
            clusters.back().add(e, eventId, t0);
            clusters.back().id = nextId++;
            lastUpdated = (int)clusters.size() - 1;
        } else {
            lastUpdated = as[0];
            clusters[as[0]].add(e, eventId, t0);
            if (as.size() >= 2) { merge(as); return; }
        }
        for (int i = (int)rm.size() - 1; i >= 0; --i) {
            if (lastUpdated > rm[i]) lastUpdated--;
            clusters.erase(clusters.begin() + rm[i]);
        }
    }
};
}  // namespace

// rows (8 doubles each): window, cluster id, n, centroid x, y, has_prev, flow dx, dy — for the
// clusters with n >= minN after each window, in cluster-deque order.  Returns the row count.
ORC_API int64_t orc_aec_run(const uint32_t *rep_xy, const int32_t *win_unique, int64_t n_windows, int64_t stride,
                            int szBuffer, double radius, int kappa, double alpha, int minN, double *rows,
                            int64_t cap, int32_t *clusters_per_window) {
    OrcAEC ae;
    ae.szBuffer = szBuffer; ae.radius = radius; ae.kappa = kappa; ae.alpha = alpha; ae.minN = minN;
    std::vector<std::array<double, 2>> prev(16384, {0.0, 0.0});  // double centroid_prev[16384][2]
    int64_t k = 0, cumulative = 0;
    for (int64_t w = 0; w < n_windows; ++w) {
        const int diff = win_unique[w];
        cumulative += diff;
        for (int i = 0; i < diff; i += 4) {  // uniqueCoords[i], [i+1] of the interleaved ints
            const uint32_t v = rep_xy[w * stride + i / 2];
            const double e[4] = {(double)cumulative / 1000.0, (double)(v & 0xffff), (double)(v >> 16), 0.0};
            ae.update(e);
        }
        clusters_per_window[w] = (int32_t)ae.clusters.size();
        for (const auto &c : ae.clusters) {
            if (c.n < ae.minN) continue;
            double xa = 0, ya = 0;
            for (const auto &p : c.dat) { xa = xa + p[0]; ya = ya + p[1]; }
            xa = xa / (double)c.dat.size();
            ya = ya / (double)c.dat.size();
            int id = c.id;
            if (id > 16384) id %= 16384;
            auto &pv = prev[id % 16384];
            const double row[8] = {(double)w, (double)c.id, (double)c.n, xa, ya,
                                   (pv[0] > 0 && pv[1] > 0) ? 1.0 : 0.0, xa - pv[0], ya - pv[1]};
            if (k < cap) std::memcpy(rows + 8 * k, row, sizeof(row));
            ++k;
            pv = {xa, ya};
        }
    }
    return k;
}
