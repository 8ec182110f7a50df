// OpenMP all-cores variant of the oracle's embarrassingly parallel stages — TEST / BASELINE
// INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg; never the product path).
//
// the CPU baseline also times the build's restatement on all host cores for
// the stages that parallelise: the downsample windows (independent), the k-means assignment
// (per point; integer-valued coordinate sums in fp64 are exact in any order, so the centroids are
// the single-thread oracle's bit for bit), the per-slice arc tests on the batch SAE (the SAE
// update stays sequential per slice — last writer in stream order, :900-923 — the slice's tests
// are independent), and NMS (slices are independent).  Every function returns what its oracle.cpp
// counterpart returns for the same arguments.
#include "oracle.cpp"

#include <omp.h>

ORC_API int omp_threads() { return omp_get_max_threads(); }

ORC_API int omp_downsample_hash(const uint32_t *xy, int64_t n, int window, int x_max, int y_max, int mult_x,
                                int mult_y, int n_buckets, uint32_t *rep_xy, uint32_t *rep_idx, int32_t *win_unique,
                                int32_t *win_repeated) {
    if (window <= 0 || n_buckets <= 0 || n < 0) return -1;
    const int64_t n_win = (n + window - 1) / window;
#pragma omp parallel
    {
        std::vector<int> map(n_buckets);  // one bucket table per thread, cleared per window (:35-44)
#pragma omp for schedule(dynamic, 16)
        for (int64_t w = 0; w < n_win; ++w) {
            std::fill(map.begin(), map.end(), 0);
            int unique = 0, repeated = 0;
            const int64_t lo = w * window, hi = std::min<int64_t>(n, lo + window);
            for (int64_t i = lo; i < hi; ++i) {  // same body as orc_downsample_hash
                const int x = (int)(xy[i] & 0xffffu), y = (int)(xy[i] >> 16);
                if (x >= 0 && x <= x_max && y >= 0 && y <= y_max) {
                    const int prev = map[(x * mult_x + y * mult_y) % n_buckets]++;
                    if (prev == 0) {
                        if (rep_xy) rep_xy[lo + unique] = xy[i];
                        if (rep_idx) rep_idx[lo + unique] = (uint32_t)i;
                        ++unique;
                    } else if (prev == 1) {
                        ++repeated;
                    }
                }
            }
            if (win_unique) win_unique[w] = unique;
            if (win_repeated) win_repeated[w] = repeated;
        }
    }
    return 0;
}

ORC_API int omp_kmeans_run_xy16(const uint32_t *xy, int64_t n, float *c, int k, int max_iters, float thr, float tol,
                                uint8_t *labels, int32_t *iters_out) {
    const int nt = omp_get_max_threads();
    std::vector<double> sx((size_t)nt * k), sy((size_t)nt * k);
    std::vector<int64_t> cnt((size_t)nt * k);
    int it = 0;
    for (; it < max_iters;) {
        std::fill(sx.begin(), sx.end(), 0.0);
        std::fill(sy.begin(), sy.end(), 0.0);
        std::fill(cnt.begin(), cnt.end(), 0);
#pragma omp parallel
        {
            const int th = omp_get_thread_num();
            double *tx = &sx[(size_t)th * k], *ty = &sy[(size_t)th * k];
            int64_t *tc = &cnt[(size_t)th * k];
#pragma omp for schedule(static)
            for (int64_t i = 0; i < n; ++i) {
                const float px = (float)(xy[i] & 0xffffu), py = (float)(xy[i] >> 16);
                const uint8_t a = assign_one(px, py, c, k, thr);
                if (a == 255) continue;
                tx[a] += px;
                ty[a] += py;
                tc[a] += 1;
            }
        }
        float shift = 0.f;
        for (int j = 0; j < k; ++j) {
            double x = 0.0, y = 0.0;
            int64_t m = 0;
            for (int th = 0; th < nt; ++th) {
                x += sx[(size_t)th * k + j];
                y += sy[(size_t)th * k + j];
                m += cnt[(size_t)th * k + j];
            }
            if (m == 0) continue;
            const float nx = (float)(x / (double)m), ny = (float)(y / (double)m);
            shift = std::max(shift, std::max(std::fabs(nx - c[2 * j]), std::fabs(ny - c[2 * j + 1])));
            c[2 * j] = nx;
            c[2 * j + 1] = ny;
        }
        ++it;
        if (tol >= 0.f && shift <= tol) break;
    }
    if (labels) {
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; ++i)
            labels[i] = assign_one((float)(xy[i] & 0xffffu), (float)(xy[i] >> 16), c, k, thr);
    }
    if (iters_out) *iters_out = it;
    return 0;
}

ORC_API int omp_fast_detect(const uint32_t *xy, const int64_t *t, int64_t n, int W, int H, int slice, int margin,
                            int border_mode, int first_detect, int64_t *sae, uint8_t *flags) {
    if (slice <= 0 || W <= 2 * margin || H <= 2 * margin) return -1;
    if (border_mode != 0) return orc_fast_detect(xy, t, n, W, H, slice, margin, border_mode, first_detect, sae, flags);
    const int64_t n_slices = (n + slice - 1) / slice;
    for (int64_t s = 0; s < n_slices; ++s) {
        const int64_t lo = s * slice, hi = std::min<int64_t>(n, lo + slice);
        for (int64_t e = lo; e < hi; ++e) {  // :900-923, sequential: last writer wins
            const int x = (int)(xy[e] & 0xffffu), y = (int)(xy[e] >> 16);
            if (x < W && y < H) sae[(int64_t)y * W + x] = t[e];
        }
        const bool detect = s >= first_detect;
#pragma omp parallel for schedule(static)
        for (int64_t e = lo; e < hi; ++e) {
            const int x = (int)(xy[e] & 0xffffu), y = (int)(xy[e] >> 16);
            flags[e] = (detect && !(x < margin || x >= W - margin || y < margin || y >= H - margin))
                           ? (uint8_t)orc_arc_test(sae, W, x, y) : (uint8_t)0;
        }
    }
    return 0;
}

ORC_API int omp_corner_nms(const uint32_t *xy, const uint8_t *flags, int64_t n, int slice, int W, int H, int box,
                           int cap, ecc_corner *out, int32_t *counts) {
    const int64_t n_slices = (n + slice - 1) / slice;
    int rc = 0;
#pragma omp parallel for schedule(dynamic, 8) reduction(| : rc)
    for (int64_t s = 0; s < n_slices; ++s) {
        const int64_t lo = s * slice, len = std::min<int64_t>(slice, n - lo);
        rc |= orc_corner_nms(xy + lo, flags + lo, len, slice, W, H, box, cap, out + s * cap, counts + s) < 0 ? 1 : 0;
    }
    return rc ? -4 : 0;
}
