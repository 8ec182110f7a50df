// Corner tracker: damped predictor-corrector with grouping.
//
// Reference: class CornerTracker, FCT/metavision_time_surface_periodic_group_track.cpp:201-537
// (the "Luenberger observer" of the README is this fixed-gain predictor-corrector: direction
// damping 0.8, velocity/direction blend 0.3, group-velocity blend 0.3).  It runs on the CPU
// once per 16384-event slice (:847), O(T*C) matching + O(T^2) grouping.
//
// MI355X design: the whole multi-slice update runs in ONE launch of one workgroup (a single
// wave64 — the algorithm is order-dependent: greedy matching in track order, greedy grouping
// in seed order), so a batch of slices costs one kernel instead of one host round trip each.
// Parallel phases use one lane per track / per detection (prediction, state update, new-track
// creation with ballot prefix sums, stable erase by compaction into a ping-pong buffer, group
// membership tests, velocity blend); the sequential phases (match claim per track, member
// sums per group) keep the reference's order.  Every fp32 expression is written in the
// reference's operation order and compiled without FMA contraction, so positions, velocities
// and directions are bit-identical to oracle/oracle.cpp (std::pow(0.8f, i-1) is a host-side
// table, :254).
#include "ecc_internal.hpp"

#include <cmath>
#include <vector>

namespace {

constexpr int kLanes = 64;
constexpr int kH = ECC_TRACK_HIST_MAX;
constexpr int kMaxDet = 4096;  // detections per slice held in LDS

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
    int32_t n_tracks, next_label, cur, n_groups, n_group_labels, err, pad0, pad1;
};

struct TrackerParams {
    float max_distance, damping, smoothing, group_radius;
    int max_frames, history, frames_to_skip;
    float pow_tab[kH + 1];
};

struct F2 { float x, y; };
__device__ __forceinline__ F2 add(F2 a, F2 b) { return F2{__fadd_rn(a.x, b.x), __fadd_rn(a.y, b.y)}; }
__device__ __forceinline__ F2 mul(F2 a, float s) { return F2{__fmul_rn(a.x, s), __fmul_rn(a.y, s)}; }
__device__ __forceinline__ float dist(F2 a, F2 b) {  // :217-222
    const float dx = __fsub_rn(a.x, b.x), dy = __fsub_rn(a.y, b.y);
    return ecc::sqrt_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)));
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

__global__ void __launch_bounds__(kLanes)
tracker_kernel(DevTrack *__restrict__ buf0, DevTrack *__restrict__ buf1, int max_tracks,
               DevGroup *__restrict__ groups, int *__restrict__ group_labels,
               uint8_t *__restrict__ work, TrackerCounters *__restrict__ ctr, TrackerParams p,
               const ecc_corner *__restrict__ corners, const int32_t *__restrict__ counts,
               int n_slices, int cap) {
    __shared__ int s_dx[kMaxDet], s_dy[kMaxDet];
    __shared__ uint8_t s_dmatched[kMaxDet];
    const int lane = threadIdx.x;
    // per-track scratch in global memory: pred x/y, best match, processed flag
    float *w_px = reinterpret_cast<float *>(work);
    float *w_py = w_px + max_tracks;
    int *w_best = reinterpret_cast<int *>(w_py + max_tracks);
    uint8_t *w_proc = reinterpret_cast<uint8_t *>(w_best + max_tracks);

    int T = ctr->n_tracks, next_label = ctr->next_label, cur = ctr->cur, err = ctr->err;
    int n_groups = 0, n_glabels = 0;
    for (int s = 0; s < n_slices; ++s) {
        DevTrack *A = cur ? buf1 : buf0;  // active tracks
        DevTrack *Bf = cur ? buf0 : buf1; // compaction target
        int C = counts[s];
        if (C > cap) C = cap;
        if (C > kMaxDet) { C = kMaxDet; err = ECC_ERR_CAPACITY; }
        for (int d = lane; d < C; d += kLanes) {
            const ecc_corner c = corners[(int64_t)s * cap + d];
            s_dx[d] = c.x;
            s_dy[d] = c.y;
            s_dmatched[d] = 0;
        }
        // 1. prediction for every active track (:451) + reset is_matched (:438-441)
        for (int i = lane; i < T; i += kLanes) {
            const F2 pp = predict(A[i], p);
            w_px[i] = pp.x;
            w_py[i] = pp.y;
            A[i].is_matched = 0;
        }
        __syncthreads();
        // 2. greedy matching in track order (:446-487): first nearest unmatched with dist < max
        for (int i = 0; i < T; ++i) {
            const bool skip = A[i].fsld > p.frames_to_skip;
            const F2 pp{w_px[i], w_py[i]};
            float bd = p.max_distance;
            int bi = 0x7fffffff;
            if (!skip) {
                for (int d = lane; d < C; d += kLanes) {
                    if (s_dmatched[d]) continue;
                    const float dd = dist(pp, F2{(float)s_dx[d], (float)s_dy[d]});
                    if (dd < bd) { bd = dd; bi = d; }
                }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const float ob = __shfl_xor(bd, o);
                const int oi = __shfl_xor(bi, o);
                if (ob < bd || (ob == bd && oi < bi)) { bd = ob; bi = oi; }
            }
            if (lane == 0) {
                w_best[i] = skip ? -2 : (bi == 0x7fffffff ? -1 : bi);
                if (!skip && bi != 0x7fffffff) s_dmatched[bi] = 1;
            }
            __syncthreads();
        }
        // 3. update matched / missed tracks (:471-497)
        for (int i = lane; i < T; i += kLanes) {
            const int b = w_best[i];
            if (b == -2) continue;
            DevTrack t = A[i];
            if (b >= 0) {
                t.x = s_dx[b];
                t.y = s_dy[b];
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
            } else {
                t.x = (int)w_px[i];                                    // Q16 truncation
                t.y = (int)w_py[i];
                t.fsld++;
                push_hist(t, p.history);
                const F2 v = estimate_velocity(t, p);
                t.vx = v.x;
                t.vy = v.y;
            }
            A[i] = t;
        }
        __syncthreads();
        // 4. new tracks for unmatched detections, in detection order (:501-514)
        for (int d0 = 0; d0 < C; d0 += kLanes) {
            const int d = d0 + lane;
            const bool nw = d < C && !s_dmatched[d];
            const uint64_t m = __ballot(nw);
            const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
            const int slot = T + __popcll(m & lt);
            if (nw) {
                if (slot < max_tracks) {
                    DevTrack t;
                    t.x = s_dx[d];
                    t.y = s_dy[d];
                    t.label = next_label + __popcll(m & lt);
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
                    A[slot] = t;
                } else {
                    err = ECC_ERR_CAPACITY;
                }
            }
            const int added = __popcll(m);
            next_label += added;
            T = min(T + added, max_tracks);
        }
        __syncthreads();
        // 5. stable erase of lost / expired tracks (:517-526) into the other buffer
        int T2 = 0;
        for (int i0 = 0; i0 < T; i0 += kLanes) {
            const int i = i0 + lane;
            bool keep = false;
            if (i < T) keep = !(A[i].fsld > p.frames_to_skip || A[i].frame_count > p.max_frames);
            const uint64_t m = __ballot(keep);
            const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
            if (keep) Bf[T2 + __popcll(m & lt)] = A[i];
            T2 += __popcll(m);
        }
        T = T2;
        cur ^= 1;
        DevTrack *R = Bf;  // now the active buffer
        __syncthreads();
        // 6. greedy grouping in seed order (:321-398)
        for (int i = lane; i < T; i += kLanes) w_proc[i] = 0;
        __syncthreads();
        n_groups = 0;
        n_glabels = 0;
        for (int i = 0; i < T; ++i) {
            if (w_proc[i] || R[i].fsld > 0) continue;          // uniform: all lanes read the same
            const F2 pi{(float)R[i].x, (float)R[i].y};
            // membership: unprocessed, detected this slice, within radius (self included)
            int cnt = 0;
            F2 sp{0.f, 0.f}, sv{0.f, 0.f};
            const int gid = n_groups;
            for (int j0 = 0; j0 < T; j0 += kLanes) {
                const int j = j0 + lane;
                bool mem = false;
                if (j < T && !w_proc[j] && R[j].fsld == 0)
                    mem = dist(pi, F2{(float)R[j].x, (float)R[j].y}) <= p.group_radius;
                uint64_t m = __ballot(mem);
                int mx = 0, my = 0, mlab = 0;
                float mvx = 0.f, mvy = 0.f;
                if (mem) {
                    w_proc[j] = 1;
                    R[j].group_id = gid;
                    mx = R[j].x; my = R[j].y; mlab = R[j].label;
                    mvx = R[j].vx; mvy = R[j].vy;
                }
                // ordered fp32 sums over members (j ascending), evaluated redundantly per lane
                while (m) {
                    const int l = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1;
                    const int xj = __shfl(mx, l), yj = __shfl(my, l), lab = __shfl(mlab, l);
                    const float vxj = __shfl(mvx, l), vyj = __shfl(mvy, l);
                    sp = add(sp, F2{(float)xj, (float)yj});
                    sv = add(sv, F2{vxj, vyj});
                    if (lane == 0 && n_glabels + cnt < max_tracks) group_labels[n_glabels + cnt] = lab;
                    cnt++;
                }
            }
            __syncthreads();
            if (cnt > 0) {
                const F2 cen = mul(sp, __fdiv_rn(1.0f, (float)cnt));
                const F2 av = mul(sv, __fdiv_rn(1.0f, (float)cnt));
                // radius = max distance of the group's members to the centroid
                float mr = 0.f;
                for (int j = lane; j < T; j += kLanes)
                    if (R[j].fsld == 0 && R[j].group_id == gid && w_proc[j])
                        mr = fmaxf(mr, dist(F2{(float)R[j].x, (float)R[j].y}, cen));
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) mr = fmaxf(mr, __shfl_xor(mr, o));
                if (lane == 0 && gid < max_tracks)
                    groups[gid] = DevGroup{gid, cnt, n_glabels, av.x, av.y, cen.x, cen.y, mr};
                n_glabels += cnt;
                n_groups++;
            }
            __syncthreads();
        }
        // velocity blend with the group average (:388-397)
        for (int i = lane; i < T; i += kLanes) {
            if (R[i].fsld == 0 && R[i].group_id >= 0 && R[i].group_id < n_groups) {
                const DevGroup &g = groups[R[i].group_id];
                R[i].vx = __fadd_rn(__fmul_rn(R[i].vx, 0.7f), __fmul_rn(g.avx, 0.3f));
                R[i].vy = __fadd_rn(__fmul_rn(R[i].vy, 0.7f), __fmul_rn(g.avy, 0.3f));
            }
        }
        __syncthreads();
    }
    const bool any_err = __any(err != 0);
    if (lane == 0) {
        if (any_err && err == 0) err = ECC_ERR_CAPACITY;
        ctr->n_tracks = T;
        ctr->next_label = next_label;
        ctr->cur = cur;
        ctr->n_groups = n_groups;
        ctr->n_group_labels = n_glabels;
        ctr->err = err;
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
    uint8_t *work = nullptr;
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
        max_detections > kMaxDet || cfg->history_size < 1 || cfg->history_size > kH ||
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
    hipSetDevice(ctx->device);
    const size_t tb = sizeof(DevTrack) * (size_t)max_tracks;
    bool ok = hipMalloc(&tr->buf[0], tb) == hipSuccess && hipMalloc(&tr->buf[1], tb) == hipSuccess &&
              hipMalloc(&tr->groups, sizeof(DevGroup) * (size_t)max_tracks) == hipSuccess &&
              hipMalloc(&tr->group_labels, sizeof(int) * (size_t)max_tracks) == hipSuccess &&
              hipMalloc(&tr->work, (size_t)max_tracks * 16 + 256) == hipSuccess &&
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
    hipFree(tr->work);
    hipFree(tr->ctr);
    delete tr;
    return ECC_OK;
}

ECC_API int ecc_tracker_update(ecc_tracker *tr, const ecc_corner *corners, const int32_t *counts,
                               int32_t n_slices, int32_t cap, ecc_stream_t stream) {
    if (!tr || n_slices < 0 || cap < 0) return ECC_ERR_INVALID;
    if (n_slices == 0) return ECC_OK;
    if (!counts || (cap > 0 && !corners)) return ECC_ERR_INVALID;
    ecc_ctx *ctx = tr->ctx;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    {
        ECC_TIMED(ctx, ecc::as_stream(stream), "tracker_kernel");
        hipLaunchKernelGGL(tracker_kernel, dim3(1), dim3(kLanes), 0, ecc::as_stream(stream),
                           tr->buf[0], tr->buf[1], tr->max_tracks, tr->groups, tr->group_labels,
                           tr->work, tr->ctr, tr->params, corners, counts, n_slices,
                           cap < tr->max_det ? cap : tr->max_det);
    }
    ECC_CHECK_LAUNCH(ctx, "tracker_kernel");
    return ECC_OK;
}

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
