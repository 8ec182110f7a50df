// The time-window-sharded step of BASELINE config C5 as a native host program: one process per
// GPU, RCCL over xGMI through libecc's ecc_dist_* entry points (no Python, no torch.distributed).
//
//   ecc_sharded_step --ranks N [--events n_per_rank] [--steps K] [--warmup W] [--width 346]
//                    [--height 260] [--k 16] [--iters 10] [--dump DIR]
//
// The launcher forks N rank processes BEFORE anything touches the GPU (each rank initialises its
// own device); rank 0 creates the RCCL unique id and hands it to the others through pipes.  Rank
// r owns events [r*n, (r+1)*n) of the seeded synthetic stream (the same stream bench.py
// shards).  Per step:
//   downsample -> per-pixel count image -> ecc_dist_allreduce_counts -> Lloyd passes over the
//   global image -> labels                                           (global centroids, exact)
//   prepare -> ecc_dist_sae_handoff -> finish + NMS                  (exact SAE hand-off)
// After the timed steps: corner pack -> ecc_dist_gather_corners -> ONE tracker on rank 0 over
// the global slice order (the reference's slice loop, FCT/…group_track.cpp:832-850).
// Rank 0 prints one JSON line; --dump writes every rank's corner flags, final SAE and NMS lists
// and rank 0's centroids, labels and merged tracks (tests/test_dist_native.py checks them
// against the oracle).
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "app_common.hpp"

namespace {

constexpr int32_t kSlice = 16384, kWindow = 8192, kCap = 4096;

#define CK(call)                                                                                         \
    do {                                                                                                 \
        int _rc = (call);                                                                                \
        if (_rc != ECC_OK) {                                                                             \
            std::fprintf(stderr, "rank %d: %s failed: %s (%s)\n", g_rank, #call, ecc_status_string(_rc),      \
                         g_ctx ? ecc_ctx_last_error(g_ctx) : "");                                        \
            std::exit(1);                                                                                \
        }                                                                                                \
    } while (0)

int g_rank = 0;
ecc_ctx *g_ctx = nullptr;

struct Dev {
    void *p = nullptr;
    size_t bytes = 0;
    explicit Dev(size_t b) : bytes(b) { CK(ecc_dev_alloc(&p, b ? b : 16)); }
    ~Dev() { ecc_dev_free(p); }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

void dump(const std::string &dir, const std::string &name, const void *dev, size_t bytes, ecc_stream_t s) {
    std::vector<char> h(bytes);
    if (bytes) CK(ecc_memcpy_d2h(h.data(), dev, bytes, s));
    CK(ecc_stream_sync(s));
    FILE *f = std::fopen((dir + "/" + name).c_str(), "wb");
    if (!f) {
        std::perror(name.c_str());
        std::exit(1);
    }
    if (bytes) std::fwrite(h.data(), 1, bytes, f);
    std::fclose(f);
}

int run_rank(int rank, int n_ranks, const uint8_t *id, int argc, char **argv) {
    g_rank = rank;
    const int64_t n = opt_int(argc, argv, "--events", 40 * kSlice);
    const int steps = opt_int(argc, argv, "--steps", 5), warmup = opt_int(argc, argv, "--warmup", 2);
    const int W = opt_int(argc, argv, "--width", 346), H = opt_int(argc, argv, "--height", 260);
    const int K = opt_int(argc, argv, "--k", 16), iters = opt_int(argc, argv, "--iters", 10);
    std::string dir;
    for (int i = 1; i + 1 < argc; ++i)
        if (!std::strcmp(argv[i], "--dump")) dir = argv[i + 1];
    if (n <= 0 || n % kSlice) {
        std::fprintf(stderr, "--events must be a positive multiple of %d\n", kSlice);
        return 2;
    }
    int n_dev = 0;
    CK(ecc_device_count(&n_dev));
    if (n_dev < 1) return 3;
    CK(ecc_ctx_create(&g_ctx, rank % n_dev));
    ecc_ctx *ctx = g_ctx;
    ecc_stream_t s = nullptr, s2 = nullptr;
    CK(ecc_stream_create(&s));
    CK(ecc_stream_create(&s2));  // the k-means chain's stream
    void *ev_fork = nullptr, *ev_join = nullptr, *ev_cnt = nullptr, *ev_ar = nullptr;
    for (void **e : {&ev_fork, &ev_join, &ev_cnt, &ev_ar}) CK(ecc_event_create(e));
    ecc_dist *d = nullptr;
    CK(ecc_dist_init(&d, ctx, id, n_ranks, rank));

    // this rank's time window of the seeded stream (bench.py: gen_events(n, first=rank*n, seed=1))
    ecc_gen_cfg gc;
    ecc_gen_cfg_default(&gc);
    gc.seed = 1;
    gc.width = W;
    gc.height = H;
    std::vector<uint32_t> xy(n);
    std::vector<int64_t> t(n);
    CK(ecc_gen_events(&gc, (int64_t)rank * n, n, xy.data(), t.data(), nullptr));
    Dev d_xy(n * 4), d_t(n * 8);
    CK(ecc_memcpy_h2d(d_xy.p, xy.data(), n * 4, s));
    CK(ecc_memcpy_h2d(d_t.p, t.data(), n * 8, s));

    const int64_t n_win = (n + kWindow - 1) / kWindow, ns = n / kSlice, HW = (int64_t)W * H;
    Dev rep_xy(n_win * kWindow * 4), uniq(n_win * 4), rep(n_win * 4), labels(n_win * kWindow);
    Dev counts(HW * 4), local(HW * 8), all(n_ranks * HW * 8), sae(HW * 8), flags(n);
    Dev c0(K * 8), cen(K * 8), nms_out(ns * kCap * sizeof(ecc_corner)), nms_cnt(ns * 4);
    std::vector<float> hc0(2 * K);
    // bench.py's initial centres, np.linspace(20, W - 20, K) against np.linspace(20, H - 20, K)
    // reversed, evaluated as numpy does (i * step + start, the last point exactly `stop`)
    auto lin = [K](double a, double b, int i) {
        return K == 1 ? a : (i == K - 1 ? b : i * ((b - a) / (K - 1)) + a);
    };
    for (int j = 0; j < K; ++j) {
        hc0[2 * j] = (float)lin(20.0, W - 20.0, j);
        hc0[2 * j + 1] = (float)lin(20.0, H - 20.0, K - 1 - j);
    }
    CK(ecc_memcpy_h2d(c0.p, hc0.data(), K * 8, s));
    ecc_hash_cfg hcfg;
    ecc_hash_cfg_default(&hcfg);
    hcfg.window = kWindow;
    ecc_kmeans_cfg kcfg;
    ecc_kmeans_cfg_default(&kcfg);
    kcfg.k = K;
    kcfg.max_iters = iters;
    kcfg.tol = -1.0f;
    ecc_corner_cfg ccfg;
    ecc_corner_cfg_default(&ccfg);
    ccfg.width = W;
    ccfg.height = H;
    ccfg.first_detect_slice = rank == 0 ? 1 : 0;  // Q15: only the stream's first slice is skipped

    auto step = [&]() {
        // k-means chain on s2, detection chain and the collectives on s
        CK(ecc_event_record(ev_fork, s));
        CK(ecc_stream_wait_event(s2, ev_fork));
        CK(ecc_downsample_hash(ctx, d_xy.as<uint32_t>(), n, &hcfg, rep_xy.as<uint32_t>(), nullptr,
                               uniq.as<int32_t>(), rep.as<int32_t>(), s2));
        CK(ecc_kmeans_counts_xy16(ctx, rep_xy.as<uint32_t>(), n_win, kWindow, uniq.as<int32_t>(), W, H,
                                  counts.as<uint32_t>(), s2));
        CK(ecc_event_record(ev_cnt, s2));
        CK(ecc_fast_detect_prepare(ctx, d_xy.as<uint32_t>(), d_t.as<int64_t>(), n, &ccfg, local.as<int64_t>(), s));
        // both collectives on ONE stream, in the same order on every rank (operations of one
        // communicator must not overlap): counts, then the SAE images
        CK(ecc_stream_wait_event(s, ev_cnt));
        CK(ecc_dist_allreduce_counts(d, counts.as<uint32_t>(), HW, s));
        CK(ecc_event_record(ev_ar, s));
        CK(ecc_dist_sae_handoff(d, local.as<int64_t>(), HW, all.as<int64_t>(), sae.as<int64_t>(), s));
        CK(ecc_stream_wait_event(s2, ev_ar));
        CK(ecc_memcpy_d2d(cen.p, c0.p, K * 8, s2));
        CK(ecc_kmeans_run_counts(ctx, counts.as<uint32_t>(), W, H, &kcfg, cen.as<float>(), nullptr, s2));
        CK(ecc_kmeans_labels_xy16(ctx, rep_xy.as<uint32_t>(), n_win, kWindow, uniq.as<int32_t>(), cen.as<float>(), K,
                                  kcfg.threshold, labels.as<uint8_t>(), s2));
        CK(ecc_event_record(ev_join, s2));
        CK(ecc_fast_detect_finish_nms(ctx, d_xy.as<uint32_t>(), d_t.as<int64_t>(), n, &ccfg, sae.as<int64_t>(),
                                      flags.as<uint8_t>(), 15, kCap, nms_out.as<ecc_corner>(), nms_cnt.as<int32_t>(),
                                      s));
        CK(ecc_stream_wait_event(s, ev_join));
    };
    Dev tbuf(8);
    auto barrier = [&]() {  // a 1-element all-reduce on the stream, then a host sync
        CK(ecc_dist_allreduce_f64_max(d, tbuf.as<double>(), 1, s));
        CK(ecc_stream_sync(s));
    };
    for (int i = 0; i < warmup; ++i) step();
    CK(ecc_stream_sync(s));
    CK(ecc_fast_detect_status(ctx, s));
    CK(ecc_corner_nms_status(ctx, s));
    CK(ecc_kmeans_counts_status(ctx, s));
    barrier();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < steps; ++i) step();
    CK(ecc_stream_sync(s));
    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    CK(ecc_memcpy_h2d(tbuf.p, &el, 8, s));
    CK(ecc_dist_allreduce_f64_max(d, tbuf.as<double>(), 1, s));  // the slowest rank's time
    CK(ecc_memcpy_d2h(&el, tbuf.p, 8, s));
    CK(ecc_stream_sync(s));

    // track merge over the last step's lists: pack -> gather in rank order -> ONE tracker (rank 0)
    Dev packed(ns * kCap * sizeof(ecc_corner)), offs((ns + 1) * 8);
    CK(ecc_corner_pack(ctx, nms_out.as<ecc_corner>(), nms_cnt.as<int32_t>(), (int32_t)ns, kCap,
                       packed.as<ecc_corner>(), offs.as<int64_t>(), s));
    int64_t ns_tot = 0, stride = 0;
    const auto tg = std::chrono::steady_clock::now();
    CK(ecc_dist_gather_corners(d, packed.as<ecc_corner>(), offs.as<int64_t>(), (int32_t)ns, nullptr, 0, nullptr, nullptr,
                               0, &ns_tot, &stride, s));
    Dev g_all(n_ranks * stride * sizeof(ecc_corner)), g_starts(ns_tot * 8), g_counts(ns_tot * 4);
    CK(ecc_dist_gather_corners(d, packed.as<ecc_corner>(), offs.as<int64_t>(), (int32_t)ns, g_all.as<ecc_corner>(),
                               n_ranks * stride, g_starts.as<int64_t>(), g_counts.as<int32_t>(), ns_tot, &ns_tot,
                               &stride, s));
    CK(ecc_stream_sync(s));
    const double gather_ms = std::chrono::duration<double>(std::chrono::steady_clock::now() - tg).count() * 1e3;
    int32_t n_tracks = 0;
    double track_ms = 0.0;
    std::vector<ecc_track> tracks(4096);
    if (rank == 0) {
        ecc_tracker_cfg tcfg;
        ecc_tracker_cfg_default(&tcfg);
        ecc_tracker *tr = nullptr;
        CK(ecc_tracker_create(ctx, &tcfg, 4096, 4096, &tr));
        const auto tt = std::chrono::steady_clock::now();
        CK(ecc_tracker_update_lists(tr, g_all.as<ecc_corner>(), g_starts.as<int64_t>(), g_counts.as<int32_t>(),
                                    (int32_t)ns_tot, s));
        CK(ecc_stream_sync(s));
        track_ms = std::chrono::duration<double>(std::chrono::steady_clock::now() - tt).count() * 1e3;
        CK(ecc_tracker_status(tr, s));
        CK(ecc_tracker_get_tracks(tr, tracks.data(), (int32_t)tracks.size(), &n_tracks, s));
        ecc_tracker_destroy(tr);
    }
    if (!dir.empty()) {
        const std::string r = std::to_string(rank);
        dump(dir, "flags_" + r + ".bin", flags.p, n, s);
        dump(dir, "sae_" + r + ".bin", sae.p, HW * 8, s);
        dump(dir, "nms_cnt_" + r + ".bin", nms_cnt.p, ns * 4, s);
        dump(dir, "nms_out_" + r + ".bin", nms_out.p, ns * kCap * sizeof(ecc_corner), s);
        dump(dir, "centroids_" + r + ".bin", cen.p, K * 8, s);
        dump(dir, "uniq_" + r + ".bin", uniq.p, n_win * 4, s);
        dump(dir, "labels_" + r + ".bin", labels.p, n_win * kWindow, s);
        if (rank == 0) {
            FILE *f = std::fopen((dir + "/tracks.bin").c_str(), "wb");
            if (f) {
                std::fwrite(tracks.data(), sizeof(ecc_track), n_tracks, f);
                std::fclose(f);
            }
        }
    }
    if (rank == 0)
        std::printf("{\"metric\": \"Mevents/s (downsample+cluster+corner)\", \"value\": %.2f, \"unit\": \"Mevents/s\", "
                    "\"n_ranks\": %d, \"events_per_rank\": %lld, \"events_total\": %lld, \"steps\": %d, "
                    "\"ms_per_step\": %.4f, \"transport\": \"RCCL (ecc_dist_*, native)\", "
                    "\"track_merge\": {\"slices\": %lld, \"corners_stride\": %lld, \"gather_ms\": %.3f, "
                    "\"tracker_ms\": %.3f, \"tracks_end\": %d}}\n",
                    (double)n_ranks * steps * n / el / 1e6, n_ranks, (long long)n, (long long)n * n_ranks, steps,
                    el / steps * 1e3, (long long)ns_tot, (long long)stride, gather_ms, track_ms, n_tracks);
    std::fflush(stdout);
    ecc_dist_destroy(d);
    for (void *e : {ev_fork, ev_join, ev_cnt, ev_ar}) ecc_event_destroy(e);
    ecc_stream_destroy(s2);
    ecc_stream_destroy(s);
    ecc_ctx_destroy(ctx);
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    const int n_ranks = opt_int(argc, argv, "--ranks", 1);
    if (n_ranks < 1 || n_ranks > 64) {
        std::fprintf(stderr, "usage: %s --ranks N [--events n] [--steps K] [--dump DIR]\n", argv[0]);
        return 2;
    }
    // one pipe per rank > 0: rank 0 writes the unique id into each.  Nothing here touches the GPU
    // before the fork.
    std::vector<int> pipes(2 * n_ranks, -1);
    for (int r = 1; r < n_ranks; ++r)
        if (pipe(&pipes[2 * r]) != 0) {
            std::perror("pipe");
            return 1;
        }
    std::vector<pid_t> kids;
    for (int r = 0; r < n_ranks; ++r) {
        const pid_t pid = fork();
        if (pid < 0) {
            std::perror("fork");
            return 1;
        }
        if (pid == 0) {
            uint8_t id[ECC_DIST_ID_BYTES];
            if (r == 0) {
                if (ecc_dist_get_unique_id(id) != ECC_OK) {
                    std::fprintf(stderr, "ecc_dist_get_unique_id failed (librccl available: %d)\n", ecc_dist_available());
                    _exit(1);
                }
                for (int q = 1; q < n_ranks; ++q)
                    if (write(pipes[2 * q + 1], id, sizeof(id)) != (ssize_t)sizeof(id)) _exit(1);
            } else {
                size_t got = 0;
                while (got < sizeof(id)) {
                    const ssize_t k = read(pipes[2 * r], id + got, sizeof(id) - got);
                    if (k <= 0) _exit(1);
                    got += (size_t)k;
                }
            }
            std::fflush(stdout);
            _exit(run_rank(r, n_ranks, id, argc, argv));
        }
        kids.push_back(pid);
    }
    int rc = 0;
    for (pid_t k : kids) {
        int st = 0;
        waitpid(k, &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = 1;
    }
    return rc;
}
