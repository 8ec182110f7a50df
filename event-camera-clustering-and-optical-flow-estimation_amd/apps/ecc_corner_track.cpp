// Host program mirroring FCT/metavision_time_surface_periodic_group_track.cpp (main :741-1102):
// 16384-event slices, batch SAE + arc test, per-slice CornerFilter(15) + CornerTracker
// (30, 30, 10, 5, 0.8, 0.3, 100), printing what the reference prints per slice
// ("Corner size", "Filtered corner size") plus the tracks and groups.  No display (OpenCV UI is
// out of scope); all slices of the file are processed in batched launches.
#include "app_common.hpp"

int main(int argc, char **argv) {
    const int W = opt_int(argc, argv, "--width", 1280), H = opt_int(argc, argv, "--height", 720);
    try {
        Events ev = load_events(argc, argv, W, H);
        const int64_t n = (int64_t)ev.xy.size();
        const int S = 16384, cap = 4096;
        const int64_t ns = (n + S - 1) / S;
        ecc::Context ctx(0);
        ecc::DeviceBuffer d_xy, d_t, d_flags(std::max<int64_t>(n, 1)), d_out(ns * cap * sizeof(ecc_corner) + 16),
            d_cnt(ns * 4 + 4);
        d_xy.upload(ev.xy.data(), n * 4, ctx.stream());
        d_t.upload(ev.t.data(), n * 8, ctx.stream());
        ecc::TimeSurfaceCornerDetector det(ctx, W, H, S);
        det.detect(d_xy.as<uint32_t>(), d_t.as<int64_t>(), n, d_flags.as<uint8_t>());
        if (ecc_corner_nms(ctx.get(), d_xy.as<uint32_t>(), d_flags.as<uint8_t>(), n, S, W, H, 15, cap,
                           d_out.as<ecc_corner>(), d_cnt.as<int32_t>(), ctx.stream()) != ECC_OK) {
            std::fprintf(stderr, "ecc_corner_nms failed\n");
            return 1;
        }
        ecc_tracker_cfg tc{30.0f, 30, 10, 5, 0.8f, 0.3f, 100.0f};  // :805-813
        ecc::CornerTracker tracker(ctx, tc);
        tracker.updateDevice(d_out.as<ecc_corner>(), d_cnt.as<int32_t>(), (int)ns, cap);
        std::vector<uint8_t> flags(n);
        std::vector<int32_t> cnt(ns);
        d_flags.download(flags.data(), n, ctx.stream());
        d_cnt.download(cnt.data(), ns * 4, ctx.stream());
        for (int64_t s = 0; s < ns; ++s) {
            int64_t c = 0;
            for (int64_t e = s * S; e < std::min<int64_t>(n, (s + 1) * S); ++e) c += flags[e];
            std::printf("slice %lld: Corner size : %lld  Filtered corner size : %d\n", (long long)s,
                        (long long)c, cnt[s]);
        }
        const auto tracks = tracker.tracks();
        tracker.refreshGroups();
        std::printf("tracks %zu groups %zu\n", tracks.size(), tracker.getCornerGroups().size());
        for (const auto &t : tracks)
            std::printf("track label %d pos (%d,%d) frames %d lost %d vel (%.6f,%.6f)\n", t.label, t.x, t.y,
                        t.frame_count, t.frames_since_last_detection, t.velocity.x, t.velocity.y);
    } catch (const ecc::Error &e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
