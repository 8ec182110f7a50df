// Host program mirroring OPT/test/cluster_event_data.cpp (clustering_test_1 :429-545): read the
// (x,y) of an event CSV, optics::compute_reachability_dists(points, min_pts = 2, eps = 10)
// (:449), get_cluster_indices(reach, 10) (:454), and print each cluster's size, centroid and
// variance (:470-530).  eps-neighbourhoods/core distances on the GPU, ordering on the host.
#include <cmath>

#include "app_common.hpp"

// --points <file>: "x,y" lines with signed integers (the KAT point sets of OPT/test/test_main.cpp)
static std::vector<std::array<int, 2>> read_points(const char *path) {
    std::vector<std::array<int, 2>> pts;
    FILE *f = std::fopen(path, "r");
    if (!f) { std::perror(path); std::exit(1); }
    int x, y;
    while (std::fscanf(f, "%d,%d", &x, &y) == 2) pts.push_back({x, y});
    std::fclose(f);
    return pts;
}

int main(int argc, char **argv) {
    try {
        std::vector<std::array<int, 2>> pts;
        if (argc >= 3 && !std::strcmp(argv[1], "--points")) {
            pts = read_points(argv[2]);
        } else {
            Events ev = load_events(argc, argv, 1280, 720);
            pts.resize(ev.xy.size());
            for (size_t i = 0; i < ev.xy.size(); ++i) pts[i] = {(int)(ev.xy[i] & 0xffff), (int)(ev.xy[i] >> 16)};
        }
        const size_t min_pts = (size_t)opt_int(argc, argv, "--min-pts", 2);
        const double eps = opt_int(argc, argv, "--eps", 10), thr = opt_int(argc, argv, "--threshold", 10);
        // --eps 0 or negative: estimated (optics.hpp:428-430)
        auto reach = ecc::optics::compute_reachability_dists(pts, min_pts, eps);
        auto clusters = ecc::optics::get_cluster_indices(reach, thr);
        std::printf("points %zu clusters %zu\n", pts.size(), clusters.size());
        for (size_t c = 0; c < clusters.size(); ++c) {
            double sx = 0, sy = 0;
            for (size_t i : clusters[c]) { sx += pts[i][0]; sy += pts[i][1]; }
            const double m = (double)clusters[c].size(), cx = sx / m, cy = sy / m;
            double vx = 0, vy = 0;
            for (size_t i : clusters[c]) { vx += (pts[i][0] - cx) * (pts[i][0] - cx); vy += (pts[i][1] - cy) * (pts[i][1] - cy); }
            std::printf("cluster %zu size %zu centroid (%.4f, %.4f) variance (%.4f, %.4f)\n", c, clusters[c].size(), cx, cy, vx / m, vy / m);
        }
        std::printf("order");
        for (const auto &r : reach) std::printf(" %zu:%.17g", r.point_index, r.reach_dist);
        std::printf("\n");
    } catch (const ecc::Error &e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
