// Host program mirroring DSA/metavision_sdk_get_started5_opencl_store.cpp (and the TWE variant):
// events -> GPU hash-map downsampler over consecutive 8192-event windows -> per window, every
// 2nd representative of the window's first half into AEClustering (the reference's slice
// callback, :370-445) -> per-cluster centroid displacement ("flow", :470-518) -> optional
// cluster frames (PPM, the reference's cv::imwrite) and CSV.
//   usage: ecc_downsample_cluster <events.raw|events.csv> | --synthetic N
//          [--width W --height H] [--radius R --min-n N --kappa K --alpha A --buffer B]
//          [--arrow-scale S] [--ppm-dir DIR] [--csv FILE]
#include <string>

#include "app_common.hpp"

static const char *opt_str(int argc, char **argv, const char *name) {
    for (int i = 1; i + 1 < argc; ++i)
        if (!std::strcmp(argv[i], name)) return argv[i + 1];
    return nullptr;
}

int main(int argc, char **argv) {
    try {
        const int W = opt_int(argc, argv, "--width", 1280), H = opt_int(argc, argv, "--height", 720);
        Events ev = load_events(argc, argv, W, H);
        ecc::Context ctx(0);
        ecc::HashDownsampler ds(ctx);
        std::vector<std::pair<int, int>> coords(ev.xy.size());
        for (size_t i = 0; i < ev.xy.size(); ++i) coords[i] = {(int)(ev.xy[i] & 0xffff), (int)(ev.xy[i] >> 16)};
        const ecc::DownsampleResult r = ds.process(coords);  // all windows in one launch

        ecc::AEClustering ae;  // the reference default-constructs it (:42)
        ae.init(opt_int(argc, argv, "--buffer", 800), opt_double(argc, argv, "--radius", 40.0),
                opt_int(argc, argv, "--kappa", 0), opt_double(argc, argv, "--alpha", 0.5),
                opt_int(argc, argv, "--min-n", 10));
        ecc::CentroidFlow flow;
        const double scale = opt_double(argc, argv, "--arrow-scale", 1.0);
        const char *ppm_dir = opt_str(argc, argv, "--ppm-dir");
        const char *csv = opt_str(argc, argv, "--csv");
        long long cumulative = 0;
        for (size_t w = 0; w < r.unique_count.size(); ++w) {
            cumulative += r.unique_count[w];  // uniqueCount (cumulative) / 1000.0 is the fake time (Q6)
            ecc::aeclustering_feed_window(ae, r.unique_coords[w], cumulative);
            const auto fl = flow.update(ae);
            std::printf("window %zu reps %d clusters %zu\n", w, r.unique_count[w], ae.clusters.size());
            for (const auto &f : fl) {
                std::printf("  cluster %d n %d centroid %.17g %.17g", f.cluster_id, f.n, f.centroid[0], f.centroid[1]);
                if (f.has_prev) std::printf(" flow %.17g %.17g\n", f.diff[0], f.diff[1]);
                else std::printf(" flow -\n");
            }
            if (ppm_dir) {
                const std::string path = std::string(ppm_dir) + "/cluster_frame_combined" + std::to_string(w + 1) + ".ppm";
                if (!ecc::write_cluster_ppm(path, W, H, ae, fl, scale)) {
                    std::perror(path.c_str());
                    return 1;
                }
            }
        }
        if (csv && !ecc::write_cluster_csv(csv, ae, ae.getMinN())) {
            std::perror(csv);
            return 1;
        }
    } catch (const ecc::Error &e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
