// Host program mirroring SMP|DSA/metavision_sdk_get_started5_opencl_store.cpp: the hash-map
// downsampler (process_coordinates) over consecutive 8192-event windows, printing per window the
// unique/repeated counts (the reference prints local_unique_count / unique_count, :87) and the
// first representatives (ecc_downsample_cluster adds the AEClustering consumer, §8f rank 2).
#include "app_common.hpp"

int main(int argc, char **argv) {
    try {
        Events ev = load_events(argc, argv, 1280, 720);
        ecc::Context ctx(0);
        ecc::HashDownsampler ds(ctx);
        std::vector<std::pair<int, int>> coords(ev.xy.size());
        for (size_t i = 0; i < ev.xy.size(); ++i) coords[i] = {(int)(ev.xy[i] & 0xffff), (int)(ev.xy[i] >> 16)};
        const ecc::DownsampleResult r = ds.process(coords);
        long long tot = 0;
        for (size_t w = 0; w < r.unique_count.size(); ++w) {
            std::printf("window %zu: unique_count: %d, repeated_count: %d\n", w, r.unique_count[w], r.repeated_count[w]);
            tot += r.unique_count[w];
        }
        std::printf("events %zu representatives %lld\n", ev.xy.size(), tot);
    } catch (const ecc::Error &e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
