// SANITIZER DRIVER — TEST INFRASTRUCTURE ONLY ("run the CPU restatement under
// -fsanitize=address,undefined").  Built by `make -C oracle sanitize` with ASan + UBSan into one
// executable with the oracle (oracle.cpp) and libecc's pure-host C++ (host/events_io.cpp: the
// generator, CSV and RAW readers, the EVT encoders; host/aeclustering.cpp: AEClustering,
// MyCluster, the flow and the writers), and run by tests/test_sanitizers.py.  It drives every
// oracle stage and those host paths over seeded inputs, including ragged and empty cases; any
// sanitizer report aborts with a non-zero status.
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <string>
#include <vector>

#include "../include/ecc.hpp"

extern "C" {
int orc_downsample_hash(const uint32_t *xy, int64_t n, int window, int x_max, int y_max, int mult_x, int mult_y,
                        int n_buckets, uint32_t *rep_xy, uint32_t *rep_idx, int32_t *win_unique, int32_t *win_repeated);
int orc_dedup_exact(const uint32_t *xy, int64_t n, int window, uint32_t *uniq_idx, int32_t *uniq_cnt, int32_t *n_unique);
int orc_kmeans_run_xy16(const uint32_t *xy, int64_t n, float *c, int k, int max_iters, float thr, float tol,
                        uint8_t *labels, int32_t *iters);
int orc_kmeans_run_f32(const float *xy, int64_t n, float *c, int k, int max_iters, float thr, float tol,
                       uint8_t *labels, int32_t *iters);
int orc_kmeans_refcompat(const float *xy, int64_t n, float *c16, int max_passes, int32_t *bin_counts_out,
                         float *partial_sums_out);
int orc_fast_detect(const uint32_t *xy, const int64_t *t, int64_t n, int W, int H, int slice, int margin,
                    int border_mode, int first_detect, int64_t *sae, uint8_t *flags);
int orc_corner_nms(const uint32_t *xy, const uint8_t *flags, int64_t n, int slice, int W, int H, int box, int cap,
                   ecc_corner *out, int32_t *counts);
void *orc_tracker_create(const ecc_tracker_cfg *cfg);
void orc_tracker_destroy(void *tr);
int orc_tracker_update(void *tr, const ecc_corner *cs, int n);
int orc_tracker_get_tracks(void *tr, ecc_track *out, int cap);
int orc_eps_neighbours(const uint32_t *xy, int64_t n_segs, int64_t stride, const int32_t *seg_counts, double eps,
                       int min_pts, int32_t *counts, double *core_dist, int64_t *offsets, int32_t *nbr, int64_t nbr_cap);
int orc_dbscan_cloud_f32(const float *pts, int n, int dim, double eps, int min_pts, int min_size, int max_size,
                         int32_t *labels, int64_t *offs, int32_t *members, int64_t cap);
int orc_radius_f32(const float *pts, int n, int dim, double eps, int min_pts, int32_t *counts, double *core_dist,
                   int64_t *offsets, int32_t *nbr, int64_t cap);
int orc_optics(const double *pts, int n, int D, int min_pts, double eps, int64_t *order, double *reach_out);
int64_t orc_evt2_decode(const uint32_t *w, int64_t n, uint32_t *xy, int64_t *t, uint8_t *p, int64_t cap);
int64_t orc_evt3_decode(const uint16_t *w, int64_t n, uint32_t *xy, int64_t *t, uint8_t *p, int64_t cap);
int64_t orc_reslice_n_us(const int64_t *t, int64_t n, int64_t period, int64_t *bounds, int64_t max_slices);
}

#define REQUIRE(c)                                                              \
    do {                                                                        \
        if (!(c)) {                                                             \
            std::fprintf(stderr, "sanitize_main: %s failed (%s:%d)\n", #c, __FILE__, __LINE__); \
            std::exit(3);                                                       \
        }                                                                       \
    } while (0)

int main(int argc, char **argv) {
    const std::string tmp = argc > 1 ? argv[1] : "/tmp";
    const int W = 346, H = 260, S = 16384;
    for (int64_t n : {int64_t(0), int64_t(1), int64_t(8191), int64_t(S * 5 + 777)}) {
        ecc_gen_cfg g;
        ecc_gen_cfg_default(&g);
        g.width = W;
        g.height = H;
        std::vector<uint32_t> xy(n + 1);
        std::vector<int64_t> t(n + 1);
        std::vector<uint8_t> p(n + 1);
        REQUIRE(ecc_gen_events(&g, 0, n, xy.data(), t.data(), p.data()) == ECC_OK);
        // downsample + exact dedup
        const int64_t nw = (n + 8191) / 8192;
        std::vector<uint32_t> rxy(nw * 8192 + 1), ridx(nw * 8192 + 1), uidx(nw * 8192 + 1);
        std::vector<int32_t> u(nw + 1), r(nw + 1), ucnt(nw * 8192 + 1), nu(nw + 1);
        REQUIRE(orc_downsample_hash(xy.data(), n, 8192, 1280, 720, 1619, 31, 8192, rxy.data(), ridx.data(), u.data(),
                                    r.data()) == 0);
        REQUIRE(orc_dedup_exact(xy.data(), n, 8192, uidx.data(), ucnt.data(), nu.data()) == 0);
        // k-means on the first window's representatives, integer and float forms + ref-compat
        std::vector<uint32_t> pts;
        for (int64_t w = 0; w < nw; ++w)
            for (int k = 0; k < u[w]; ++k) pts.push_back(rxy[w * 8192 + k]);
        std::vector<float> c(32), f(2 * pts.size() + 2);
        for (int k = 0; k < 16; ++k) { c[2 * k] = 20.f + 19.f * k; c[2 * k + 1] = 240.f - 13.f * k; }
        for (size_t i = 0; i < pts.size(); ++i) { f[2 * i] = (float)(pts[i] & 0xffff); f[2 * i + 1] = (float)(pts[i] >> 16); }
        std::vector<uint8_t> lab(pts.size() + 1);
        int32_t it = 0;
        std::vector<float> c2 = c;
        REQUIRE(orc_kmeans_run_xy16(pts.data(), (int64_t)pts.size(), c.data(), 16, 10, 50.f, -1.f, lab.data(), &it) == 0);
        REQUIRE(orc_kmeans_run_f32(f.data(), (int64_t)pts.size(), c2.data(), 16, 10, 50.f, -1.f, lab.data(), &it) == 0);
        std::vector<float> c16(16), sums(32);
        std::vector<int32_t> bins(8);
        for (int k = 0; k < 16; ++k) c16[k] = 10.f + 15.f * k;
        orc_kmeans_refcompat(f.data(), std::min<int64_t>((int64_t)pts.size(), 2048), c16.data(), 5, bins.data(),
                             sums.data());
        // SAE + arc corners (both border modes) + NMS + tracker
        std::vector<int64_t> sae((size_t)W * H, 0);
        std::vector<uint8_t> flags(n + 1);
        for (int bm = 0; bm < 2; ++bm) {
            std::fill(sae.begin(), sae.end(), 0);
            REQUIRE(orc_fast_detect(xy.data(), t.data(), n, W, H, S, 4, bm, 1, sae.data(), flags.data()) == 0);
        }
        const int64_t ns = (n + S - 1) / S, cap = 4096;
        std::vector<ecc_corner> nms((size_t)std::max<int64_t>(ns, 1) * cap);
        std::vector<int32_t> cnt(ns + 1);
        REQUIRE(orc_corner_nms(xy.data(), flags.data(), n, S, W, H, 15, (int)cap, nms.data(), cnt.data()) == 0);
        const ecc_tracker_cfg tc{30.f, 30, 10, 5, 0.8f, 0.3f, 100.f};  // FCT/…group_track.cpp:805-813
        void *tr = orc_tracker_create(&tc);
        for (int64_t s = 0; s < ns; ++s) orc_tracker_update(tr, nms.data() + s * cap, cnt[s]);
        std::vector<ecc_track> tracks(4096);
        orc_tracker_get_tracks(tr, tracks.data(), 4096);
        orc_tracker_destroy(tr);
        // eps-neighbourhoods (windowed int), DBSCAN + radius on an (x, y, t) float cloud, OPTICS
        if (nw > 0) {
            std::vector<int32_t> counts(nw * 8192);
            std::vector<double> core(nw * 8192);
            std::vector<int64_t> offs(nw * 8192 + 1);
            orc_eps_neighbours(rxy.data(), nw, 8192, u.data(), 10.0, 5, counts.data(), core.data(), offs.data(), nullptr, 0);
            std::vector<int32_t> nbr(offs[nw * 8192] + 1);
            REQUIRE(orc_eps_neighbours(rxy.data(), nw, 8192, u.data(), 10.0, 5, nullptr, nullptr, offs.data(),
                                       nbr.data(), (int64_t)nbr.size()) == 0);
        }
        const int m = (int)std::min<int64_t>(n, 3000);
        std::vector<float> cloud(3 * (size_t)m + 3);
        for (int i = 0; i < m; ++i) {
            cloud[3 * i] = (float)(xy[i] & 0xffff) + 0.25f;
            cloud[3 * i + 1] = (float)(xy[i] >> 16) - 0.5f;
            cloud[3 * i + 2] = (float)((t[i] - t[0]) * 0.3);
        }
        std::vector<int32_t> dl(m + 1), mem(8 * (size_t)m + 8), rc(m + 1);
        std::vector<int64_t> doffs(m + 2), roffs(m + 1);
        std::vector<double> rcore(m + 1);
        orc_dbscan_cloud_f32(cloud.data(), m, 3, 8.0, 6, 2, 100000, dl.data(), doffs.data(), mem.data(),
                             (int64_t)mem.size());
        orc_radius_f32(cloud.data(), m, 3, 8.0, 70, rc.data(), rcore.data(), roffs.data(), nullptr, 0);
        std::vector<double> d2((size_t)m * 2 + 2);
        for (int i = 0; i < m; ++i) { d2[2 * i] = cloud[3 * i]; d2[2 * i + 1] = cloud[3 * i + 1]; }
        std::vector<int64_t> order(m + 1);
        std::vector<double> reach(m + 1);
        orc_optics(d2.data(), m, 2, 5, 6.0, order.data(), reach.data());
        // RAW: encode -> file -> probe / read words -> decode (both formats), reslicing
        for (int fmt : {ECC_RAW_EVT2, ECC_RAW_EVT3}) {
            const int64_t wcap = 8 * n + 64 + 2 * ((n ? t[n - 1] : 0) >> 12) + 64;
            std::vector<uint16_t> words((size_t)wcap * 2 + 2);
            const int64_t nwords = ecc_evt_encode(fmt, xy.data(), t.data(), p.data(), n, words.data(), wcap);
            REQUIRE(nwords >= 0);
            const std::string path = tmp + "/sanitize_" + std::to_string(fmt) + ".raw";
            FILE *fp = std::fopen(path.c_str(), "wb");
            REQUIRE(fp);
            std::fprintf(fp, "%% evt %s\n%% end\n", fmt == ECC_RAW_EVT2 ? "2.0" : "3.0");
            const size_t wb = fmt == ECC_RAW_EVT2 ? 4 : 2;
            std::fwrite(words.data(), wb, (size_t)nwords, fp);
            std::fclose(fp);
            ecc_raw_info info;
            REQUIRE(ecc_raw_probe(path.c_str(), &info) == ECC_OK);
            std::vector<uint8_t> back((size_t)nwords * wb + 16);
            REQUIRE(ecc_raw_read_words(path.c_str(), &info, 0, nwords, back.data()) == nwords);
            std::vector<uint32_t> dxy(12 * (size_t)nwords + 1);
            std::vector<int64_t> dt(12 * (size_t)nwords + 1);
            std::vector<uint8_t> dp(12 * (size_t)nwords + 1);
            const int64_t got = fmt == ECC_RAW_EVT2
                                    ? orc_evt2_decode(reinterpret_cast<const uint32_t *>(back.data()), nwords, dxy.data(),
                                                      dt.data(), dp.data(), (int64_t)dxy.size())
                                    : orc_evt3_decode(reinterpret_cast<const uint16_t *>(back.data()), nwords, dxy.data(),
                                                      dt.data(), dp.data(), (int64_t)dxy.size());
            REQUIRE(got == n);
            std::remove(path.c_str());
        }
        if (n > 0) {
            std::vector<int64_t> bounds(((t[n - 1] - t[0]) / 50 + 4));
            orc_reslice_n_us(t.data(), n, 50, bounds.data(), (int64_t)bounds.size());
        }
        // CSV reader round trip
        {
            const std::string path = tmp + "/sanitize.csv";
            FILE *fp = std::fopen(path.c_str(), "w");
            REQUIRE(fp);
            for (int64_t i = 0; i < std::min<int64_t>(n, 2000); ++i)
                std::fprintf(fp, "%u,%u,%lld,%u\n", xy[i] & 0xffff, xy[i] >> 16, (long long)t[i], p[i]);
            std::fclose(fp);
            const int64_t k = ecc_count_csv(path.c_str());
            REQUIRE(k == std::min<int64_t>(n, 2000));
            std::vector<uint32_t> cx(k + 1);
            std::vector<int64_t> ct(k + 1);
            std::vector<uint8_t> cp(k + 1);
            REQUIRE(ecc_read_csv(path.c_str(), cx.data(), ct.data(), cp.data(), k) == k);
            std::remove(path.c_str());
        }
        // AEClustering over the windows (the DSA slice path), flow and writers
        ecc::AEClustering ae;
        ae.init(800, 40.0, 0, 0.5, 10);
        ecc::CentroidFlow flow;
        int64_t cum = 0;
        for (int64_t w = 0; w < nw; ++w) {
            std::vector<std::pair<int, int>> reps;
            for (int k = 0; k < u[w]; ++k) reps.push_back({(int)(rxy[w * 8192 + k] & 0xffff), (int)(rxy[w * 8192 + k] >> 16)});
            cum += u[w];
            ecc::aeclustering_feed_window(ae, reps, cum);
            const auto fl = flow.update(ae);
            ecc::write_cluster_ppm(tmp + "/sanitize.ppm", W, H, ae, fl, 3.0);
            ecc::write_cluster_csv(tmp + "/sanitize_clusters.csv", ae, ae.getMinN());
        }
        std::remove((tmp + "/sanitize.ppm").c_str());
        std::remove((tmp + "/sanitize_clusters.csv").c_str());
        std::printf("n=%lld windows=%lld reps=%zu slices=%lld ok\n", (long long)n, (long long)nw, pts.size(), (long long)ns);
    }
    return 0;
}
