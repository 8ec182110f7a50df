// Host program mirroring KM/assign_to_centers2.c (main :105-568): data[i] = i % 100 for 4096
// floats (2048 points), 8 centroids {1,1,10,10,...,80,80} (:131), threshold 50; the k-means
// loop runs on the GPU in "fixed" mode (correct Lloyd update, Appendix A Q7-Q9) and prints the
// updated centroids with their point counts like the reference (:539-543).
#include "app_common.hpp"

int main() {
    try {
        std::vector<std::array<float, 2>> pts(2048);
        for (int i = 0; i < 4096; ++i) pts[i / 2][i % 2] = (float)(i % 100);
        std::vector<std::array<float, 2>> c = {{1, 1}, {10, 10}, {20, 20}, {30, 30}, {50, 50}, {60, 60}, {70, 70}, {80, 80}};
        ecc::Context ctx(0);
        ecc::KMeans km(ctx, 8, 20, 50.f, 10.f);  // the reference stops when error_max <= 10 (:545)
        int iters = 0;
        const std::vector<uint8_t> lab = km.fit(pts, c, &iters);
        std::vector<int> cnt(8, 0);
        for (uint8_t l : lab) if (l < 8) cnt[l]++;
        std::printf("updated centroids (%d iterations)\n", iters);
        for (int j = 0; j < 8; ++j) std::printf("(%f, %f, %d) ", c[j][0], c[j][1], cnt[j]);
        std::printf("\n");
    } catch (const ecc::Error &e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
