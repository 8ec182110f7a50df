// Host program mirroring the DBSCAN part of PCC/pcl_cluster.cpp (:97-148): DBSCAN with eps 20,
// core minPts 20, cluster size 100..25000 over the event points (x,y of a CSV; PCL's PCD input,
// VoxelGrid and RANSAC stages are out of scope), writing "x,y,z,cluster%8" CSV lines (:140).
#include "app_common.hpp"

int main(int argc, char **argv) {
    try {
        Events ev = load_events(argc, argv, 1280, 720);
        std::vector<ecc::PointXYZ> cloud(ev.xy.size());
        for (size_t i = 0; i < ev.xy.size(); ++i) cloud[i] = {(float)(ev.xy[i] & 0xffff), (float)(ev.xy[i] >> 16), 0.f};
        ecc::Context ctx(0);
        ecc::DBSCANSimpleCluster ec(ctx);
        ec.setCorePointMinPts(opt_int(argc, argv, "--min-pts", 20));
        ec.setClusterTolerance(opt_int(argc, argv, "--eps", 20));
        ec.setMinClusterSize(opt_int(argc, argv, "--min-size", 100));
        ec.setMaxClusterSize(opt_int(argc, argv, "--max-size", 25000));
        ec.setInputCloud(cloud);
        std::vector<ecc::PointIndices> clusters;
        ec.extract(clusters);
        std::printf("cluster size : %zu\n", clusters.size());
        for (size_t j = 0; j < clusters.size(); ++j)
            for (int idx : clusters[j].indices)
                std::printf("%g,%g,%g,%zu\n", cloud[idx].x, cloud[idx].y, cloud[idx].z, j % 8);
    } catch (const ecc::Error &e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
