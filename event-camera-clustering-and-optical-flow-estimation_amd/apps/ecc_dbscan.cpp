// Host program mirroring the DBSCAN part of PCC/pcl_cluster.cpp (:97-148): DBSCAN with eps 20,
// core minPts 20, cluster size 100..25000 over the event points, writing "x,y,z,cluster%8" CSV
// lines (:140).  The cloud is (x, y, 0), or with --t-scale S the (x, y, t) event cloud with
// z = float(t * S) (north_star's clustering over event point clouds).  PCL's PCD input, VoxelGrid
// and RANSAC stages are out of scope.  --precomp runs DBSCANPrecompCluster (the driver's "test 2",
// :106-108); --cloud-first calls setInputCloud before the setters, which for the precomputed
// variant freezes the adjacency at the tolerance set so far (DBSCAN_precomp.h:10-16, :28).
#include "app_common.hpp"

int main(int argc, char **argv) {
    try {
        Events ev = load_events(argc, argv, 1280, 720);
        const double ts = opt_double(argc, argv, "--t-scale", 0.0);
        std::vector<ecc::PointXYZ> cloud(ev.xy.size());
        for (size_t i = 0; i < ev.xy.size(); ++i)
            cloud[i] = {(float)(ev.xy[i] & 0xffff), (float)(ev.xy[i] >> 16), ts != 0.0 ? (float)(ev.t[i] * ts) : 0.f};
        ecc::Context ctx(0);
        const bool precomp = has_flag(argc, argv, "--precomp"), cloud_first = has_flag(argc, argv, "--cloud-first");
        ecc::DBSCANSimpleCluster simple(ctx);
        ecc::DBSCANPrecompCluster pre(ctx);
        ecc::DBSCANSimpleCluster &ec = precomp ? pre : simple;
        if (cloud_first) ec.setInputCloud(cloud);
        ec.setCorePointMinPts(opt_int(argc, argv, "--min-pts", 20));
        ec.setClusterTolerance(opt_double(argc, argv, "--eps", 20.0));
        ec.setMinClusterSize(opt_int(argc, argv, "--min-size", 100));
        ec.setMaxClusterSize(opt_int(argc, argv, "--max-size", 25000));
        if (!cloud_first) ec.setInputCloud(cloud);
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
