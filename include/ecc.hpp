// ecc.hpp — C++ host layer of the MI355X event pipeline, mirroring the reference's own
// operator interfaces (same names, argument meaning and error behaviour) on top of the C ABI in
// ecc.h, so a reference host program switches by changing its includes:
//
//   reference                                                    here
//   CornerFilter::filterCorners      FCT/…group_track.cpp:81-152   ecc::CornerFilter::filterCorners
//   CornerTracker(...)::updateTrackedCorners / getCornerGroups
//                                    FCT/…group_track.cpp:401-536  ecc::CornerTracker
//   struct Corner / TrackedCorner / CornerGroup / DirectionVector
//                                    FCT/…group_track.cpp:61-199   ecc::Corner ... (cv::Point2f ->
//                                                                  ecc::Point2f, cv::Point -> ecc::Point)
//   optics::compute_reachability_dists<N>(pts, min_pts, eps)
//                                    OPT/include/optics/optics.hpp:413-565  ecc::optics::compute_reachability_dists
//                                                                  (runtime N instead of the template N)
//   optics::get_cluster_indices / epsilon_estimation
//                                    optics.hpp:674-690, 369-387   ecc::optics::...
//   DBSCANSimpleCluster / DBSCANPrecompCluster::{setInputCloud, setClusterTolerance,
//     setCorePointMinPts, setMin/MaxClusterSize, extract}
//                                    PCC/DBSCAN_simple.h:14-143, DBSCAN_precomp.h  ecc::DBSCANSimpleCluster ...
//   process_coordinates + host slice path  SMP/…opencl_store.cpp:250-417  ecc::HashDownsampler
//   assign_to_centers + k-means host loop  KM/assign_to_centers2.c:184-548 ecc::KMeans
//   aggregate lambda (batch SAE + arc test) FCT/…group_track.cpp:884-1070  ecc::TimeSurfaceCornerDetector
//
// Errors: the C ABI returns negative ecc_status codes; this layer throws ecc::Error (the
// reference hosts perror()+exit(1); its host programs in apps/ do the same on an ecc::Error).
// Compute always runs on the GPU through libecc; there is no CPU fallback.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <cmath>
#include <deque>
#include <limits>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "ecc.h"

#pragma GCC visibility push(default)
namespace ecc {

class Error : public std::runtime_error {
  public:
    Error(int status, const std::string &what)
        : std::runtime_error(what + ": " + ecc_status_string(status)), status_(status) {}
    int status() const { return status_; }

  private:
    int status_;
};

// One GPU context + stream (replaces create_device/clCreateContext/clCreateCommandQueue).
class Context {
  public:
    explicit Context(int device = 0);
    ~Context();
    Context(const Context &) = delete;
    Context &operator=(const Context &) = delete;
    ecc_ctx *get() const { return ctx_; }
    ecc_stream_t stream() const { return stream_; }
    void sync() const;
    // process-wide default context on device 0 (the reference's single global OpenCL device)
    static Context &default_context();

  private:
    ecc_ctx *ctx_ = nullptr;
    ecc_stream_t stream_ = nullptr;
};

// Owning device buffer.
class DeviceBuffer {
  public:
    DeviceBuffer() = default;
    explicit DeviceBuffer(size_t bytes);
    ~DeviceBuffer();
    DeviceBuffer(DeviceBuffer &&o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
    DeviceBuffer &operator=(DeviceBuffer &&o) noexcept;
    DeviceBuffer(const DeviceBuffer &) = delete;
    DeviceBuffer &operator=(const DeviceBuffer &) = delete;
    void *data() const { return p_; }
    size_t size() const { return n_; }
    void reserve(size_t bytes);  // grows (content not kept)
    template <typename T> T *as() const { return static_cast<T *>(p_); }
    void upload(const void *src, size_t bytes, ecc_stream_t s);
    void download(void *dst, size_t bytes, ecc_stream_t s) const;

  private:
    void *p_ = nullptr;
    size_t n_ = 0;
};

inline uint32_t pack_xy(int x, int y) { return (uint32_t)(x & 0xffff) | ((uint32_t)(y & 0xffff) << 16); }

// ------------------------------------------------------------------------------ corners
struct Corner {  // FCT/…group_track.cpp:61-67
    int x;
    int y;
    int label;
};

struct Point {  // cv::Point
    int x, y;
};

struct Point2f {  // cv::Point2f
    float x, y;
};

struct DirectionVector {  // :163-175
    Point2f current;
    Point2f target;
    float damping;
    float smoothing;
};

struct TrackedCorner {  // :177-190
    int x;
    int y;
    int label;
    int frame_count;
    bool is_matched;
    int frames_since_last_detection;
    std::deque<Point> position_history;
    Point2f velocity;
    DirectionVector direction;
    int group_id;
};

struct CornerGroup {  // :193-199
    std::vector<int> corner_labels;
    Point2f average_velocity;
    Point2f centroid;
    float radius;
};

class CornerFilter {  // :69-153
  public:
    static std::vector<Corner> filterCorners(const std::vector<Corner> &corners, int image_width,
                                             int image_height, int box_size, float threshold);
    static std::vector<Corner> filterCorners(Context &ctx, const std::vector<Corner> &corners,
                                             int image_width, int image_height, int box_size,
                                             float threshold);
};

class CornerTracker {  // :201-537, device-resident state
  public:
    CornerTracker(float max_matching_distance = 30.0f, int max_frames = 30, int history_size = 10,
                  int frames_to_skip = 5, float damping = 0.8f, float smoothing = 0.3f,
                  float group_rad = 50.0f);
    CornerTracker(Context &ctx, const ecc_tracker_cfg &cfg, int max_tracks = ECC_TRACKER_MAX_TRACKS,
                  int max_detections = 4096);
    ~CornerTracker();
    CornerTracker(const CornerTracker &) = delete;
    CornerTracker &operator=(const CornerTracker &) = delete;

    std::vector<TrackedCorner> updateTrackedCorners(const std::vector<Corner> &current_corners);
    const std::map<int, CornerGroup> &getCornerGroups() const { return groups_; }
    // Batched form: n_slices NMS outputs already on the device (one launch for all slices).
    void updateDevice(const ecc_corner *d_corners, const int32_t *d_counts, int n_slices, int cap);
    std::vector<TrackedCorner> tracks();  // current state (host copy)
    void refreshGroups();

  private:
    Context *ctx_;
    ecc_tracker *tr_ = nullptr;
    int max_tracks_, max_det_;
    DeviceBuffer d_corners_, d_count_;
    std::map<int, CornerGroup> groups_;
};

// Batch SAE + arc-test corner detector (the aggregate lambda, :884-1070), stream-continuable.
class TimeSurfaceCornerDetector {
  public:
    // any_order: timestamps need not be non-decreasing (ecc_corner_cfg.any_order; exact path)
    TimeSurfaceCornerDetector(Context &ctx, int width, int height, int slice_events = 16384,
                              int border_mode = 0, bool any_order = false);
    // xy/t on the device; flags (device, n bytes) receive 1 for corner events.  The SAE carries
    // over between calls; the first call skips the first slice (time_surface_flag, :926).
    void detect(const uint32_t *d_xy, const int64_t *d_t, int64_t n, uint8_t *d_flags);
    int64_t *sae() const { return sae_.as<int64_t>(); }
    const ecc_corner_cfg &config() const { return cfg_; }

  private:
    Context &ctx_;
    ecc_corner_cfg cfg_;
    DeviceBuffer sae_;
    bool first_ = true;
};

// ------------------------------------------------------------------------------ ingest
// RAW recording reader (the role of Metavision::Camera::from_file(argv[1]), FCT/…group_track.cpp
// :756-760): the host streams payload words from disk, the GPU decodes them (ecc_evt_decode)
// with the carry state between chunks, so a recording of any length decodes piecewise.
class RawFileReader {
  public:
    RawFileReader(Context &ctx, const std::string &path, int64_t chunk_words = int64_t(1) << 24);
    const ecc_raw_info &info() const { return info_; }
    // Decodes the next chunk; device arrays stay valid until the next call.  0 at end of file.
    int64_t next(const uint32_t **d_xy, const int64_t **d_t, const uint8_t **d_p);
    // Whole recording into host vectors.
    void read_all(std::vector<uint32_t> &xy, std::vector<int64_t> &t, std::vector<uint8_t> &p);

  private:
    Context &ctx_;
    std::string path_;
    ecc_raw_info info_{};
    int64_t chunk_, pos_ = 0;
    std::vector<uint8_t> host_;
    DeviceBuffer words_, xy_, t_, p_, n_, state_;
};

// n-events / n-µs slicing (EventBufferReslicerAlgorithm::Condition::make_n_events /
// make_n_us): slice k = events [bounds[k], bounds[k+1]).  t on the device.
std::vector<int64_t> reslice_n_events(int64_t n, int64_t n_events);
std::vector<int64_t> reslice_n_us(Context &ctx, const int64_t *d_t, int64_t n, int64_t period_us);

// ------------------------------------------------------------------------------ downsample / k-means
struct DownsampleResult {
    std::vector<int32_t> unique_count, repeated_count;  // per window
    std::vector<std::vector<std::pair<int, int>>> unique_coords;  // per window (ascending index)
};

class HashDownsampler {  // process_coordinates + slice path (SMP/…opencl_store.cpp:341-417)
  public:
    explicit HashDownsampler(Context &ctx, const ecc_hash_cfg *cfg = nullptr);
    // device-level: all windows of a batch in one launch
    void run(const uint32_t *d_xy, int64_t n, uint32_t *d_rep_xy, uint32_t *d_rep_idx,
             int32_t *d_unique, int32_t *d_repeated);
    // host convenience: (x,y) pairs in, per-window unique coordinates out
    DownsampleResult process(const std::vector<std::pair<int, int>> &coords);
    const ecc_hash_cfg &config() const { return cfg_; }

  private:
    Context &ctx_;
    ecc_hash_cfg cfg_;
};

// Exact dedup of one window.  FCT/metavision_time_surface_periodic.cpp:
// CoordinateInfo :47-52, analyzeCoordinates :68-120 over the reference's int data[] laid out
// x0, y0, x1, y1, ... (ARRAY_SIZE = 16384 ints).  Returns uniqueCount; `coords` (optional) gets the
// distinct coordinates in first-occurrence order with their counts.  GPU: ecc_dedup_exact.
struct CoordinateInfo {
    int x, y, count;
};
int analyzeCoordinates(Context &ctx, const int *data, int n_ints = 16384, std::vector<CoordinateInfo> *coords = nullptr);

class KMeans {  // assign_to_centers + host loop, "fixed" mode (Appendix A Q7-Q10)
  public:
    KMeans(Context &ctx, int k, int max_iters = 20, float threshold = 50.f, float tol = 1e-3f);
    // host convenience: points (x,y floats), centroids in/out; returns labels (255 = none)
    std::vector<uint8_t> fit(const std::vector<std::array<float, 2>> &points,
                             std::vector<std::array<float, 2>> &centroids, int *iters = nullptr);
    const ecc_kmeans_cfg &config() const { return cfg_; }
    // the reference's own loop ("ref_compat", Appendix A Q7-Q9: 8 centres, <= 16384 points, bins of
    // 2048 never cleared, the ss[j+1] index quirk, the int-abs restart test); returns the passes
    static int fit_ref_compat(Context &ctx, const std::vector<std::array<float, 2>> &points,
                              std::array<float, 16> &centroids, int max_passes = 50,
                              std::array<int32_t, 8> *bin_counts = nullptr);

  private:
    Context &ctx_;
    ecc_kmeans_cfg cfg_;
};

// ------------------------------------------------------------------------------ AEClustering
// Host restatement of the reference's downsample consumer:
// DSA/MyCluster.{h,cpp} and DSA/AEClustering.{h,cpp} — a per-event incremental clusterer,
// serial by construction, fed from the GPU downsampler.  Eigen::VectorXd(2) is a
// std::array<double, 2>; arithmetic is the same double-precision expressions.
using Vec2d = std::array<double, 2>;

class MyCluster {  // MyCluster.h:9-77
  public:
    MyCluster();                       // :5-11
    MyCluster(double alpha, int kappa);  // :13-20 (without the constructor print)
    void reset(int kappa, double alpha, int minN);
    // e = {t, x, y, pol}; t relative to t0 is stored; eventId is post-incremented (:26-49)
    void add(const std::deque<double> &e, int &eventId, double t0);
    void forget(double t);             // :51-63, guarded on an empty cluster (Appendix A Q18)
    double manhattanDistance(const Vec2d &x) const;               // :65-68
    double manhattanDistanceWithSampling(const Vec2d &x) const;   // :70-99 (std::rand, as the reference)
    void setN(int n) { n_ = n; }
    void setDatId(const std::deque<int> &v) { datId_ = v; }
    void setDat(const std::deque<Vec2d> &v) { dat_ = v; }
    void setDatT(const std::deque<double> &v) { datT_ = v; }
    void setDatPol(const std::deque<bool> &v) { datPol_ = v; }
    void setMu(const Vec2d &mu) { mu_ = mu; }
    void setMuPrev(const Vec2d &mu) { muPrev_ = mu; }
    void setClusterId(int id) { clusterId_ = id; }
    int getN() const { return n_; }
    const std::deque<int> &getDatId() const { return datId_; }
    const std::deque<Vec2d> &getDat() const { return dat_; }
    const std::deque<double> &getDatT() const { return datT_; }
    const std::deque<bool> &getDatPol() const { return datPol_; }
    Vec2d getClusterCentroid() const;  // :180-195 mean of the stored points
    const Vec2d &getMu() const { return mu_; }
    const Vec2d &getMuPrev() const { return muPrev_; }
    int getClusterId() const { return clusterId_; }

  private:
    std::deque<int> datId_;
    std::deque<Vec2d> dat_;
    std::deque<double> datT_;
    std::deque<bool> datPol_;
    double alpha_ = 0.5;
    Vec2d mu_{0.0, 0.0}, muPrev_{0.0, 0.0};
    int n_ = 0, kappa_ = 0, clusterId_ = 0;
};

class AEClustering {  // AEClustering.h:6-44
  public:
    AEClustering();  // :7-18: minN 10, buffer 800, radius 40, alpha 0.5, kappa 0
    void init(int szBuffer, double radius = 10, int kappa = 10, double alpha = 0.5, int minN = 5);
    // e = {t, x, y, pol}; always returns false, as the reference (:51-125)
    bool update(const std::deque<double> &e);
    int getLastUpdatedClusterIdx() const { return lastUpdatedCluster_; }
    int getMinN() const { return minN_; }
    double t = 0.0;
    std::deque<MyCluster> clusters;

  private:
    void updateBuffer_(double t);                        // :141-149
    void merge_clusters_(const std::deque<int> &assigned);  // :151-211
    int minN_, szBuffer_;
    std::deque<double> tBuffer_;
    double tMin_, radius_, alpha_;
    int kappa_, eventId_;
    double t0_;
    int lastUpdatedCluster_, clusterID_;
};

// The downsample -> clusterer hand-off of DSA/…opencl_store.cpp:428-445 for one window's
// representatives (ascending index): the reference walks the interleaved int array with
// i += 4 while i < diff, i.e. representatives k = 0, 2, 4, ... with 2k < n_reps, each fed as
// {cumulative_unique / 1000.0, x, y, 0} (the fake time axis, Appendix A Q6; per-window counts, Q4).
void aeclustering_feed_window(AEClustering &ae, const std::vector<std::pair<int, int>> &reps,
                              int64_t cumulative_unique);

// Centroid-displacement "flow" (DSA/…opencl_store.cpp:470-518,
// TWE/…opencl_store.cpp:396-448): per slice, every cluster with getN() >= minN gets
// cen = getClusterCentroid(), prev = centroid_prev[id % 16384], diff = cen - prev, drawn as an
// arrow from prev to prev + scale * diff (scale 1 DSA, 3 TWE) when prev.x > 0 && prev.y > 0;
// then centroid_prev[id] = cen.
struct ClusterFlow {
    int cluster_id, n;
    Vec2d centroid, prev, diff;
    bool has_prev;
};

class CentroidFlow {
  public:
    std::vector<ClusterFlow> update(const AEClustering &ae);

  private:
    std::vector<Vec2d> prev_ = std::vector<Vec2d>(16384, Vec2d{0.0, 0.0});  // double centroid_prev[16384][2]
};

// Writers: the per-slice cluster frame the reference draws with OpenCV and saves with
// cv::imwrite (DSA/…opencl_store.cpp:479-555) as a binary PPM (no OpenCV here): points in
// the 10-colour palette by id % 10, centroid green, previous centroid red, flow arrow green.
// CSV: one "x,y,t,cluster" line per clustered point (PCC/pcl_cluster.cpp:140 layout).
bool write_cluster_ppm(const std::string &path, int width, int height, const AEClustering &ae,
                       const std::vector<ClusterFlow> &flow, double arrow_scale = 1.0);
bool write_cluster_csv(const std::string &path, const AEClustering &ae, int minN);

// ------------------------------------------------------------------------------ OPTICS
namespace optics {

struct reachability_dist {  // optics.hpp:57-65
    reachability_dist(std::size_t point_index_, double reach_dist_)
        : point_index(point_index_), reach_dist(reach_dist_) {}
    std::string to_string() const;
    std::size_t point_index;
    double reach_dist;
};
bool operator<(const reachability_dist &lhs, const reachability_dist &rhs);   // :67-69
bool operator==(const reachability_dist &lhs, const reachability_dist &rhs);  // :70-72

// eps-balls, core distances and neighbour lists on the GPU for any number of points in 1-3
// dimensions (ecc_radius_*_f64: one global cell grid, fp64 distances in the reference's
// operation order), the ordered seed-set expansion on the host (sequential by nature,
// :525-555).  The reference's template N (points.size() must equal it, :422-425) is the runtime
// size.  epsilon <= 0: estimated with epsilon_estimation (:428-430).
std::vector<reachability_dist> compute_reachability_dists(
    const std::vector<std::array<int, 2>> &points, std::size_t min_pts, double epsilon = -1.0);
std::vector<reachability_dist> compute_reachability_dists(
    const std::vector<std::array<int, 3>> &points, std::size_t min_pts, double epsilon = -1.0);
std::vector<reachability_dist> compute_reachability_dists(
    const std::vector<std::array<double, 1>> &points, std::size_t min_pts, double epsilon = -1.0);
std::vector<reachability_dist> compute_reachability_dists(
    const std::vector<std::array<double, 2>> &points, std::size_t min_pts, double epsilon = -1.0);
std::vector<reachability_dist> compute_reachability_dists(
    const std::vector<std::array<double, 3>> &points, std::size_t min_pts, double epsilon = -1.0);
std::vector<reachability_dist> compute_reachability_dists(
    Context &ctx, const std::vector<std::array<int, 2>> &points, std::size_t min_pts, double epsilon = -1.0);
std::vector<reachability_dist> compute_reachability_dists(
    Context &ctx, const std::vector<std::array<int, 3>> &points, std::size_t min_pts, double epsilon = -1.0);
std::vector<reachability_dist> compute_reachability_dists(
    Context &ctx, const std::vector<std::array<double, 1>> &points, std::size_t min_pts, double epsilon = -1.0);
std::vector<reachability_dist> compute_reachability_dists(
    Context &ctx, const std::vector<std::array<double, 2>> &points, std::size_t min_pts, double epsilon = -1.0);
std::vector<reachability_dist> compute_reachability_dists(
    Context &ctx, const std::vector<std::array<double, 3>> &points, std::size_t min_pts, double epsilon = -1.0);
// the same over a raw host array of n D-dim points (the ecc_optics_f64 C ABI)
std::vector<reachability_dist> optics_f64_export(ecc_ctx *ctx, ecc_stream_t s, const double *pts, int64_t n, int D,
                                                 std::size_t min_pts, double epsilon);

template <typename T, std::size_t dimension>
double epsilon_estimation(const std::vector<std::array<T, dimension>> &points, std::size_t min_pts);

std::vector<std::vector<std::size_t>> get_cluster_indices(
    const std::vector<reachability_dist> &reach_dists, double reachability_threshold);

}  // namespace optics

// ------------------------------------------------------------------------------ DBSCAN
struct PointXYZ {  // pcl::PointXYZ
    float x, y, z;
};
struct PointIndices {  // pcl::PointIndices
    std::vector<int> indices;
};

class DBSCANSimpleCluster {  // PCC/DBSCAN_simple.h:14-143 (GPU radius search + extraction, any size)
  public:
    explicit DBSCANSimpleCluster(Context &ctx = Context::default_context()) : ctx_(ctx) {}
    virtual ~DBSCANSimpleCluster() = default;
    virtual void setInputCloud(const std::vector<PointXYZ> &cloud) { cloud_ = cloud; }
    void setClusterTolerance(double tolerance) { eps_ = tolerance; }
    void setMinClusterSize(int min_cluster_size) { min_pts_per_cluster_ = min_cluster_size; }
    void setMaxClusterSize(int max_cluster_size) { max_pts_per_cluster_ = max_cluster_size; }
    void setCorePointMinPts(int core_point_min_pts) { minPts_ = core_point_min_pts; }
    // float x,y,z clouds of any size (ecc_dbscan_cloud_f32); clusters sorted by size,
    // descending (ties: smallest member index first, then creation order)
    void extract(std::vector<PointIndices> &cluster_indices);

  protected:
    // the tolerance the neighbourhoods are built with (radiusSearch(i, eps_, ...), :36, :61)
    virtual double searchTolerance() const { return eps_; }
    Context &ctx_;
    std::vector<PointXYZ> cloud_;
    double eps_{0.0};
    int minPts_{1};
    int min_pts_per_cluster_{1};
    int max_pts_per_cluster_{std::numeric_limits<int>::max()};
};

// DBSCAN_precomp.h:7-55: the adjacency is precomputed in setInputCloud with the tolerance set AT
// THAT TIME (precomp() reads eps_, :28) — a later setClusterTolerance does not change it.  The
// neighbourhoods themselves are the same test as the simple variant's, so extraction is shared.
class DBSCANPrecompCluster : public DBSCANSimpleCluster {
  public:
    using DBSCANSimpleCluster::DBSCANSimpleCluster;
    void setInputCloud(const std::vector<PointXYZ> &cloud) override {
        cloud_ = cloud;
        precomp_eps_ = eps_;
    }

  protected:
    double searchTolerance() const override { return precomp_eps_; }
    double precomp_eps_{0.0};
};

// Neighbour lists of 2-D integer points (x,y of the cloud) on the GPU: CSR, ascending indices
// (DBSCAN_precomp.h's adjacency row order); any number of points and any min_pts.
void eps_neighbour_lists(Context &ctx, const std::vector<std::array<int, 2>> &points, double eps,
                         std::vector<int64_t> &offsets, std::vector<int32_t> &nbr,
                         int min_pts = 1, std::vector<double> *core_dist = nullptr);

// ---- template definitions
namespace optics {
// optics.hpp:340-387 — bounding box (max initialised from points[1], Q20), uniform-density
// eps for min_pts points per unit ball.
template <typename T, std::size_t dimension>
double epsilon_estimation(const std::vector<std::array<T, dimension>> &points, std::size_t min_pts) {
    if (points.size() <= 1) return 0;
    const double d = static_cast<double>(dimension);
    std::array<T, dimension> mn(points[0]), mx(points[1]);
    for (const auto &p : points)
        for (std::size_t i = 0; i < dimension; i++) {
            if (p[i] < mn[i]) mn[i] = p[i];
            if (p[i] > mx[i]) mx[i] = p[i];
        }
    double volume = 1;
    for (std::size_t i = 0; i < dimension; i++) volume *= std::abs(static_cast<double>(mx[i] - mn[i]));
    const double space_per_minpts = (volume / static_cast<double>(points.size())) * static_cast<double>(min_pts);
    const double unit_ball = std::sqrt(std::pow(M_PI, d)) / std::tgamma(d / 2.0 + 1.0);
    return std::pow(space_per_minpts / unit_ball, 1.0 / d);
}
}  // namespace optics

}  // namespace ecc
#pragma GCC visibility pop
