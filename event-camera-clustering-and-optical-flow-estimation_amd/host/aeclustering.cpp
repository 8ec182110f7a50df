// AEClustering / MyCluster host restatement + centroid flow and the
// cluster-frame writers (§8f rank 4).  See include/ecc.hpp for the reference anchors.
//
// Quirks kept:
//   * the reference's unqualified abs() on doubles at global scope binds to C's int abs(int)
//     (MyCluster.cpp:66, :82, :93): each axis distance is truncated toward zero, summed as int;
//   * merge_clusters_ returns before the emptied clusters are erased (AEClustering.cpp:107-110);
//   * kappa = 0 (the default) makes the sampled distance DBL_MAX, so it never assigns (Q19);
//   * forget() on an empty cluster is guarded (the reference reads datT_[0] first, Q18).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <limits>

#include "../../include/ecc.hpp"

namespace ecc {

namespace {
// int abs(int) of the truncated double, as the reference's unqualified abs(double) resolves
inline int iabs_trunc(double v) { return std::abs(static_cast<int>(v)); }
}  // namespace

MyCluster::MyCluster() = default;

MyCluster::MyCluster(double alpha, int kappa) : alpha_(alpha), kappa_(kappa) {}

void MyCluster::reset(int kappa, double alpha, int) {
    kappa_ = kappa;
    alpha_ = alpha;
}

void MyCluster::add(const std::deque<double> &e, int &eventId, double t0) {
    const double t = e[0] - t0;
    const Vec2d pix{e[1], e[2]};
    datId_.push_back(eventId);
    dat_.push_back(pix);
    datT_.push_back(t);
    datPol_.push_back(e[3] != 0.0);
    if (n_ == 0) {
        mu_ = pix;
    } else {  // updateMu_: mu = (1 - alpha) * mu + alpha * pix (MyCluster.cpp:199-201)
        mu_[0] = (1 - alpha_) * mu_[0] + alpha_ * pix[0];
        mu_[1] = (1 - alpha_) * mu_[1] + alpha_ * pix[1];
    }
    n_++;
    eventId++;
}

void MyCluster::forget(double t) {
    while (n_ > 0 && !datT_.empty() && datT_[0] < t) {
        dat_.pop_front();
        datId_.pop_front();
        datT_.pop_front();
        if (!datPol_.empty()) datPol_.pop_front();
        n_--;
    }
}

double MyCluster::manhattanDistance(const Vec2d &x) const {
    return iabs_trunc(x[0] - mu_[0]) + iabs_trunc(x[1] - mu_[1]);
}

double MyCluster::manhattanDistanceWithSampling(const Vec2d &x) const {
    // nearest member by truncating Manhattan distance: all members while the cluster holds fewer
    // than kappa, else kappa members drawn with std::rand() (MyCluster.cpp:72-99; kappa 0 by
    // default, so the draw never happens and the result is DBL_MAX, Q19)
    auto l1 = [&x](const Vec2d &y) -> double { return iabs_trunc(x[0] - y[0]) + iabs_trunc(x[1] - y[1]); };
    double nearest = std::numeric_limits<double>::max();
    if (kappa_ > n_) {
        for (const auto &y : dat_) nearest = std::min(nearest, l1(y));
        return nearest;
    }
    for (int draw = 0; draw < kappa_; ++draw) nearest = std::min(nearest, l1(dat_[std::rand() % (int)dat_.size()]));
    return nearest;
}

Vec2d MyCluster::getClusterCentroid() const {
    double xAcc = 0, yAcc = 0;
    for (const auto &p : dat_) {
        xAcc = xAcc + p[0];
        yAcc = yAcc + p[1];
    }
    xAcc = xAcc / (double)dat_.size();
    yAcc = yAcc / (double)dat_.size();
    return Vec2d{xAcc, yAcc};
}

AEClustering::AEClustering()
    : minN_(10), szBuffer_(800), tMin_(0), radius_(40), alpha_(0.5), kappa_(0), eventId_(0), t0_(-1),
      lastUpdatedCluster_(-1), clusterID_(0) {}

void AEClustering::init(int szBuffer, double radius, int kappa, double alpha, int minN) {
    szBuffer_ = szBuffer;
    radius_ = radius;
    alpha_ = alpha;
    minN_ = minN;
    kappa_ = kappa;
}

bool AEClustering::update(const std::deque<double> &e) {
    if (t0_ < 0) t0_ = e[0];
    const Vec2d pix{e[1], e[2]};
    t = e[0] - t0_;
    std::deque<int> assigned, removed;
    updateBuffer_(t);
    for (int ii = 0; ii < (int)clusters.size(); ii++) {  // proximity (:66-88)
        clusters[ii].forget(tMin_);
        if (clusters[ii].getN() == 0) {
            removed.push_back(ii);
        } else if (clusters[ii].manhattanDistance(pix) <= radius_) {
            assigned.push_back(ii);
        } else if (clusters[ii].getN() > minN_) {
            if (clusters[ii].manhattanDistanceWithSampling(pix) <= radius_) assigned.push_back(ii);
        }
    }
    if (assigned.empty()) {  // new cluster (:92-100)
        clusters.push_back(MyCluster(alpha_, kappa_));
        clusters.back().add(e, eventId_, t0_);
        clusters.back().setClusterId(clusterID_);
        clusterID_++;
        lastUpdatedCluster_ = (int)clusters.size() - 1;
    } else {
        lastUpdatedCluster_ = assigned[0];
        clusters[assigned[0]].add(e, eventId_, t0_);
        if (assigned.size() >= 2) {  // merge, and return before erasing the empty ones (:105-110)
            merge_clusters_(assigned);
            return false;
        }
    }
    for (int ii = (int)removed.size() - 1; ii >= 0; ii--) {
        if (lastUpdatedCluster_ > removed[ii]) lastUpdatedCluster_--;
        clusters.erase(clusters.begin() + removed[ii]);
    }
    return false;
}

void AEClustering::updateBuffer_(double tt) {
    tBuffer_.push_back(tt);
    if ((int)tBuffer_.size() > szBuffer_) tBuffer_.pop_front();
    tMin_ = tBuffer_[0];
}

void AEClustering::merge_clusters_(const std::deque<int> &assigned) {
    const int m = (int)assigned.size();
    std::vector<int> nn(m), count(m, 0);
    int aux_n = 0;
    for (int ii = 0; ii < m; ii++) {
        nn[ii] = clusters[assigned[ii]].getN();
        aux_n += nn[ii];
    }
    Vec2d aux_mu{0.0, 0.0};
    for (int ii = 0; ii < m; ii++) {
        const double w = (double)clusters[assigned[ii]].getN() / (double)aux_n;
        const Vec2d &mu = clusters[assigned[ii]].getMu();
        aux_mu[0] += w * mu[0];
        aux_mu[1] += w * mu[1];
    }
    // k-way merge by time, ties to the lowest assigned position (:180-196)
    std::deque<int> aux_datId;
    std::deque<Vec2d> aux_dat;
    std::deque<double> aux_datT;
    std::deque<bool> aux_datPol;
    for (;;) {
        int idx = -1;
        double tt = std::numeric_limits<double>::max();
        for (int jj = 0; jj < m; jj++) {
            const MyCluster &c = clusters[assigned[jj]];
            if (count[jj] < nn[jj] && c.getDatT()[count[jj]] < tt) {
                idx = jj;
                tt = c.getDatT()[count[jj]];
            }
        }
        if (idx < 0) break;
        const MyCluster &c = clusters[assigned[idx]];
        aux_datId.push_back(c.getDatId()[count[idx]]);
        aux_dat.push_back(c.getDat()[count[idx]]);
        aux_datT.push_back(c.getDatT()[count[idx]]);
        aux_datPol.push_back(c.getDatPol()[count[idx]]);
        count[idx]++;
    }
    MyCluster &dst = clusters[assigned[0]];
    dst.setN((int)aux_dat.size());
    dst.setDatId(aux_datId);
    dst.setDat(aux_dat);
    dst.setDatT(aux_datT);
    dst.setDatPol(aux_datPol);
    dst.setMu(aux_mu);
    for (int ii = m - 1; ii > 0; ii--) clusters.erase(clusters.begin() + assigned[ii]);
}

void aeclustering_feed_window(AEClustering &ae, const std::vector<std::pair<int, int>> &reps,
                              int64_t cumulative_unique) {
    std::deque<double> ev(4, 0.0);
    const int64_t diff = (int64_t)reps.size();
    for (int64_t i = 0; i < diff; i += 4) {  // ints of the interleaved array: representative i / 2
        ev[0] = (double)cumulative_unique / 1000.0;
        ev[1] = reps[i / 2].first;
        ev[2] = reps[i / 2].second;
        ev[3] = 0;
        ae.update(ev);
    }
}

std::vector<ClusterFlow> CentroidFlow::update(const AEClustering &ae) {
    std::vector<ClusterFlow> out;
    const int minN = ae.getMinN();
    for (const auto &cc : ae.clusters) {
        if (cc.getN() < minN) continue;
        int id = cc.getClusterId();
        if (id > 16384) id = id % 16384;  // TWE/…opencl_store.cpp:401-405
        ClusterFlow f;
        f.cluster_id = cc.getClusterId();
        f.n = cc.getN();
        f.centroid = cc.getClusterCentroid();
        f.prev = prev_[id % 16384];
        f.diff = Vec2d{f.centroid[0] - f.prev[0], f.centroid[1] - f.prev[1]};
        f.has_prev = f.prev[0] > 0 && f.prev[1] > 0;
        prev_[id % 16384] = f.centroid;
        out.push_back(f);
    }
    return out;
}

// ---- writers -------------------------------------------------------------------------------
namespace {
struct Rgb {
    unsigned char r, g, b;
};
// the reference's 10-colour BGR palette (DSA/…opencl_store.cpp:356-368), as RGB
const Rgb kPalette[10] = {{0, 0, 255},   {0, 255, 0},   {255, 0, 0}, {0, 255, 255}, {255, 0, 255},
                          {255, 255, 0}, {0, 0, 128},   {0, 128, 0}, {128, 0, 0},   {0, 128, 128}};

struct Image {
    int w, h;
    std::vector<unsigned char> px;
    Image(int w_, int h_) : w(w_), h(h_), px((size_t)w_ * h_ * 3, 0) {}
    void dot(int x, int y, Rgb c, int r = 1) {  // cv::circle(..., radius r, filled)
        for (int dy = -r; dy <= r; ++dy)
            for (int dx = -r; dx <= r; ++dx)
                if (dx * dx + dy * dy <= r * r) set(x + dx, y + dy, c);
    }
    void set(int x, int y, Rgb c) {
        if (x < 0 || y < 0 || x >= w || y >= h) return;
        unsigned char *p = &px[((size_t)y * w + x) * 3];
        p[0] = c.r;
        p[1] = c.g;
        p[2] = c.b;
    }
    void line(int x0, int y0, int x1, int y1, Rgb c) {  // Bresenham
        const int dx = std::abs(x1 - x0), sx = x0 < x1 ? 1 : -1;
        const int dy = -std::abs(y1 - y0), sy = y0 < y1 ? 1 : -1;
        int err = dx + dy;
        for (;;) {
            set(x0, y0, c);
            if (x0 == x1 && y0 == y1) break;
            const int e2 = 2 * err;
            if (e2 >= dy) { err += dy; x0 += sx; }
            if (e2 <= dx) { err += dx; y0 += sy; }
        }
    }
};
}  // namespace

bool write_cluster_ppm(const std::string &path, int width, int height, const AEClustering &ae,
                       const std::vector<ClusterFlow> &flow, double arrow_scale) {
    if (width <= 0 || height <= 0) return false;
    Image img(width, height);
    const int minN = ae.getMinN();
    for (const auto &cc : ae.clusters) {
        if (cc.getN() < minN) continue;
        const Rgb col = kPalette[cc.getClusterId() % 10];
        for (const auto &p : cc.getDat()) img.dot((int)p[0], (int)p[1], col);
    }
    for (const auto &f : flow) {
        img.dot((int)f.centroid[0], (int)f.centroid[1], Rgb{0, 255, 0});
        img.dot((int)f.prev[0], (int)f.prev[1], Rgb{255, 0, 0});
        if (f.has_prev)
            img.line((int)f.prev[0], (int)f.prev[1], (int)(f.prev[0] + f.diff[0] * arrow_scale),
                     (int)(f.prev[1] + f.diff[1] * arrow_scale), Rgb{0, 255, 0});
    }
    FILE *fp = std::fopen(path.c_str(), "wb");
    if (!fp) return false;
    std::fprintf(fp, "P6\n%d %d\n255\n", width, height);
    const bool ok = std::fwrite(img.px.data(), 1, img.px.size(), fp) == img.px.size();
    return std::fclose(fp) == 0 && ok;
}

bool write_cluster_csv(const std::string &path, const AEClustering &ae, int minN) {
    FILE *fp = std::fopen(path.c_str(), "w");
    if (!fp) return false;
    for (const auto &cc : ae.clusters) {
        if (cc.getN() < minN) continue;
        for (size_t i = 0; i < cc.getDat().size(); ++i)
            std::fprintf(fp, "%.17g,%.17g,%.17g,%d\n", cc.getDat()[i][0], cc.getDat()[i][1], cc.getDatT()[i],
                         cc.getClusterId());
    }
    return std::fclose(fp) == 0;
}

}  // namespace ecc
