// C++ host layer (include/ecc.hpp) over the C ABI: mirrors the reference's class interfaces.
// All compute goes through libecc's HIP kernels; the host only does what the reference does
// sequentially by nature (OPTICS seed-set ordering, DBSCAN cluster expansion) on GPU-computed
// neighbourhoods, plus argument marshalling.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <set>
#include <sstream>

#include "../../include/ecc.hpp"

namespace ecc {

static void check(int rc, const char *what) {
    if (rc != ECC_OK) throw Error(rc, what);
}

// ------------------------------------------------------------------------------ runtime
Context::Context(int device) {
    check(ecc_set_device(device), "ecc_set_device");
    check(ecc_ctx_create(&ctx_, device), "ecc_ctx_create");
    check(ecc_stream_create(&stream_), "ecc_stream_create");
}

Context::~Context() {
    if (ctx_) ecc_ctx_destroy(ctx_);
    if (stream_) ecc_stream_destroy(stream_);
}

void Context::sync() const { check(ecc_stream_sync(stream_), "ecc_stream_sync"); }

Context &Context::default_context() {
    static Context ctx(0);
    return ctx;
}

DeviceBuffer::DeviceBuffer(size_t bytes) { reserve(bytes); }

DeviceBuffer::~DeviceBuffer() {
    if (p_) ecc_dev_free(p_);
}

DeviceBuffer &DeviceBuffer::operator=(DeviceBuffer &&o) noexcept {
    if (this != &o) {
        if (p_) ecc_dev_free(p_);
        p_ = o.p_;
        n_ = o.n_;
        o.p_ = nullptr;
        o.n_ = 0;
    }
    return *this;
}

void DeviceBuffer::reserve(size_t bytes) {
    if (bytes <= n_ && p_) return;
    if (p_) ecc_dev_free(p_);
    p_ = nullptr;
    n_ = 0;
    check(ecc_dev_alloc(&p_, bytes ? bytes : 16), "ecc_dev_alloc");
    n_ = bytes;
}

void DeviceBuffer::upload(const void *src, size_t bytes, ecc_stream_t s) {
    reserve(bytes);
    if (bytes) check(ecc_memcpy_h2d(p_, src, bytes, s), "ecc_memcpy_h2d");
}

void DeviceBuffer::download(void *dst, size_t bytes, ecc_stream_t s) const {
    if (bytes) check(ecc_memcpy_d2h(dst, p_, bytes, s), "ecc_memcpy_d2h");
}

// ------------------------------------------------------------------------------ corners
std::vector<Corner> CornerFilter::filterCorners(const std::vector<Corner> &corners, int w, int h,
                                                int box, float threshold) {
    return filterCorners(Context::default_context(), corners, w, h, box, threshold);
}

std::vector<Corner> CornerFilter::filterCorners(Context &ctx, const std::vector<Corner> &corners,
                                                int w, int h, int box, float /*threshold: unused
                                                in the reference too, :107-108*/) {
    if (corners.empty()) return {};  // :88-89
    const int64_t n = (int64_t)corners.size();
    if (n > 16384) throw Error(ECC_ERR_INVALID, "filterCorners: more than 16384 corners in one call");
    std::vector<uint32_t> xy(n);
    std::vector<uint8_t> flags(n, 1);
    for (int64_t i = 0; i < n; ++i) xy[i] = pack_xy(corners[i].x, corners[i].y);
    DeviceBuffer d_xy, d_f, d_out(sizeof(ecc_corner) * n), d_cnt(sizeof(int32_t));
    d_xy.upload(xy.data(), xy.size() * 4, ctx.stream());
    d_f.upload(flags.data(), flags.size(), ctx.stream());
    check(ecc_corner_nms(ctx.get(), d_xy.as<uint32_t>(), d_f.as<uint8_t>(), n, (int32_t)n, w, h,
                         box, (int32_t)n, d_out.as<ecc_corner>(), d_cnt.as<int32_t>(), ctx.stream()),
          "ecc_corner_nms");
    int32_t k = 0;
    d_cnt.download(&k, 4, ctx.stream());
    std::vector<ecc_corner> out(k);
    d_out.download(out.data(), sizeof(ecc_corner) * k, ctx.stream());
    std::vector<Corner> res(k);
    for (int i = 0; i < k; ++i) res[i] = Corner{out[i].x, out[i].y, out[i].label};
    return res;
}

CornerTracker::CornerTracker(float max_matching_distance, int max_frames, int history_size,
                             int frames_to_skip, float damping, float smoothing, float group_rad)
    : ctx_(&Context::default_context()), max_tracks_(ECC_TRACKER_MAX_TRACKS), max_det_(4096) {
    ecc_tracker_cfg c{max_matching_distance, max_frames, history_size, frames_to_skip, damping,
                      smoothing, group_rad};
    check(ecc_tracker_create(ctx_->get(), &c, max_tracks_, max_det_, &tr_), "ecc_tracker_create");
}

CornerTracker::CornerTracker(Context &ctx, const ecc_tracker_cfg &cfg, int max_tracks,
                             int max_detections)
    : ctx_(&ctx), max_tracks_(max_tracks), max_det_(max_detections) {
    check(ecc_tracker_create(ctx.get(), &cfg, max_tracks, max_detections, &tr_), "ecc_tracker_create");
}

CornerTracker::~CornerTracker() {
    if (tr_) ecc_tracker_destroy(tr_);
}

void CornerTracker::updateDevice(const ecc_corner *d_corners, const int32_t *d_counts, int n_slices,
                                 int cap) {
    check(ecc_tracker_update(tr_, d_corners, d_counts, n_slices, cap, ctx_->stream()), "ecc_tracker_update");
}

std::vector<TrackedCorner> CornerTracker::tracks() {
    check(ecc_tracker_status(tr_, ctx_->stream()), "tracker device status");
    std::vector<ecc_track> raw(max_tracks_);
    int32_t n = 0;
    check(ecc_tracker_get_tracks(tr_, raw.data(), max_tracks_, &n, ctx_->stream()), "ecc_tracker_get_tracks");
    std::vector<TrackedCorner> out(n);
    for (int i = 0; i < n; ++i) {
        const ecc_track &t = raw[i];
        TrackedCorner &o = out[i];
        o.x = t.x; o.y = t.y; o.label = t.label; o.frame_count = t.frame_count;
        o.is_matched = t.is_matched != 0;
        o.frames_since_last_detection = t.frames_since_last_detection;
        for (int k = 0; k < t.hist_len; ++k) o.position_history.push_back(Point{t.hist_x[k], t.hist_y[k]});
        o.velocity = Point2f{t.vx, t.vy};
        o.direction = DirectionVector{Point2f{t.dir_cur_x, t.dir_cur_y}, Point2f{t.dir_tgt_x, t.dir_tgt_y}, 0.f, 0.f};
        o.group_id = t.group_id;
    }
    return out;
}

void CornerTracker::refreshGroups() {
    std::vector<ecc_group> g(max_tracks_);
    std::vector<int32_t> labels(max_tracks_);
    int32_t n = 0;
    check(ecc_tracker_get_groups(tr_, g.data(), max_tracks_, &n, labels.data(), max_tracks_, ctx_->stream()),
          "ecc_tracker_get_groups");
    groups_.clear();
    for (int i = 0; i < n; ++i) {
        CornerGroup cg;
        cg.corner_labels.assign(labels.begin() + g[i].first_label_offset,
                                labels.begin() + g[i].first_label_offset + g[i].n_labels);
        cg.average_velocity = Point2f{g[i].avg_vx, g[i].avg_vy};
        cg.centroid = Point2f{g[i].cx, g[i].cy};
        cg.radius = g[i].radius;
        groups_[g[i].id] = cg;
    }
}

std::vector<TrackedCorner> CornerTracker::updateTrackedCorners(const std::vector<Corner> &cs) {
    const int n = (int)std::min<size_t>(cs.size(), (size_t)max_det_);
    std::vector<ecc_corner> raw(std::max(n, 1));
    for (int i = 0; i < n; ++i) raw[i] = ecc_corner{cs[i].x, cs[i].y, cs[i].label};
    d_corners_.upload(raw.data(), sizeof(ecc_corner) * raw.size(), ctx_->stream());
    const int32_t cnt = n;
    d_count_.upload(&cnt, 4, ctx_->stream());
    updateDevice(d_corners_.as<ecc_corner>(), d_count_.as<int32_t>(), 1, (int)raw.size());
    refreshGroups();
    return tracks();
}

// ------------------------------------------------------------------------------ ingest
RawFileReader::RawFileReader(Context &ctx, const std::string &path, int64_t chunk_words)
    : ctx_(ctx), path_(path), chunk_(chunk_words > 0 ? chunk_words : int64_t(1) << 24) {
    check(ecc_raw_probe(path.c_str(), &info_), "ecc_raw_probe");
    const int64_t max_events = chunk_ * (info_.format == ECC_RAW_EVT3 ? 12 : 1);  // <= 12 per VECT_12 word
    host_.resize((size_t)(chunk_ * info_.word_bytes));
    words_.reserve(host_.size());
    xy_.reserve((size_t)max_events * 4);
    t_.reserve((size_t)max_events * 8);
    p_.reserve((size_t)max_events);
    n_.reserve(8);
    state_.reserve(ECC_EVT_STATE_BYTES);
    check(ecc_memset_async(state_.data(), 0, ECC_EVT_STATE_BYTES, ctx_.stream()), "memset(state)");
}

int64_t RawFileReader::next(const uint32_t **d_xy, const int64_t **d_t, const uint8_t **d_p) {
    const int64_t got = ecc_raw_read_words(path_.c_str(), &info_, pos_, chunk_, host_.data());
    if (got < 0) throw Error((int)got, "ecc_raw_read_words");
    if (got == 0) return 0;
    pos_ += got;
    words_.upload(host_.data(), (size_t)(got * info_.word_bytes), ctx_.stream());
    const int64_t cap = (int64_t)p_.size();
    check(ecc_evt_decode(ctx_.get(), info_.format, words_.data(), got, xy_.as<uint32_t>(), t_.as<int64_t>(),
                         p_.as<uint8_t>(), cap, n_.as<int64_t>(), state_.data(), ctx_.stream()),
          "ecc_evt_decode");
    int64_t n = 0;
    n_.download(&n, 8, ctx_.stream());
    ctx_.sync();
    if (d_xy) *d_xy = xy_.as<uint32_t>();
    if (d_t) *d_t = t_.as<int64_t>();
    if (d_p) *d_p = p_.as<uint8_t>();
    return n;
}

void RawFileReader::read_all(std::vector<uint32_t> &xy, std::vector<int64_t> &t, std::vector<uint8_t> &p) {
    xy.clear(); t.clear(); p.clear();
    pos_ = 0;
    check(ecc_memset_async(state_.data(), 0, ECC_EVT_STATE_BYTES, ctx_.stream()), "memset(state)");
    const uint32_t *dx;
    const int64_t *dt;
    const uint8_t *dp;
    for (int64_t n; (n = next(&dx, &dt, &dp)) > 0;) {
        const size_t o = xy.size();
        xy.resize(o + n); t.resize(o + n); p.resize(o + n);
        check(ecc_memcpy_d2h(xy.data() + o, dx, (size_t)n * 4, ctx_.stream()), "d2h xy");
        check(ecc_memcpy_d2h(t.data() + o, dt, (size_t)n * 8, ctx_.stream()), "d2h t");
        check(ecc_memcpy_d2h(p.data() + o, dp, (size_t)n, ctx_.stream()), "d2h p");
        ctx_.sync();
    }
}

std::vector<int64_t> reslice_n_events(int64_t n, int64_t n_events) {
    std::vector<int64_t> b;
    if (n_events <= 0) throw Error(ECC_ERR_INVALID, "reslice_n_events");
    for (int64_t k = 0; k < n; k += n_events) b.push_back(k);
    b.push_back(n);
    return b;
}

std::vector<int64_t> reslice_n_us(Context &ctx, const int64_t *d_t, int64_t n, int64_t period_us) {
    if (n <= 0) return {0};
    int64_t first = 0, last = 0;
    check(ecc_memcpy_d2h(&first, d_t, 8, ctx.stream()), "d2h t[0]");
    check(ecc_memcpy_d2h(&last, d_t + n - 1, 8, ctx.stream()), "d2h t[n-1]");
    ctx.sync();
    if (period_us <= 0 || last < first) throw Error(ECC_ERR_INVALID, "reslice_n_us");
    const int64_t base = (first >= 0 ? first / period_us : -((-first + period_us - 1) / period_us)) * period_us;
    const int64_t ns = (last - base) / period_us + 1;
    DeviceBuffer bounds((size_t)(ns + 1) * 8), d_ns(8);
    check(ecc_reslice_n_us(ctx.get(), d_t, n, period_us, bounds.as<int64_t>(), ns, d_ns.as<int64_t>(),
                           ctx.stream()),
          "ecc_reslice_n_us");
    check(ecc_evt_status(ctx.get(), ctx.stream()), "ecc_reslice_n_us");
    std::vector<int64_t> b((size_t)ns + 1);
    bounds.download(b.data(), b.size() * 8, ctx.stream());
    ctx.sync();
    return b;
}

TimeSurfaceCornerDetector::TimeSurfaceCornerDetector(Context &ctx, int width, int height,
                                                     int slice_events, int border_mode, bool any_order)
    : ctx_(ctx) {
    ecc_corner_cfg_default(&cfg_);
    cfg_.width = width;
    cfg_.height = height;
    cfg_.slice_events = slice_events;
    cfg_.border_mode = border_mode;
    cfg_.any_order = any_order ? 1 : 0;
    sae_.reserve((size_t)width * height * 8);
    check(ecc_memset_async(sae_.data(), 0, (size_t)width * height * 8, ctx.stream()), "memset(sae)");
}

void TimeSurfaceCornerDetector::detect(const uint32_t *d_xy, const int64_t *d_t, int64_t n,
                                       uint8_t *d_flags) {
    cfg_.first_detect_slice = first_ ? 1 : 0;
    check(ecc_fast_detect(ctx_.get(), d_xy, d_t, n, &cfg_, sae_.as<int64_t>(), d_flags, ctx_.stream()),
          "ecc_fast_detect");
    check(ecc_fast_detect_status(ctx_.get(), ctx_.stream()), "ecc_fast_detect");
    first_ = false;
}

// ------------------------------------------------------------------------------ downsample / k-means
HashDownsampler::HashDownsampler(Context &ctx, const ecc_hash_cfg *cfg) : ctx_(ctx) {
    if (cfg) cfg_ = *cfg;
    else ecc_hash_cfg_default(&cfg_);
}

void HashDownsampler::run(const uint32_t *d_xy, int64_t n, uint32_t *d_rep_xy, uint32_t *d_rep_idx,
                          int32_t *d_unique, int32_t *d_repeated) {
    check(ecc_downsample_hash(ctx_.get(), d_xy, n, &cfg_, d_rep_xy, d_rep_idx, d_unique, d_repeated,
                              ctx_.stream()), "ecc_downsample_hash");
}

DownsampleResult HashDownsampler::process(const std::vector<std::pair<int, int>> &coords) {
    const int64_t n = (int64_t)coords.size();
    const int64_t nw = (n + cfg_.window - 1) / cfg_.window;
    DownsampleResult r;
    r.unique_count.assign(nw, 0);
    r.repeated_count.assign(nw, 0);
    r.unique_coords.assign(nw, {});
    if (n == 0) return r;
    std::vector<uint32_t> xy(n);
    for (int64_t i = 0; i < n; ++i) {
        const int x = coords[i].first, y = coords[i].second;
        // negative / >u16 coordinates are outside 0<=x<=1280 anyway (:56); map them out of range
        xy[i] = (x < 0 || y < 0 || x > 65535 || y > 65535) ? 0xffffffffu : pack_xy(x, y);
    }
    DeviceBuffer d_xy, d_rep((size_t)nw * cfg_.window * 4), d_u((size_t)nw * 4), d_r((size_t)nw * 4);
    d_xy.upload(xy.data(), n * 4, ctx_.stream());
    run(d_xy.as<uint32_t>(), n, d_rep.as<uint32_t>(), nullptr, d_u.as<int32_t>(), d_r.as<int32_t>());
    std::vector<uint32_t> rep((size_t)nw * cfg_.window);
    d_u.download(r.unique_count.data(), nw * 4, ctx_.stream());
    d_r.download(r.repeated_count.data(), nw * 4, ctx_.stream());
    d_rep.download(rep.data(), rep.size() * 4, ctx_.stream());
    for (int64_t w = 0; w < nw; ++w)
        for (int k = 0; k < r.unique_count[w]; ++k) {
            const uint32_t v = rep[w * cfg_.window + k];
            r.unique_coords[w].push_back({(int)(v & 0xffff), (int)(v >> 16)});
        }
    return r;
}

int analyzeCoordinates(Context &ctx, const int *data, int n_ints, std::vector<CoordinateInfo> *coords) {
    const int n = n_ints / 2;  // the reference walks i = 0, 2, ... < ARRAY_SIZE (:74)
    if (n_ints < 0 || n > 8192) throw Error(ECC_ERR_INVALID, "analyzeCoordinates: more than 8192 pairs");
    if (coords) coords->clear();
    if (n == 0) return 0;
    std::vector<uint32_t> xy(n);
    for (int i = 0; i < n; ++i) {
        const int x = data[2 * i], y = data[2 * i + 1];
        if (x < 0 || y < 0 || x > 65535 || y > 65535)
            throw Error(ECC_ERR_INVALID, "analyzeCoordinates: coordinate outside 0..65535");
        xy[i] = pack_xy(x, y);
    }
    ecc_stream_t s = ctx.stream();
    DeviceBuffer d_xy, d_idx((size_t)n * 4), d_cnt((size_t)n * 4), d_u(4);
    d_xy.upload(xy.data(), (size_t)n * 4, s);
    check(ecc_dedup_exact(ctx.get(), d_xy.as<uint32_t>(), n, n, d_idx.as<uint32_t>(), d_cnt.as<int32_t>(),
                          d_u.as<int32_t>(), s),
          "ecc_dedup_exact");
    int32_t u = 0;
    d_u.download(&u, 4, s);
    std::vector<uint32_t> idx(coords ? n : 0);
    std::vector<int32_t> cnt(coords ? n : 0);
    if (coords) {
        d_idx.download(idx.data(), (size_t)n * 4, s);
        d_cnt.download(cnt.data(), (size_t)n * 4, s);
    }
    ctx.sync();  // one sync for the count and the lists
    if (coords)
        for (int k = 0; k < u; ++k) coords->push_back(CoordinateInfo{data[2 * idx[k]], data[2 * idx[k] + 1], cnt[k]});
    return u;
}

KMeans::KMeans(Context &ctx, int k, int max_iters, float threshold, float tol) : ctx_(ctx) {
    cfg_ = ecc_kmeans_cfg{k, max_iters, threshold, tol};
}

std::vector<uint8_t> KMeans::fit(const std::vector<std::array<float, 2>> &points,
                                 std::vector<std::array<float, 2>> &centroids, int *iters) {
    if ((int)centroids.size() != cfg_.k) throw Error(ECC_ERR_INVALID, "KMeans::fit: centroids.size() != k");
    const int64_t n = (int64_t)points.size();
    DeviceBuffer d_p, d_c, d_l(std::max<int64_t>(n, 1)), d_it(4);
    d_p.upload(points.data(), n * 8, ctx_.stream());
    d_c.upload(centroids.data(), cfg_.k * 8, ctx_.stream());
    check(ecc_kmeans_run_f32(ctx_.get(), d_p.as<float>(), n, &cfg_, d_c.as<float>(), d_l.as<uint8_t>(),
                             d_it.as<int32_t>(), ctx_.stream()), "ecc_kmeans_run_f32");
    std::vector<uint8_t> labels(n);
    d_l.download(labels.data(), n, ctx_.stream());
    d_c.download(centroids.data(), cfg_.k * 8, ctx_.stream());
    if (iters) d_it.download(iters, 4, ctx_.stream());
    return labels;
}

int KMeans::fit_ref_compat(Context &ctx, const std::vector<std::array<float, 2>> &points,
                           std::array<float, 16> &centroids, int max_passes, std::array<int32_t, 8> *bin_counts) {
    const int64_t n = (int64_t)points.size();
    DeviceBuffer d_p(std::max<int64_t>(n * 8, 8)), d_c(64), d_n(4), d_b(32);
    if (n) d_p.upload(points.data(), n * 8, ctx.stream());
    d_c.upload(centroids.data(), 64, ctx.stream());
    check(ecc_kmeans_refcompat_f32(ctx.get(), d_p.as<float>(), n, d_c.as<float>(), max_passes, d_n.as<int32_t>(),
                                   d_b.as<int32_t>(), nullptr, ctx.stream()),
          "ecc_kmeans_refcompat_f32");
    int32_t passes = 0;
    d_c.download(centroids.data(), 64, ctx.stream());
    d_n.download(&passes, 4, ctx.stream());
    if (bin_counts) d_b.download(bin_counts->data(), 32, ctx.stream());
    ctx.sync();
    return passes;
}

// ------------------------------------------------------------------------------ eps lists
void eps_neighbour_lists(Context &ctx, const std::vector<std::array<int, 2>> &points, double eps,
                         std::vector<int64_t> &offsets, std::vector<int32_t> &nbr, int min_pts,
                         std::vector<double> *core_dist) {
    const int64_t n = (int64_t)points.size();
    offsets.assign(n + 1, 0);
    nbr.clear();
    if (n == 0) return;
    ecc_stream_t s = ctx.stream();
    int mnx = points[0][0], mny = points[0][1], mxx = mnx, mxy = mny;
    for (const auto &p : points) {
        mnx = std::min(mnx, p[0]); mny = std::min(mny, p[1]);
        mxx = std::max(mxx, p[0]); mxy = std::max(mxy, p[1]);
    }
    const bool windowed = n <= 16384 && (int64_t)mxx - mnx <= 65535 && (int64_t)mxy - mny <= 65535 &&
                          (!core_dist || min_pts <= 64);
    DeviceBuffer d_cnt(n * 4), d_core(core_dist ? n * 8 : 8), d_off((n + 1) * 8), d_pts;
    if (windowed) {  // one segment of packed u16 pixels (translation keeps every distance)
        std::vector<uint32_t> xy(n);
        for (int64_t i = 0; i < n; ++i) xy[i] = pack_xy(points[i][0] - mnx, points[i][1] - mny);
        d_pts.upload(xy.data(), n * 4, s);
        check(ecc_eps_counts(ctx.get(), d_pts.as<uint32_t>(), 1, n, nullptr, eps, std::max(1, min_pts),
                             d_cnt.as<int32_t>(), core_dist ? d_core.as<double>() : nullptr, s),
              "ecc_eps_counts");
    } else {  // any size / span / min_pts: the global grid over the points as doubles (exact for int)
        std::vector<double> f(2 * n);
        for (int64_t i = 0; i < n; ++i) { f[2 * i] = points[i][0]; f[2 * i + 1] = points[i][1]; }
        d_pts.upload(f.data(), f.size() * 8, s);
        check(ecc_radius_counts_f64(ctx.get(), d_pts.as<double>(), n, 2, eps, std::max(1, min_pts), d_cnt.as<int32_t>(),
                                    core_dist ? d_core.as<double>() : nullptr, s),
              "ecc_radius_counts_f64");
    }
    // list size from the counts (one small readback, as the reference reads sizes back)
    std::vector<int32_t> cnt(n);
    d_cnt.download(cnt.data(), n * 4, s);
    int64_t total = 0;
    for (int32_t c : cnt) total += c;
    DeviceBuffer d_nbr(std::max<int64_t>(total, 1) * 4);
    if (windowed) {
        check(ecc_eps_lists(ctx.get(), d_pts.as<uint32_t>(), 1, n, nullptr, eps, d_cnt.as<int32_t>(),
                            d_off.as<int64_t>(), d_nbr.as<int32_t>(), total, s),
              "ecc_eps_lists");
        int64_t tot2 = 0;
        check(ecc_eps_total(ctx.get(), d_off.as<int64_t>(), n, &tot2, s), "ecc_eps_lists capacity");
    } else {
        check(ecc_radius_lists_f64(ctx.get(), d_pts.as<double>(), n, 2, eps, d_cnt.as<int32_t>(), d_off.as<int64_t>(),
                                   d_nbr.as<int32_t>(), nullptr, total, s),
              "ecc_radius_lists_f64");
        check(ecc_lists_sort_ascending(ctx.get(), n, d_off.as<int64_t>(), total, d_nbr.as<int32_t>(), nullptr, s),
              "ecc_lists_sort_ascending");
        check(ecc_radius_status(ctx.get(), s), "ecc_radius_lists_f64");
    }
    offsets.resize(n + 1);
    nbr.resize(total);
    d_off.download(offsets.data(), (n + 1) * 8, s);
    d_nbr.download(nbr.data(), total * 4, s);
    if (core_dist) {
        core_dist->resize(n);
        d_core.download(core_dist->data(), n * 8, s);
    }
    ctx.sync();
}

// ------------------------------------------------------------------------------ OPTICS
namespace optics {

std::string reachability_dist::to_string() const {
    return "{" + std::to_string(point_index) + "," + std::to_string(reach_dist) + "}";
}

bool operator<(const reachability_dist &l, const reachability_dist &r) {
    return (l.reach_dist <= r.reach_dist && l.reach_dist >= r.reach_dist) ? (l.point_index < r.point_index)
                                                                          : (l.reach_dist < r.reach_dist);
}

bool operator==(const reachability_dist &l, const reachability_dist &r) {
    return (l.reach_dist <= r.reach_dist && l.reach_dist >= r.reach_dist) && (l.point_index == r.point_index);
}

namespace {

// GPU eps-balls (ecc_radius_*_f64: counts, core distances, lists) + the ordered expansion on the
// host (optics.hpp:525-555, sequential by nature) for n points of D doubles (host, row-major).
// The seed set (a std::set ordered by (reach, index), :67-69, erase + re-insert on a decrease)
// is a binary heap with lazy deletion: reachabilities only decrease, so a superseded entry is
// larger than the live one and is skipped when popped — the live entries pop in the same
// (reach, index) order as from the set.
std::vector<reachability_dist> optics_f64(ecc_ctx *ctx, ecc_stream_t s, const double *pts, int64_t n, int D,
                                          std::size_t min_pts, double epsilon) {
    if (n == 0) return {};
    if (min_pts < 1) throw Error(ECC_ERR_INVALID, "compute_reachability_dists: min_pts must be >= 1");
    if (D < 1 || D > 3) throw Error(ECC_ERR_INVALID, "compute_reachability_dists: dimension must be 1..3");
    if (n >= INT32_MAX) throw Error(ECC_ERR_INVALID, "compute_reachability_dists: too many points");
    static const bool timing = std::getenv("ECC_OPTICS_TIMING") != nullptr;  // phase split to stderr
    auto t_last = std::chrono::steady_clock::now();
    auto mark = [&](const char *what) {
        if (!timing) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "optics_f64 %-10s %8.2f ms\n", what,
                     std::chrono::duration<double, std::milli>(now - t_last).count());
        t_last = now;
    };
    DeviceBuffer d_pts, d_cnt((size_t)n * 4), d_core((size_t)n * 8), d_off((size_t)(n + 1) * 8);
    d_pts.upload(pts, (size_t)n * D * 8, s);
    check(ecc_radius_counts_f64(ctx, d_pts.as<double>(), n, D, epsilon, (int32_t)min_pts, d_cnt.as<int32_t>(),
                                d_core.as<double>(), s),
          "ecc_radius_counts_f64");
    check(ecc_radius_lists_f64(ctx, d_pts.as<double>(), n, D, epsilon, d_cnt.as<int32_t>(), d_off.as<int64_t>(), nullptr,
                               nullptr, 0, s),
          "ecc_radius_lists_f64 (size)");
    int64_t total = 0;
    check(ecc_memcpy_d2h(&total, d_off.as<int64_t>() + n, 8, s), "read list size");
    check(ecc_stream_sync(s), "sync");
    mark("counts");
    DeviceBuffer d_nbr((size_t)std::max<int64_t>(total, 1) * 4), d_nd((size_t)std::max<int64_t>(total, 1) * 8);
    check(ecc_radius_lists_f64(ctx, d_pts.as<double>(), n, D, epsilon, d_cnt.as<int32_t>(), d_off.as<int64_t>(),
                               d_nbr.as<int32_t>(), d_nd.as<double>(), total, s),
          "ecc_radius_lists_f64");
    std::vector<int64_t> off((size_t)n + 1);
    std::vector<int32_t> nbr((size_t)total);
    std::vector<double> nd((size_t)total);
    std::vector<double> core((size_t)n);
    d_off.download(off.data(), off.size() * 8, s);
    d_nbr.download(nbr.data(), nbr.size() * 4, s);
    d_nd.download(nd.data(), nd.size() * 8, s);
    d_core.download(core.data(), core.size() * 8, s);
    check(ecc_stream_sync(s), "sync");
    check(ecc_radius_status(ctx, s), "ecc_radius_lists_f64 capacity");
    mark("lists+copy");
    struct Seed {
        double r;
        int64_t idx;
    };
    auto after = [](const Seed &a, const Seed &b) {  // heap order: the smallest (reach, index) on top
        return (a.r <= b.r && a.r >= b.r) ? (a.idx > b.idx) : (a.r > b.r);
    };
    std::vector<Seed> heap;
    std::vector<char> processed((size_t)n, 0);
    std::vector<double> reach((size_t)n, -1.0);
    std::vector<int64_t> ordered;
    ordered.reserve((size_t)n);
    auto update = [&](int64_t p, double cd) {  // :315-337
        for (int64_t k = off[p]; k < off[p + 1]; ++k) {
            const int64_t o = nbr[k];
            if (processed[o]) continue;
            const double nr = std::max(cd, nd[k]);  // geom::dist(point, points[o]), from the GPU
            if (reach[o] < 0.0 || nr < reach[o]) {
                reach[o] = nr;
                heap.push_back(Seed{nr, o});
                std::push_heap(heap.begin(), heap.end(), after);
            }
        }
    };
    for (int64_t p = 0; p < n; ++p) {  // :525-555
        if (processed[p]) continue;
        processed[p] = 1;
        ordered.push_back(p);
        if (core[p] < 0.0) continue;
        update(p, core[p]);
        while (!heap.empty()) {
            std::pop_heap(heap.begin(), heap.end(), after);
            const Seed sd = heap.back();
            heap.pop_back();
            if (processed[sd.idx] || !(sd.r <= reach[sd.idx] && sd.r >= reach[sd.idx])) continue;  // superseded
            processed[sd.idx] = 1;
            ordered.push_back(sd.idx);
            if (core[sd.idx] < 0.0) continue;
            update(sd.idx, core[sd.idx]);
        }
    }
    mark("expansion");
    std::vector<reachability_dist> result;
    result.reserve((size_t)n);
    for (int64_t idx : ordered) result.emplace_back((std::size_t)idx, reach[idx]);
    return result;
}

template <typename T, std::size_t D>
std::vector<reachability_dist> optics_points(Context &ctx, const std::vector<std::array<T, D>> &points,
                                             std::size_t min_pts, double epsilon) {
    if (points.empty()) return {};
    if (epsilon <= 0.0) epsilon = epsilon_estimation(points, min_pts);  // optics.hpp:428-430
    // square_distance takes d = p1[i] - p2[i] in the coordinate type, then d * d in double
    // (kdTree.hpp:186-187): exact in double for int and double coordinates alike
    std::vector<double> flat(points.size() * D);
    for (std::size_t i = 0; i < points.size(); ++i)
        for (std::size_t d = 0; d < D; ++d) flat[i * D + d] = static_cast<double>(points[i][d]);
    return optics_f64(ctx.get(), ctx.stream(), flat.data(), (int64_t)points.size(), (int)D, min_pts, epsilon);
}

}  // namespace

std::vector<reachability_dist> optics_f64_export(ecc_ctx *ctx, ecc_stream_t s, const double *pts, int64_t n, int D,
                                                 std::size_t min_pts, double epsilon) {
    return optics_f64(ctx, s, pts, n, D, min_pts, epsilon);
}

std::vector<reachability_dist> compute_reachability_dists(Context &ctx, const std::vector<std::array<int, 2>> &points,
                                                          std::size_t min_pts, double epsilon) {
    return optics_points(ctx, points, min_pts, epsilon);
}
std::vector<reachability_dist> compute_reachability_dists(Context &ctx, const std::vector<std::array<int, 3>> &points,
                                                          std::size_t min_pts, double epsilon) {
    return optics_points(ctx, points, min_pts, epsilon);
}
std::vector<reachability_dist> compute_reachability_dists(Context &ctx, const std::vector<std::array<double, 1>> &points,
                                                          std::size_t min_pts, double epsilon) {
    return optics_points(ctx, points, min_pts, epsilon);
}
std::vector<reachability_dist> compute_reachability_dists(Context &ctx, const std::vector<std::array<double, 2>> &points,
                                                          std::size_t min_pts, double epsilon) {
    return optics_points(ctx, points, min_pts, epsilon);
}
std::vector<reachability_dist> compute_reachability_dists(Context &ctx, const std::vector<std::array<double, 3>> &points,
                                                          std::size_t min_pts, double epsilon) {
    return optics_points(ctx, points, min_pts, epsilon);
}
std::vector<reachability_dist> compute_reachability_dists(const std::vector<std::array<int, 2>> &points,
                                                          std::size_t min_pts, double epsilon) {
    return optics_points(Context::default_context(), points, min_pts, epsilon);
}
std::vector<reachability_dist> compute_reachability_dists(const std::vector<std::array<int, 3>> &points,
                                                          std::size_t min_pts, double epsilon) {
    return optics_points(Context::default_context(), points, min_pts, epsilon);
}
std::vector<reachability_dist> compute_reachability_dists(const std::vector<std::array<double, 1>> &points,
                                                          std::size_t min_pts, double epsilon) {
    return optics_points(Context::default_context(), points, min_pts, epsilon);
}
std::vector<reachability_dist> compute_reachability_dists(const std::vector<std::array<double, 2>> &points,
                                                          std::size_t min_pts, double epsilon) {
    return optics_points(Context::default_context(), points, min_pts, epsilon);
}
std::vector<reachability_dist> compute_reachability_dists(const std::vector<std::array<double, 3>> &points,
                                                          std::size_t min_pts, double epsilon) {
    return optics_points(Context::default_context(), points, min_pts, epsilon);
}

std::vector<std::vector<std::size_t>> get_cluster_indices(const std::vector<reachability_dist> &rd,
                                                          double thr) {  // optics.hpp:674-690
    std::vector<std::vector<std::size_t>> result;
    for (const auto &r : rd) {
        if (r.reach_dist < 0.0 || r.reach_dist >= thr || result.empty()) result.push_back({r.point_index});
        else result.back().push_back(r.point_index);
    }
    return result;
}

}  // namespace optics

// ------------------------------------------------------------------------------ DBSCAN
void DBSCANSimpleCluster::extract(std::vector<PointIndices> &cluster_indices) {  // DBSCAN_simple.h:27-90
    // The reference's own input (float x, y, z; any size): radiusSearch (:118-142) and the
    // seed-queue expansion (union-find closed form) both run on the GPU over one global cell grid
    // (ecc_dbscan_cloud_f32); the host only turns labels + duplicate memberships into PointIndices.
    cluster_indices.clear();
    const int64_t n = (int64_t)cloud_.size();
    if (n == 0) return;
    static_assert(sizeof(PointXYZ) == 12, "PointXYZ must be three packed floats");
    ecc_stream_t s = ctx_.stream();
    DeviceBuffer d_pts, d_lab(n * 4), d_nc(4), d_nd(8);
    d_pts.upload(cloud_.data(), (size_t)n * 12, s);
    int64_t dup_cap = std::max<int64_t>(n, 1024), nd = 0;
    DeviceBuffer d_dups;
    for (;;) {
        d_dups.reserve((size_t)dup_cap * 16);
        check(ecc_dbscan_cloud_f32(ctx_.get(), reinterpret_cast<const float *>(d_pts.data()), n, 3, searchTolerance(), minPts_,
                                   min_pts_per_cluster_, max_pts_per_cluster_, d_lab.as<int32_t>(), d_nc.as<int32_t>(),
                                   d_dups.as<int64_t>(), dup_cap, d_nd.as<int64_t>(), s),
              "ecc_dbscan_cloud_f32");
        const int st = ecc_dbscan_cloud_status(ctx_.get(), s);
        d_nd.download(&nd, 8, s);
        ctx_.sync();
        if (st == ECC_ERR_CAPACITY && nd > dup_cap) {  // more duplicate memberships than room: grow, rerun
            dup_cap = nd;
            continue;
        }
        check(st, "ecc_dbscan_cloud_f32");
        break;
    }
    int32_t nc = 0;
    std::vector<int32_t> lab(n);
    d_nc.download(&nc, 4, s);
    d_lab.download(lab.data(), n * 4, s);
    std::vector<int64_t> dups((size_t)nd * 2);
    if (nd) d_dups.download(dups.data(), (size_t)nd * 16, s);
    ctx_.sync();
    std::vector<std::vector<int>> members((size_t)nc);
    for (int64_t i = 0; i < n; ++i)
        if (lab[i] >= 0) members[lab[i]].push_back((int)i);
    for (int64_t k = 0; k < nd; ++k) members[dups[2 * k + 1]].push_back((int)dups[2 * k]);
    for (auto &m : members) {
        std::sort(m.begin(), m.end());  // :82
        cluster_indices.push_back(PointIndices{m});
    }
}

}  // namespace ecc

// C ABI of the OPTICS entry (optics::compute_reachability_dists, OPT/include/optics/optics.hpp:
// 413-565) for bindings: HOST points in, HOST ordering out.
extern "C" __attribute__((visibility("default"))) int ecc_optics_f64(ecc_ctx *ctx, const double *pts, int64_t n,
                                                                    int32_t dim, int32_t min_pts, double eps,
                                                                    int64_t *order, double *reach, ecc_stream_t stream) {
    if (!ctx || n < 0 || (n > 0 && (!pts || !order || !reach)) || dim < 1 || dim > 3) return ECC_ERR_INVALID;
    try {
        if (n == 0) return ECC_OK;
        if (eps <= 0.0) {  // optics.hpp:369-387 (bounding box max from points[1], Q20)
            if (n <= 1) {
                eps = 0.0;
            } else {
                double mn[3], mx[3];
                for (int d = 0; d < dim; ++d) { mn[d] = pts[d]; mx[d] = pts[dim + d]; }
                for (int64_t i = 0; i < n; ++i)
                    for (int d = 0; d < dim; ++d) {
                        if (pts[i * dim + d] < mn[d]) mn[d] = pts[i * dim + d];
                        if (pts[i * dim + d] > mx[d]) mx[d] = pts[i * dim + d];
                    }
                double vol = 1;
                for (int d = 0; d < dim; ++d) vol *= std::abs(mx[d] - mn[d]);
                const double dd = (double)dim;
                const double space = (vol / (double)n) * (double)min_pts;
                const double ball = std::sqrt(std::pow(M_PI, dd)) / std::tgamma(dd / 2.0 + 1.0);
                eps = std::pow(space / ball, 1.0 / dd);
            }
        }
        const auto r = ecc::optics::optics_f64_export(ctx, stream, pts, n, dim, (std::size_t)min_pts, eps);
        for (int64_t i = 0; i < n; ++i) {
            order[i] = (int64_t)r[i].point_index;
            reach[i] = r[i].reach_dist;
        }
        return ECC_OK;
    } catch (const ecc::Error &e) {
        return e.status();
    } catch (...) {
        return ECC_ERR_NOMEM;
    }
}
