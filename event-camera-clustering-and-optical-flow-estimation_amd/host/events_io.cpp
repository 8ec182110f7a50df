// Host-side event sources: deterministic synthetic streams, CSV event files and the RAW
// (EVT 2.0 / EVT 3.0) file header + payload reader.
//
// The reference ingests events through Metavision's Camera::from_file(argv[1]) / live camera
// callbacks (FCT/…group_track.cpp:756-765, 1073-1074) and its OPTICS driver reads "x,y,t,p" CSV
// files (OPT/test/cluster_event_data.cpp:21-55, fixture OPT/test/event_raw_data8.csv).  RAW
// payload words are decoded on the GPU (csrc/evt.hip, ecc_evt_decode); this file only parses
// the '%' header and streams the little-endian words from disk.
//
// Generator: counter-based splitmix64 streams, so any slice [first, first+n) of
// an event stream can be produced independently and in parallel; 70 % edge events of moving
// convex polygons (so the time surface has corners), 20 % Gaussian blobs (sigma 4 px, so
// k-means has structure), 10 % uniform noise; t non-decreasing at `rate` events per µs.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/ecc.h"

#define ECC_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() { s += 0x9E3779B97F4A7C15ull; return splitmix64(s); }
    double uni() { return (double)(next() >> 11) * 0x1.0p-53; }  // [0,1)
};

struct Polygon {
    double cx0, cy0, vx, vy;  // px, px/µs
    double r, ang0, omega;    // px, rad, rad/µs
    int sides;
};

struct Scene {
    std::vector<Polygon> polys;
    std::vector<double> bx, by;
};

Scene make_scene(const ecc_gen_cfg &c) {
    Scene sc;
    Rng r(splitmix64(c.seed ^ 0x5CE7E5CE7E5CE7Eull));
    for (int i = 0; i < c.n_polygons; ++i) {
        Polygon p;
        p.r = 12.0 + 18.0 * r.uni() * std::min(1.0, std::min(c.width, c.height) / 120.0);
        p.cx0 = p.r + r.uni() * std::max(1.0, c.width - 2 * p.r);
        p.cy0 = p.r + r.uni() * std::max(1.0, c.height - 2 * p.r);
        const double speed = (0.5 + 4.5 * r.uni()) / 1000.0;  // 0.5..5 px/ms
        const double dir = 2 * M_PI * r.uni();
        p.vx = speed * std::cos(dir);
        p.vy = speed * std::sin(dir);
        p.ang0 = 2 * M_PI * r.uni();
        p.omega = (r.uni() - 0.5) * 2e-6;
        p.sides = 3 + (int)(r.uni() * 4.0);
        sc.polys.push_back(p);
    }
    for (int i = 0; i < c.n_blobs; ++i) {
        sc.bx.push_back(8 + r.uni() * std::max(1.0, c.width - 16.0));
        sc.by.push_back(8 + r.uni() * std::max(1.0, c.height - 16.0));
    }
    return sc;
}

// reflect a coordinate into [lo, hi] (triangle wave)
inline double bounce(double v, double lo, double hi) {
    const double span = hi - lo;
    if (span <= 0) return lo;
    double u = std::fmod(v - lo, 2 * span);
    if (u < 0) u += 2 * span;
    return lo + (u <= span ? u : 2 * span - u);
}

void gen_range(const ecc_gen_cfg &c, const Scene &sc, int64_t first, int64_t n, uint32_t *xy,
               int64_t *t, uint8_t *p) {
    const uint64_t key = splitmix64(c.seed);
    for (int64_t k = 0; k < n; ++k) {
        const int64_t i = first + k;
        const int64_t ti = c.t0 + (int64_t)std::floor((double)i / c.rate_mev_s);
        Rng r(key ^ splitmix64((uint64_t)i));
        const double u = r.uni();
        double x, y;
        if (u < c.frac_edges && !sc.polys.empty()) {
            const Polygon &pg = sc.polys[(size_t)(r.uni() * sc.polys.size()) % sc.polys.size()];
            const double tt = (double)(ti - c.t0);
            const double cx = bounce(pg.cx0 + pg.vx * tt, pg.r, c.width - 1 - pg.r);
            const double cy = bounce(pg.cy0 + pg.vy * tt, pg.r, c.height - 1 - pg.r);
            const double ang = pg.ang0 + pg.omega * tt;
            const int e = (int)(r.uni() * pg.sides) % pg.sides;
            const double a0 = ang + 2 * M_PI * e / pg.sides, a1 = ang + 2 * M_PI * (e + 1) / pg.sides;
            const double lam = r.uni();
            x = cx + pg.r * ((1 - lam) * std::cos(a0) + lam * std::cos(a1));
            y = cy + pg.r * ((1 - lam) * std::sin(a0) + lam * std::sin(a1));
        } else if (u < c.frac_edges + c.frac_blobs && !sc.bx.empty()) {
            const size_t b = (size_t)(r.uni() * sc.bx.size()) % sc.bx.size();
            const double u1 = std::max(r.uni(), 1e-300), u2 = r.uni();
            const double rad = std::sqrt(-2.0 * std::log(u1)) * 4.0;  // sigma 4 px
            x = sc.bx[b] + rad * std::cos(2 * M_PI * u2);
            y = sc.by[b] + rad * std::sin(2 * M_PI * u2);
        } else {
            x = r.uni() * c.width;
            y = r.uni() * c.height;
        }
        int xi = (int)std::floor(x + 0.5), yi = (int)std::floor(y + 0.5);
        xi = std::min(std::max(xi, 0), c.width - 1);
        yi = std::min(std::max(yi, 0), c.height - 1);
        if (xy) xy[k] = (uint32_t)xi | ((uint32_t)yi << 16);
        if (t) t[k] = ti;
        if (p) p[k] = (uint8_t)(r.next() & 1u);
    }
}

}  // namespace

ECC_HOST_API void ecc_gen_cfg_default(ecc_gen_cfg *c) {
    if (!c) return;
    c->seed = 1;
    c->width = 346;
    c->height = 260;
    c->rate_mev_s = 10.0;
    c->t0 = 0;
    c->n_polygons = 8;
    c->n_blobs = 16;
    c->frac_edges = 0.7f;
    c->frac_blobs = 0.2f;
}

ECC_HOST_API int ecc_gen_events(const ecc_gen_cfg *c, int64_t first, int64_t n, uint32_t *xy,
                                int64_t *t, uint8_t *p) {
    if (!c || n < 0 || first < 0 || c->width < 1 || c->height < 1 || c->width > 65535 ||
        c->height > 65535 || !(c->rate_mev_s > 0))
        return ECC_ERR_INVALID;
    const Scene sc = make_scene(*c);
    unsigned nt = std::thread::hardware_concurrency();
    if (const char *e = std::getenv("OMP_NUM_THREADS")) nt = std::max(1, std::atoi(e));
    nt = std::max(1u, std::min(nt, 16u));
    if (n < (int64_t)1 << 16) nt = 1;
    std::vector<std::thread> th;
    const int64_t per = (n + nt - 1) / nt;
    for (unsigned w = 0; w < nt; ++w) {
        const int64_t lo = w * per, hi = std::min<int64_t>(n, lo + per);
        if (lo >= hi) break;
        th.emplace_back([&, lo, hi] {
            gen_range(*c, sc, first + lo, hi - lo, xy ? xy + lo : nullptr, t ? t + lo : nullptr,
                      p ? p + lo : nullptr);
        });
    }
    for (auto &x : th) x.join();
    return ECC_OK;
}

// CSV "x,y,t,p" per line (OPT/test/event_raw_data8.csv); lines that do not parse are skipped.
static int64_t csv_scan(const char *path, uint32_t *xy, int64_t *t, uint8_t *p, int64_t cap) {
    FILE *f = std::fopen(path, "r");
    if (!f) return ECC_ERR_INVALID;
    char line[512];
    int64_t n = 0;
    while (std::fgets(line, sizeof(line), f)) {
        long long x, y, ts = 0, pol = 0;
        const int got = std::sscanf(line, "%lld,%lld,%lld,%lld", &x, &y, &ts, &pol);
        if (got < 2 || x < 0 || y < 0 || x > 65535 || y > 65535) continue;
        if (n < cap) {
            if (xy) xy[n] = (uint32_t)x | ((uint32_t)y << 16);
            if (t) t[n] = ts;
            if (p) p[n] = (uint8_t)(pol != 0);
        }
        ++n;
    }
    std::fclose(f);
    return n;
}

ECC_HOST_API int64_t ecc_count_csv(const char *path) {
    return csv_scan(path, nullptr, nullptr, nullptr, 0);
}

ECC_HOST_API int64_t ecc_read_csv(const char *path, uint32_t *xy, int64_t *t, uint8_t *p, int64_t cap) {
    const int64_t n = csv_scan(path, xy, t, p, cap);
    return n < 0 ? n : std::min(n, cap);
}

// ---- RAW files (include/ecc.h §8) ----------------------------------------------------------
// Header: lines starting with '%' up to "% end" (or the first line not starting with '%').
// Recognised keys: "% evt 2.0|3.0", "% format EVT2|EVT3[;height=H;width=W]", "% geometry WxH".
static int parse_format_name(const char *v) {
    if (!std::strncmp(v, "EVT3", 4) || !std::strncmp(v, "evt3", 4) || !std::strncmp(v, "3.0", 3)) return ECC_RAW_EVT3;
    if (!std::strncmp(v, "EVT2", 4) || !std::strncmp(v, "evt2", 4) || !std::strncmp(v, "2.0", 3)) return ECC_RAW_EVT2;
    return ECC_RAW_UNKNOWN;
}

ECC_HOST_API int ecc_raw_probe(const char *path, ecc_raw_info *info) {
    if (!path || !info) return ECC_ERR_INVALID;
    std::memset(info, 0, sizeof(*info));
    FILE *f = std::fopen(path, "rb");
    if (!f) return ECC_ERR_INVALID;
    int64_t pos = 0;
    char line[1024];
    for (;;) {
        const int c = std::fgetc(f);
        if (c != '%') break;  // payload starts here
        std::ungetc(c, f);
        if (!std::fgets(line, sizeof(line), f)) break;
        const size_t len = std::strlen(line);
        pos += (int64_t)len;
        if (len == sizeof(line) - 1 && line[len - 1] != '\n') {  // over-long header line: skip the rest
            int d;
            while ((d = std::fgetc(f)) != EOF && d != '\n') ++pos;
            if (d == '\n') ++pos;
        }
        char *v = line + 1;
        while (*v == ' ') ++v;
        if (!std::strncmp(v, "end", 3) && (v[3] == '\n' || v[3] == '\r' || v[3] == 0)) break;
        if (!std::strncmp(v, "evt ", 4)) {
            info->format = parse_format_name(v + 4);
        } else if (!std::strncmp(v, "format ", 7)) {
            const int fmt = parse_format_name(v + 7);
            if (fmt) info->format = fmt;
            const char *h = std::strstr(v, "height="), *w = std::strstr(v, "width=");
            if (h) info->height = std::atoi(h + 7);
            if (w) info->width = std::atoi(w + 6);
        } else if (!std::strncmp(v, "geometry ", 9)) {
            int w = 0, h = 0;
            if (std::sscanf(v + 9, "%dx%d", &w, &h) == 2) {
                info->width = w;
                info->height = h;
            }
        }
    }
    std::fseek(f, 0, SEEK_END);
    const int64_t size = (int64_t)std::ftell(f);
    std::fclose(f);
    if (info->format == ECC_RAW_UNKNOWN) return ECC_ERR_INVALID;
    info->word_bytes = info->format == ECC_RAW_EVT2 ? 4 : 2;
    info->header_bytes = pos;
    info->n_words = size > pos ? (size - pos) / info->word_bytes : 0;
    return ECC_OK;
}

ECC_HOST_API int64_t ecc_raw_read_words(const char *path, const ecc_raw_info *info, int64_t first_word, int64_t n,
                                        void *buf) {
    if (!path || !info || !buf || first_word < 0 || n < 0 || info->word_bytes <= 0) return ECC_ERR_INVALID;
    if (first_word >= info->n_words) return 0;
    n = std::min(n, info->n_words - first_word);
    FILE *f = std::fopen(path, "rb");
    if (!f) return ECC_ERR_INVALID;
    if (std::fseek(f, (long)(info->header_bytes + first_word * info->word_bytes), SEEK_SET) != 0) {
        std::fclose(f);
        return ECC_ERR_INVALID;
    }
    const size_t got = std::fread(buf, (size_t)info->word_bytes, (size_t)n, f);
    std::fclose(f);
    return (int64_t)got;  // little-endian host (x86-64): words are used as read
}

// RAW writer (include/ecc.h §8).  EVT 2.0: TIME_HIGH on every change of t >> 6.  EVT 3.0:
// TIME_HIGH on every change of t >> 12 (with 0xFFF, 0 pairs per 2^24 loop crossed), TIME_LOW
// on every change of t, ADDR_Y on every change of y, vector words for row runs.
ECC_HOST_API int64_t ecc_evt_encode(int32_t format, const uint32_t *xy, const int64_t *t, const uint8_t *p,
                                    int64_t n, void *out, int64_t cap) {
    if (n < 0 || cap < 0 || (n > 0 && (!xy || !t || !p)) || (cap > 0 && !out)) return ECC_ERR_INVALID;
    int64_t k = 0;
    if (format == ECC_RAW_EVT2) {
        auto *o = static_cast<uint32_t *>(out);
        int64_t last = -1;
        for (int64_t i = 0; i < n; ++i) {
            if (i && t[i] < t[i - 1]) return ECC_ERR_UNSORTED_TIME;
            const int64_t th = t[i] >> 6;
            if (th != last) {
                if (k < cap) o[k] = 0x80000000u | (uint32_t)(th & 0x0FFFFFFF);
                ++k;
                last = th;
            }
            const uint32_t x = xy[i] & 0x7FFu, y = (xy[i] >> 16) & 0x7FFu;
            if (k < cap) o[k] = ((uint32_t)(p[i] & 1u) << 28) | ((uint32_t)(t[i] & 63) << 22) | (x << 11) | y;
            ++k;
        }
        return k;
    }
    if (format != ECC_RAW_EVT3) return ECC_ERR_INVALID;
    auto *o = static_cast<uint16_t *>(out);
    auto put = [&](uint32_t v) {
        if (k < cap) o[k] = (uint16_t)v;
        ++k;
    };
    int64_t last_hi = -1, last_t = -1, last_y = -1;
    for (int64_t i = 0; i < n;) {
        if (i && t[i] < t[i - 1]) return ECC_ERR_UNSORTED_TIME;
        const int64_t ti = t[i], hi = ti >> 12;
        if (hi != last_hi) {
            if (last_hi >= 0)
                for (int64_t L = last_hi >> 12; L < (hi >> 12); ++L) {
                    put(0x8FFFu);
                    put(0x8000u);
                }
            put(0x8000u | (uint32_t)(hi & 0xFFF));
            last_hi = hi;
            last_t = -1;
        }
        if (ti != last_t) {
            put(0x6000u | (uint32_t)(ti & 0xFFF));
            last_t = ti;
        }
        const uint32_t y = (xy[i] >> 16) & 0x7FFu, x0 = xy[i] & 0x7FFu, pi = p[i] & 1u;
        if ((int64_t)y != last_y) {
            put(y);
            last_y = y;
        }
        int64_t j = i + 1;
        while (j < n && t[j] == ti && ((xy[j] >> 16) & 0x7FFu) == y && (p[j] & 1u) == pi &&
               (xy[j] & 0x7FFu) > (xy[j - 1] & 0x7FFu) && (xy[j] & 0x7FFu) < x0 + 12)
            ++j;
        if (j - i >= 3) {
            uint32_t m = 0;
            for (int64_t q = i; q < j; ++q) m |= 1u << ((xy[q] & 0x7FFu) - x0);
            put(0x3000u | (pi << 11) | x0);
            put(0x4000u | m);
            i = j;
        } else {
            put(0x2000u | (pi << 11) | x0);
            ++i;
        }
    }
    return k;
}
