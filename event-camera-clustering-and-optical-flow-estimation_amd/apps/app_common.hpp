// Shared helpers of the host programs: event input as argv[1], the way the reference mains take
// Camera::from_file(argv[1]) — a Prophesee RAW recording (EVT 2.0 / 3.0, GPU-decoded), a CSV
// "x,y,t,p" file, or --synthetic N for a seeded stream.
#pragma once
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ecc.hpp"

struct Events {
    std::vector<uint32_t> xy;
    std::vector<int64_t> t;
    std::vector<uint8_t> p;
};

inline Events load_events(int argc, char **argv, int width, int height) {
    Events ev;
    if (argc >= 3 && !std::strcmp(argv[1], "--synthetic")) {
        const int64_t n = std::atoll(argv[2]);
        ecc_gen_cfg g;
        ecc_gen_cfg_default(&g);
        g.width = width;
        g.height = height;
        ev.xy.resize(n); ev.t.resize(n); ev.p.resize(n);
        if (ecc_gen_events(&g, 0, n, ev.xy.data(), ev.t.data(), ev.p.data()) != ECC_OK) {
            std::fprintf(stderr, "event generation failed\n");
            std::exit(1);
        }
        return ev;
    }
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <events.raw|events.csv> | --synthetic N\n", argv[0]);
        std::exit(1);
    }
    const size_t len = std::strlen(argv[1]);
    if (len > 4 && !std::strcmp(argv[1] + len - 4, ".raw")) {
        try {
            ecc::RawFileReader rd(ecc::Context::default_context(), argv[1]);
            rd.read_all(ev.xy, ev.t, ev.p);
        } catch (const ecc::Error &e) {
            std::fprintf(stderr, "%s: %s\n", argv[1], e.what());
            std::exit(1);
        }
        return ev;
    }
    const int64_t n = ecc_count_csv(argv[1]);
    if (n < 0) {
        std::perror(argv[1]);  // reference style: perror + exit(1)
        std::exit(1);
    }
    ev.xy.resize(n); ev.t.resize(n); ev.p.resize(n);
    ecc_read_csv(argv[1], ev.xy.data(), ev.t.data(), ev.p.data(), n);
    return ev;
}

inline int opt_int(int argc, char **argv, const char *name, int def) {
    for (int i = 1; i + 1 < argc; ++i)
        if (!std::strcmp(argv[i], name)) return std::atoi(argv[i + 1]);
    return def;
}

inline double opt_double(int argc, char **argv, const char *name, double def) {
    for (int i = 1; i + 1 < argc; ++i)
        if (!std::strcmp(argv[i], name)) return std::atof(argv[i + 1]);
    return def;
}

inline bool has_flag(int argc, char **argv, const char *name) {
    for (int i = 1; i < argc; ++i)
        if (!std::strcmp(argv[i], name)) return true;
    return false;
}
