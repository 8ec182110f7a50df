// Event ingest on the GPU: EVT 2.0 / EVT 3.0 RAW decoders and the n-µs reslicer (SURVEY.md
// §8f rank 1).
//
// Reference: the host programs decode through Metavision::Camera::from_file(argv[1])
// (FCT/…group_track.cpp:756-760) and slice with EventBufferReslicerAlgorithm
// (make_n_events :772-774, make_n_us DSA/…opencl_store.cpp:351) on one CPU decode thread.
// Metavision/OpenEB is not vendored; the word formats restated here are the published
// EVT 2.0 / EVT 3.0 specifications (include/ecc.h §8).
//
// MI355X design.  Both formats are state machines over a word stream (EVT 2.0: the last
// TIME_HIGH; EVT 3.0: the last y, TIME_LOW, TIME_HIGH + loop count, vector base x and
// polarity), and every state variable is a "last value set before this word" or a running
// sum — an associative summary.  So decoding is a three-phase scan, all HBM-streaming:
//   1. evt_summary_kernel: one workgroup per chunk folds its words into the chunk's
//      summary (64 B of consecutive words per lane, 16-B loads; wave-shuffle scan over the lanes);
//   2. evt_group_kernel + evt_carry_kernel: a two-level scan of the chunk summaries into
//      per-chunk carry-in states and int64 event offsets (advancing the caller's streaming
//      state);
//   3. evt_decode_kernel: each chunk re-reads its words, takes every lane's carry-in (EVT 3.0:
//      the chunk-local lane prefix the summary pass stored, 16 B per lane, combined with the
//      chunk's carry; EVT 2.0: the same wave-shuffle scan recomputed), walks its words per lane
//      into an LDS window of decoded events and writes the window out coalesced.
// Algorithmic bytes: words read twice (2 x 2 B or 2 x 4 B per word) + 13 B per event out
// (xy u32, t i64, p u8); EVT 3.0 adds the lane prefixes (16 B per 32 words, written + read).
#include "ecc_internal.hpp"

namespace {

constexpr int kThreads = 256;
// Each lane owns 64 B of words: 16 EVT 2.0 or 32 EVT 3.0 words (F::kPer); a workgroup owns a
// chunk of kThreads * F::kPer words.
constexpr int kFlagWord = 3;               // ctx->flags[3]: bit 1 capacity, bit 2 unsorted t

// ---- EVT 3.0 -------------------------------------------------------------------------------
// 16-bit words, type = w >> 12:
//   0x0 ADDR_Y      y = w & 0x7FF                       0x6 TIME_LOW   tl = w & 0xFFF
//   0x2 ADDR_X      event (x = w & 0x7FF, p = bit 11)   0x8 TIME_HIGH  th = w & 0xFFF
//   0x3 VECT_BASE_X base = w & 0x7FF, pol = bit 11      0x4 VECT_12    mask 12 bits, base += 12
//   0x5 VECT_8      mask 8 bits, base += 8              0x7, 0xA, 0xE, 0xF: no CD event
// t = loops << 24 | th << 12 | tl; loops counts TIME_HIGH decreases.
struct S3 {
    int32_t y, tl;               // -1: not set in the range
    int32_t th_first, th_last;   // -1: no TIME_HIGH in the range
    int32_t loops;               // TIME_HIGH decreases inside the range
    int32_t base;                // -1: no VECT_BASE_X; else x | pol << 16 of the last one
    int32_t inc;                 // x advance after the last base (or over the whole range)
    int32_t n;                   // CD events
};

struct Evt3 {
    using Word = uint16_t;
    using S = S3;
    static constexpr int kPer = 32;
    static constexpr int kOut = 2048;  // decode window (events): 26.6 KB of LDS, six workgroups per CU
    // The summary pass keeps every lane's chunk-local exclusive prefix (16 B per 64 B of words),
    // so the decode pass skips the fold and the block scan.  Within a chunk: n < 2^17,
    // loops < 2^15; the x advance only matters modulo 2^16 (x = (base + inc + b) & 0xFFFF).
    static constexpr bool kLanePrefix = true;
    __device__ static uint4 pack(const S &v) {
        uint4 w;
        w.x = ((uint32_t)v.y & 0x7FFu) | (v.y >= 0 ? 1u << 11 : 0u) | (((uint32_t)v.tl & 0xFFFu) << 12) |
              (v.tl >= 0 ? 1u << 24 : 0u);
        w.y = ((uint32_t)v.th_first & 0xFFFu) | (v.th_first >= 0 ? 1u << 12 : 0u) |
              (((uint32_t)v.th_last & 0xFFFu) << 13) | (v.th_last >= 0 ? 1u << 25 : 0u);
        w.z = (v.base >= 0 ? 1u : 0u) | (((uint32_t)v.base & 0x7FFu) << 1) | ((((uint32_t)v.base >> 16) & 1u) << 12) |
              ((uint32_t)v.inc << 16);
        w.w = ((uint32_t)v.n & 0x1FFFFu) | ((uint32_t)v.loops << 17);
        return w;
    }
    __device__ static S unpack(const uint4 w) {
        S v;
        v.y = (w.x >> 11 & 1u) ? (int32_t)(w.x & 0x7FFu) : -1;
        v.tl = (w.x >> 24 & 1u) ? (int32_t)(w.x >> 12 & 0xFFFu) : -1;
        v.th_first = (w.y >> 12 & 1u) ? (int32_t)(w.y & 0xFFFu) : -1;
        v.th_last = (w.y >> 25 & 1u) ? (int32_t)(w.y >> 13 & 0xFFFu) : -1;
        v.base = (w.z & 1u) ? (int32_t)((w.z >> 1 & 0x7FFu) | ((w.z >> 12 & 1u) << 16)) : -1;
        v.inc = (int32_t)(w.z >> 16);
        v.n = (int32_t)(w.w & 0x1FFFFu);
        v.loops = (int32_t)(w.w >> 17);
        return v;
    }
    __device__ static int prefix_n(const uint4 w) { return (int)(w.w & 0x1FFFFu); }
    __device__ static S identity() { return S{-1, -1, -1, -1, 0, -1, 0, 0}; }
    __device__ static S cat(const S &a, const S &b) {  // a, then b
        S r;
        r.y = b.y >= 0 ? b.y : a.y;
        r.tl = b.tl >= 0 ? b.tl : a.tl;
        r.th_first = a.th_first >= 0 ? a.th_first : b.th_first;
        r.th_last = b.th_last >= 0 ? b.th_last : a.th_last;
        r.loops = a.loops + b.loops + ((a.th_last >= 0 && b.th_first >= 0 && b.th_first < a.th_last) ? 1 : 0);
        r.base = b.base >= 0 ? b.base : a.base;
        r.inc = b.base >= 0 ? b.inc : a.inc + b.inc;
        r.n = a.n + b.n;
        return r;
    }
    // s = cat(s, word(w)), branch-free: lanes hold words of different types, so a switch would
    // run every case body per word.
    __device__ static void fold(S &s, uint32_t w) {
        const uint32_t ty = w >> 12;
        const int32_t v11 = (int32_t)(w & 0x7FFu), v12 = (int32_t)(w & 0xFFFu);
        s.y = ty == 0x0 ? v11 : s.y;
        s.tl = ty == 0x6 ? v12 : s.tl;
        const bool th_w = ty == 0x8;
        s.loops += (th_w && s.th_last >= 0 && v12 < s.th_last) ? 1 : 0;
        s.th_first = (th_w && s.th_first < 0) ? v12 : s.th_first;
        s.th_last = th_w ? v12 : s.th_last;
        const bool base_w = ty == 0x3;
        s.base = base_w ? (v11 | (int32_t)((w >> 11 & 1u) << 16)) : s.base;
        s.inc = base_w ? 0 : s.inc + (ty == 0x4 ? 12 : ty == 0x5 ? 8 : 0);
        const uint32_t vm = ty == 0x4 ? (w & 0xFFFu) : ty == 0x5 ? (w & 0xFFu) : 0u;
        s.n += (ty == 0x2 ? 1 : 0) + __popc(vm);
    }
    // Decoder registers rebuilt from a prefix summary (the state before the first word).
    struct Regs {
        uint32_t y, tl, th, pol, base;
        int32_t loops;
        bool has_th;
    };
    __device__ static Regs regs(const S &p) {
        Regs r;
        r.y = p.y >= 0 ? (uint32_t)p.y : 0u;
        r.tl = p.tl >= 0 ? (uint32_t)p.tl : 0u;
        r.th = p.th_last >= 0 ? (uint32_t)p.th_last : 0u;
        r.has_th = p.th_last >= 0;
        r.loops = p.loops;
        r.pol = p.base >= 0 ? ((uint32_t)p.base >> 16) : 0u;
        r.base = (p.base >= 0 ? ((uint32_t)p.base & 0xFFFFu) : 0u) + (uint32_t)p.inc;
        return r;
    }
    template <class Emit>
    __device__ static void step(Regs &r, uint32_t w, Emit &emit) {
        const uint32_t ty = w >> 12, v11 = w & 0x7FFu, v12 = w & 0xFFFu;
        const int64_t t = ((int64_t)r.loops << 24) | (int64_t)(r.th << 12 | r.tl);
        uint32_t vm = ty == 0x4 ? v12 : ty == 0x5 ? (w & 0xFFu) : 0u;
        if (ty == 0x2) emit(v11 | (r.y << 16), t, (uint8_t)(w >> 11 & 1u));
        while (vm) {
            const uint32_t b = __builtin_ctz(vm);
            vm &= vm - 1u;
            emit(((r.base + b) & 0xFFFFu) | (r.y << 16), t, (uint8_t)r.pol);
        }
        r.y = ty == 0x0 ? v11 : r.y;
        r.tl = ty == 0x6 ? v12 : r.tl;
        const bool th_w = ty == 0x8;
        r.loops += (th_w && r.has_th && v12 < r.th) ? 1 : 0;
        r.th = th_w ? v12 : r.th;
        r.has_th = r.has_th || th_w;
        const bool base_w = ty == 0x3;
        r.pol = base_w ? (w >> 11 & 1u) : r.pol;
        r.base = base_w ? v11 : r.base + (ty == 0x4 ? 12u : ty == 0x5 ? 8u : 0u);
    }
};

// ---- EVT 2.0 -------------------------------------------------------------------------------
// 32-bit words, type = w >> 28:
//   0x0 CD_OFF / 0x1 CD_ON: ts_lsb = w >> 22 & 0x3F, x = w >> 11 & 0x7FF, y = w & 0x7FF
//   0x8 TIME_HIGH: th = w & 0x0FFFFFFF;  t = th << 6 | ts_lsb
//   0xA EXT_TRIGGER, 0xE OTHERS, 0xF CONTINUED: no CD event
struct S2 {
    int32_t th;  // -1: no TIME_HIGH in the range
    int32_t n;
    int32_t pad[6];
};

struct Evt2 {
    using Word = uint32_t;
    using S = S2;
    static constexpr int kPer = 16;
    static constexpr int kOut = 1024;  // decode window (events): small LDS -> occupancy
    static constexpr bool kLanePrefix = false;  // the EVT 2.0 fold is a few operations: recompute it
    __device__ static uint4 pack(const S &) { return make_uint4(0u, 0u, 0u, 0u); }
    __device__ static S unpack(const uint4) { return identity(); }
    __device__ static int prefix_n(const uint4) { return 0; }
    __device__ static S identity() { return S{-1, 0, {0, 0, 0, 0, 0, 0}}; }
    __device__ static S cat(const S &a, const S &b) {
        S r = identity();
        r.th = b.th >= 0 ? b.th : a.th;
        r.n = a.n + b.n;
        return r;
    }
    __device__ static void fold(S &s, uint32_t w) {
        const uint32_t ty = w >> 28;
        if (ty <= 1u) s.n += 1;
        else if (ty == 0x8u) s.th = (int32_t)(w & 0x0FFFFFFFu);
    }
    struct Regs {
        uint32_t th;
    };
    __device__ static Regs regs(const S &p) { return Regs{p.th >= 0 ? (uint32_t)p.th : 0u}; }
    template <class Emit>
    __device__ static void step(Regs &r, uint32_t w, Emit &emit) {
        const uint32_t ty = w >> 28;
        if (ty <= 1u)
            emit((w >> 11 & 0x7FFu) | ((w & 0x7FFu) << 16), ((int64_t)r.th << 6) | (int64_t)(w >> 22 & 0x3Fu),
                 (uint8_t)ty);
        else if (ty == 0x8u)
            r.th = w & 0x0FFFFFFFu;
    }
};

static_assert(sizeof(S3) == 32 && sizeof(S2) == 32, "summary = 32 B");
static_assert(ECC_EVT_STATE_BYTES >= 32, "state holds one summary");

// The chunk's words: lane l owns words [l*kPer, (l+1)*kPer), loaded with 16-B loads.
template <class F>
__device__ inline void load_words(const typename F::Word *__restrict__ words, int64_t n_words, int64_t c,
                                  uint32_t (&w)[F::kPer], int &nw) {
    constexpr int kPer = F::kPer, kChunk = kThreads * kPer;
    using Word = typename F::Word;
    const int64_t first = c * kChunk + (int64_t)threadIdx.x * kPer;
    const int64_t left = n_words - first;
    nw = left <= 0 ? 0 : (left < kPer ? (int)left : kPer);
    constexpr int kVec = 16 / sizeof(Word);  // words per 16-B load
    if (nw == kPer && ((reinterpret_cast<uintptr_t>(words + first) & 15u) == 0)) {
#pragma unroll
        for (int v = 0; v < kPer / kVec; ++v) {
            const uint4 q = *reinterpret_cast<const uint4 *>(words + first + v * kVec);
            const uint32_t d[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int e = 0; e < kVec; ++e)
                w[v * kVec + e] = sizeof(Word) == 4 ? d[e] : (d[e / 2] >> (16 * (e & 1))) & 0xFFFFu;
        }
    } else {
#pragma unroll
        for (int e = 0; e < kPer; ++e) w[e] = e < nw ? (uint32_t)words[first + e] : 0u;
    }
}

// Summary shuffles: the 32-B summaries move between lanes as eight 32-bit fields.
template <class S>
__device__ inline S shfl_up_s(const S &v, int d) {
    static_assert(sizeof(S) == 32, "summary = 8 x int32");
    S r;
    const int *a = reinterpret_cast<const int *>(&v);
    int *b = reinterpret_cast<int *>(&r);
#pragma unroll
    for (int f = 0; f < 8; ++f) b[f] = __shfl_up(a[f], d);
    return r;
}

// Exclusive scan of per-lane summaries over a workgroup of NT lanes: wave64 inclusive scans
// with shuffles, then the wave totals through LDS.  Returns the lane's exclusive prefix and
// the workgroup total through *total.
template <class F, int NT>
__device__ typename F::S block_excl_scan(const typename F::S &mine, typename F::S *wtot, typename F::S *total) {
    using S = typename F::S;
    constexpr int kW = NT / 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    S inc = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const S o = shfl_up_s(inc, d);
        if (lane >= d) inc = F::cat(o, inc);
    }
    S ex = shfl_up_s(inc, 1);
    if (lane == 0) ex = F::identity();
    if (lane == 63) wtot[wave] = inc;
    __syncthreads();
    S pre = F::identity();
    for (int w = 0; w < wave; ++w) pre = F::cat(pre, wtot[w]);
    if (total) {
        S t = F::identity();
#pragma unroll
        for (int w = 0; w < kW; ++w) t = F::cat(t, wtot[w]);
        *total = t;
    }
    __syncthreads();
    return F::cat(pre, ex);
}

template <class F>
__global__ void __launch_bounds__(kThreads)
evt_summary_kernel(const typename F::Word *__restrict__ words, int64_t n_words, typename F::S *__restrict__ sums,
                   uint4 *__restrict__ lanepre) {
    using S = typename F::S;
    __shared__ S wtot[kThreads / 64];
    constexpr int kPer = F::kPer;
    uint32_t w[kPer];
    int nw;
    load_words<F>(words, n_words, blockIdx.x, w, nw);
    S s = F::identity();
#pragma unroll
    for (int e = 0; e < kPer; ++e)
        if (e < nw) F::fold(s, w[e]);
    S tot;
    const S ex = block_excl_scan<F, kThreads>(s, wtot, &tot);
    if constexpr (F::kLanePrefix) lanepre[(int64_t)blockIdx.x * kThreads + threadIdx.x] = F::pack(ex);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// Carry-in states and event offsets in two levels.  evt_group_kernel: one workgroup per group
// of kGroup chunks scans their summaries (group-local exclusive prefixes + the group total).
// evt_carry_kernel: one workgroup scans the group totals in rounds of kGroup (one round covers
// 2^18 chunks), starting from the caller's streaming state, and writes the int64
// event offset of every group, the total -> *n_out, and the advanced state.
constexpr int kGroup = 512;

template <class F>
__global__ void __launch_bounds__(kGroup)
evt_group_kernel(const typename F::S *__restrict__ sums, int64_t n_chunks, typename F::S *__restrict__ carry_local,
                 int32_t *__restrict__ off_local, typename F::S *__restrict__ gsum) {
    using S = typename F::S;
    __shared__ S wtot[kGroup / 64];
    const int64_t c = (int64_t)blockIdx.x * kGroup + threadIdx.x;
    const S v = c < n_chunks ? sums[c] : F::identity();
    S tot;
    const S ex = block_excl_scan<F, kGroup>(v, wtot, &tot);
    if (c < n_chunks) {
        carry_local[c] = ex;
        off_local[c] = ex.n;  // < 512 chunks * 8192 words * 12 events
    }
    if (threadIdx.x == 0) gsum[blockIdx.x] = tot;
}

template <class F>
__global__ void __launch_bounds__(kGroup)
evt_carry_kernel(const typename F::S *__restrict__ gsum, int64_t n_groups, typename F::S *__restrict__ gcarry,
                 int64_t *__restrict__ goff, typename F::S *state, int64_t *n_out, int64_t cap, int32_t *err) {
    using S = typename F::S;
    __shared__ S wtot[kGroup / 64];
    __shared__ int64_t wn[kGroup / 64];
    __shared__ S run_s;
    __shared__ int64_t run_n;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) {
        run_s = state ? *state : F::identity();
        run_n = 0;
    }
    __syncthreads();
    for (int64_t g0 = 0; g0 < n_groups; g0 += kGroup) {
        const int64_t g = g0 + tid;
        const S v = g < n_groups ? gsum[g] : F::identity();
        S tot;
        const S ex = block_excl_scan<F, kGroup>(v, wtot, &tot);
        int64_t x = v.n;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int64_t o = __shfl_up(x, d);
            if (lane >= d) x += o;
        }
        if (lane == 63) wn[wave] = x;
        __syncthreads();
        int64_t pre = 0, all = 0;
        for (int w = 0; w < kGroup / 64; ++w) {
            if (w < wave) pre += wn[w];
            all += wn[w];
        }
        if (g < n_groups) {
            gcarry[g] = F::cat(run_s, ex);
            goff[g] = run_n + pre + x - v.n;
        }
        __syncthreads();
        if (tid == 0) {
            run_s = F::cat(run_s, tot);
            run_n += all;
        }
        __syncthreads();
    }
    if (tid == 0) {
        if (n_out) *n_out = run_n;
        if (run_n > cap) atomicOr(err, 2);
        if (state) {
            S ns = run_s;
            ns.n = 0;
            *state = ns;
        }
    }
}

// Decoded events are staged in LDS windows of F::kOut events and written out coalesced (a
// lane's own run of events would touch a different cache line per lane and store).  Lanes
// whose events miss the current window skip the walk.

template <class F>
__global__ void __launch_bounds__(kThreads)
evt_decode_kernel(const typename F::Word *__restrict__ words, int64_t n_words, const typename F::S *__restrict__ sums,
                  const typename F::S *__restrict__ carry_local, const int32_t *__restrict__ off_local,
                  const typename F::S *__restrict__ gcarry, const int64_t *__restrict__ goff,
                  const uint4 *__restrict__ lanepre, uint32_t *__restrict__ xy, int64_t *__restrict__ t,
                  uint8_t *__restrict__ p, int64_t cap) {
    using S = typename F::S;
    constexpr int kOut = F::kOut;
    __shared__ S wtot[kThreads / 64];
    __shared__ int64_t o_t[kOut];
    __shared__ uint32_t o_xy[kOut];
    __shared__ uint8_t o_p[kOut];
    constexpr int kPer = F::kPer;
    uint32_t w[kPer];
    int nw;
    load_words<F>(words, n_words, blockIdx.x, w, nw);
    const int g = blockIdx.x / kGroup;
    const int64_t n_chunk = sums[blockIdx.x].n;
    S exl;        // the lane's exclusive prefix within the chunk
    int lane_n;   // this lane's events
    if constexpr (F::kLanePrefix) {
        const int64_t li = (int64_t)blockIdx.x * kThreads + threadIdx.x;
        exl = F::unpack(lanepre[li]);
        lane_n = (threadIdx.x + 1 < kThreads ? F::prefix_n(lanepre[li + 1]) : (int)n_chunk) - exl.n;
    } else {
        S s = F::identity();
#pragma unroll
        for (int e = 0; e < kPer; ++e)
            if (e < nw) F::fold(s, w[e]);
        exl = block_excl_scan<F, kThreads>(s, wtot, nullptr);
        lane_n = s.n;
    }
    const S cin = F::cat(gcarry[g], carry_local[blockIdx.x]);
    const S ex = F::cat(cin, exl);
    const int64_t base = goff[g] + off_local[blockIdx.x];
    const int lane_first = exl.n;  // this lane's first event within the chunk
    for (int64_t w0 = 0; w0 < n_chunk; w0 += kOut) {
        if (lane_first < w0 + kOut && lane_first + lane_n > w0) {
            typename F::Regs r = F::regs(ex);
            int64_t pos = lane_first - w0;
            auto emit = [&](uint32_t v, int64_t ts, uint8_t pol) {
                if (pos >= 0 && pos < kOut) {
                    o_xy[pos] = v;
                    o_t[pos] = ts;
                    o_p[pos] = pol;
                }
                ++pos;
            };
            for (int e = 0; e < nw; ++e) F::step(r, w[e], emit);
        }
        __syncthreads();
        const int m = (int)(n_chunk - w0 < kOut ? n_chunk - w0 : kOut);
        for (int i = threadIdx.x; i < m; i += kThreads) {
            const int64_t g = base + w0 + i;
            if (g < cap) {
                if (xy) xy[g] = o_xy[i];
                if (t) t[g] = o_t[i];
                if (p) p[g] = o_p[i];
            }
        }
        __syncthreads();
    }
}

template <class F>
int decode(ecc_ctx *ctx, const void *words_v, int64_t n_words, uint32_t *xy, int64_t *t, uint8_t *p, int64_t cap,
           int64_t *n_out, void *state, hipStream_t s) {
    using S = typename F::S;
    const auto *words = static_cast<const typename F::Word *>(words_v);
    constexpr int kChunk = kThreads * F::kPer;
    const int64_t n_chunks = (n_words + kChunk - 1) / kChunk;
    if (n_chunks > INT32_MAX) return ECC_ERR_INVALID;
    const int64_t n_groups = (n_chunks + kGroup - 1) / kGroup;
    // workspace: sums | carry_local | off_local | gsum | gcarry | goff | lane prefixes
    size_t o = 0;
    auto carve = [&](size_t bytes) { const size_t at = o; o = ecc::align_up(o + bytes, 256); return at; };
    const size_t o_sums = carve((size_t)n_chunks * sizeof(S)), o_cl = carve((size_t)n_chunks * sizeof(S));
    const size_t o_ol = carve((size_t)n_chunks * 4), o_gs = carve((size_t)n_groups * sizeof(S));
    const size_t o_gc = carve((size_t)n_groups * sizeof(S)), o_go = carve((size_t)n_groups * 8);
    const size_t o_lp = carve(F::kLanePrefix ? (size_t)n_chunks * kThreads * sizeof(uint4) : 16);
    int rc = ecc::ws_reserve(ctx, o);
    if (rc) return rc;
    char *ws = static_cast<char *>(ctx->ws);
    S *sums = reinterpret_cast<S *>(ws + o_sums), *carry_local = reinterpret_cast<S *>(ws + o_cl);
    int32_t *off_local = reinterpret_cast<int32_t *>(ws + o_ol);
    S *gsum = reinterpret_cast<S *>(ws + o_gs), *gcarry = reinterpret_cast<S *>(ws + o_gc);
    int64_t *goff = reinterpret_cast<int64_t *>(ws + o_go);
    uint4 *lanepre = reinterpret_cast<uint4 *>(ws + o_lp);
    int32_t *err = ctx->flags + kFlagWord;
    ECC_CHECK_HIP(ctx, hipMemsetAsync(err, 0, 4, s), "memset(evt err)");
    if (n_chunks == 0) {
        if (n_out) ECC_CHECK_HIP(ctx, hipMemsetAsync(n_out, 0, 8, s), "memset(n_out)");
        return ECC_OK;
    }
    {
        ECC_TIMED(ctx, s, "evt_summary_kernel");
        hipLaunchKernelGGL(evt_summary_kernel<F>, dim3((unsigned)n_chunks), dim3(kThreads), 0, s, words, n_words, sums, lanepre);
    }
    {
        ECC_TIMED(ctx, s, "evt_group_kernel");
        hipLaunchKernelGGL(evt_group_kernel<F>, dim3((unsigned)n_groups), dim3(kGroup), 0, s, sums, n_chunks,
                           carry_local, off_local, gsum);
    }
    {
        ECC_TIMED(ctx, s, "evt_carry_kernel");
        hipLaunchKernelGGL(evt_carry_kernel<F>, dim3(1), dim3(kGroup), 0, s, gsum, n_groups, gcarry, goff,
                           static_cast<S *>(state), n_out, cap, err);
    }
    {
        ECC_TIMED(ctx, s, "evt_decode_kernel");
        hipLaunchKernelGGL(evt_decode_kernel<F>, dim3((unsigned)n_chunks), dim3(kThreads), 0, s, words, n_words, sums,
                           carry_local, off_local, gcarry, goff, (const uint4 *)lanepre, xy, t, p, cap);
    }
    ECC_CHECK_LAUNCH(ctx, "evt decode");
    return ECC_OK;
}

// ---- n-µs reslicer -------------------------------------------------------------------------
// Event i opens slices (k_{i-1}, k_i] (k = (t - t_base) / period); each writes bounds[k] = i.
// Reads t[i-1], t[i] (8 B/event, the neighbour from cache); writes one int64 per slice.
__global__ void __launch_bounds__(kThreads)
reslice_n_us_kernel(const int64_t *__restrict__ t, int64_t n, int64_t period, int64_t *__restrict__ bounds,
                    int64_t max_slices, int64_t *n_slices, int32_t *err) {
    const int64_t t0 = t[0];
    const int64_t base = (t0 >= 0 ? t0 / period : -((-t0 + period - 1) / period)) * period;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
        const int64_t ti = t[i];
        const int64_t k = (ti - base) / period;
        int64_t kp = -1;
        if (i > 0) {
            const int64_t tp = t[i - 1];
            if (tp > ti) atomicOr(err, 4);
            kp = (tp - base) / period;
        }
        for (int64_t q = kp + 1; q <= k && q < max_slices; ++q) bounds[q] = i;
        if (i == n - 1) {
            const int64_t ns = k + 1;
            if (n_slices) *n_slices = ns;
            if (ns > max_slices) atomicOr(err, 2);
            bounds[ns < max_slices ? ns : max_slices] = n;
        }
    }
}

}  // namespace

ECC_API int ecc_evt_decode(ecc_ctx *ctx, int32_t format, const void *words, int64_t n_words, uint32_t *xy,
                           int64_t *t, uint8_t *p, int64_t cap, int64_t *n_out, void *state,
                           ecc_stream_t stream) {
    if (!ctx || n_words < 0 || cap < 0 || (n_words > 0 && !words)) return ECC_ERR_INVALID;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    if (format == ECC_RAW_EVT3) return decode<Evt3>(ctx, words, n_words, xy, t, p, cap, n_out, state, s);
    if (format == ECC_RAW_EVT2) return decode<Evt2>(ctx, words, n_words, xy, t, p, cap, n_out, state, s);
    return ECC_ERR_INVALID;
}

ECC_API int ecc_evt_status(ecc_ctx *ctx, ecc_stream_t stream) {
    if (!ctx) return ECC_ERR_INVALID;
    int32_t f = 0;
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(&f, ctx->flags + kFlagWord, 4, hipMemcpyDeviceToHost, ecc::as_stream(stream)),
                  "read evt err");
    ECC_CHECK_HIP(ctx, hipStreamSynchronize(ecc::as_stream(stream)), "sync");
    if (f & 4) return ECC_ERR_UNSORTED_TIME;
    if (f & 2) return ECC_ERR_CAPACITY;
    return ECC_OK;
}

ECC_API int ecc_reslice_n_us(ecc_ctx *ctx, const int64_t *t, int64_t n, int64_t period_us, int64_t *bounds,
                             int64_t max_slices, int64_t *n_slices, ecc_stream_t stream) {
    if (!ctx || n < 0 || period_us <= 0 || max_slices < 0 || !bounds || (n > 0 && !t)) return ECC_ERR_INVALID;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t s = ecc::as_stream(stream);
    int32_t *err = ctx->flags + kFlagWord;
    ECC_CHECK_HIP(ctx, hipMemsetAsync(err, 0, 4, s), "memset(evt err)");
    if (n == 0) {
        ECC_CHECK_HIP(ctx, hipMemsetAsync(bounds, 0, 8, s), "bounds[0]");
        if (n_slices) ECC_CHECK_HIP(ctx, hipMemsetAsync(n_slices, 0, 8, s), "n_slices");
        return ECC_OK;
    }
    const int64_t blocks = std::min<int64_t>((n + kThreads - 1) / kThreads, 8192);
    ECC_TIMED(ctx, s, "reslice_n_us_kernel");
    hipLaunchKernelGGL(reslice_n_us_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s, t, n, period_us, bounds,
                       max_slices, n_slices, err);
    ECC_CHECK_LAUNCH(ctx, "reslice");
    return ECC_OK;
}
