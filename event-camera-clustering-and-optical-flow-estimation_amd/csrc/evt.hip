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
//   1. evt_summary_kernel: one workgroup per 4096-word chunk folds its words into the chunk's
//      summary (16 consecutive words per lane, 16-B loads; LDS scan over the lanes);
//   2. evt_carry_kernel: one workgroup scans the chunk summaries into per-chunk carry-in
//      states and int64 event offsets (and advances the caller's streaming state);
//   3. evt_decode_kernel: each chunk re-reads its words, rebuilds the per-lane carry-in with
//      the same LDS scan, and walks its 16 words emitting events at their final positions.
// Algorithmic bytes: words read twice (2 x 2 B or 2 x 4 B per word) + 13 B per event out
// (xy u32, t i64, p u8).
#include "ecc_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr int kPer = 16;                   // words per lane
constexpr int kChunk = kThreads * kPer;    // words per workgroup
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
    __device__ static void fold(S &s, uint32_t w) {  // s = cat(s, word(w)), specialised
        switch (w >> 12) {
            case 0x0: s.y = (int32_t)(w & 0x7FFu); break;
            case 0x2: s.n += 1; break;
            case 0x3: s.base = (int32_t)((w & 0x7FFu) | ((w >> 11 & 1u) << 16)); s.inc = 0; break;
            case 0x4: s.n += __popc(w & 0xFFFu); s.inc += 12; break;
            case 0x5: s.n += __popc(w & 0xFFu); s.inc += 8; break;
            case 0x6: s.tl = (int32_t)(w & 0xFFFu); break;
            case 0x8: {
                const int32_t th = (int32_t)(w & 0xFFFu);
                if (s.th_last >= 0 && th < s.th_last) s.loops += 1;
                if (s.th_first < 0) s.th_first = th;
                s.th_last = th;
                break;
            }
            default: break;
        }
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
        const int64_t t = ((int64_t)r.loops << 24) | (int64_t)(r.th << 12 | r.tl);
        switch (w >> 12) {
            case 0x0: r.y = w & 0x7FFu; break;
            case 0x2: emit((w & 0x7FFu) | (r.y << 16), t, (uint8_t)(w >> 11 & 1u)); break;
            case 0x3: r.base = w & 0x7FFu; r.pol = w >> 11 & 1u; break;
            case 0x4:
            case 0x5: {
                const int nb = (w >> 12) == 0x4 ? 12 : 8;
                uint32_t m = w & ((1u << nb) - 1u);
                while (m) {
                    const uint32_t b = __builtin_ctz(m);
                    m &= m - 1u;
                    emit(((r.base + b) & 0xFFFFu) | (r.y << 16), t, (uint8_t)r.pol);
                }
                r.base += (uint32_t)nb;
                break;
            }
            case 0x6: r.tl = w & 0xFFFu; break;
            case 0x8: {
                const uint32_t th = w & 0xFFFu;
                if (r.has_th && th < r.th) r.loops += 1;
                r.th = th;
                r.has_th = true;
                break;
            }
            default: break;
        }
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
                                  uint32_t (&w)[kPer], int &nw) {
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

// Exclusive scan of per-lane summaries over the workgroup (Hillis-Steele in LDS); returns
// the lane's exclusive prefix, and the inclusive total through *total.
template <class F>
__device__ typename F::S block_excl_scan(const typename F::S &mine, typename F::S *sh, typename F::S *total) {
    using S = typename F::S;
    const int tid = threadIdx.x;
    sh[tid] = mine;
    __syncthreads();
    for (int d = 1; d < kThreads; d <<= 1) {
        S v = sh[tid];
        if (tid >= d) v = F::cat(sh[tid - d], v);
        __syncthreads();
        sh[tid] = v;
        __syncthreads();
    }
    if (total) *total = sh[kThreads - 1];
    const S ex = tid ? sh[tid - 1] : F::identity();
    __syncthreads();
    return ex;
}

template <class F>
__global__ void __launch_bounds__(kThreads)
evt_summary_kernel(const typename F::Word *__restrict__ words, int64_t n_words, typename F::S *__restrict__ sums) {
    using S = typename F::S;
    __shared__ S sh[kThreads];
    uint32_t w[kPer];
    int nw;
    load_words<F>(words, n_words, blockIdx.x, w, nw);
    S s = F::identity();
#pragma unroll
    for (int e = 0; e < kPer; ++e)
        if (e < nw) F::fold(s, w[e]);
    S tot;
    block_excl_scan<F>(s, sh, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// One workgroup: carry[c] = state before chunk c (the caller's streaming state first),
// off[c] = events before chunk c (int64), off[n_chunks] = total -> *n_out; state advanced.
template <class F>
__global__ void __launch_bounds__(kThreads)
evt_carry_kernel(const typename F::S *__restrict__ sums, int64_t n_chunks, typename F::S *__restrict__ carry,
                 int64_t *__restrict__ off, typename F::S *state, int64_t *n_out, int64_t cap, int32_t *err) {
    using S = typename F::S;
    __shared__ S sh[kThreads];
    __shared__ int64_t sn[kThreads];
    const int tid = threadIdx.x;
    const int64_t per = (n_chunks + kThreads - 1) / kThreads;
    const int64_t lo = tid * per, hi = lo + per < n_chunks ? lo + per : n_chunks;
    S s = F::identity();
    int64_t n = 0;
    for (int64_t c = lo; c < hi; ++c) {
        const S v = sums[c];
        s = F::cat(s, v);
        n += v.n;
    }
    S tot;
    S ex = block_excl_scan<F>(s, sh, &tot);
    // int64 event counts: separate scan (summary n fields are per-chunk int32)
    sn[tid] = n;
    __syncthreads();
    for (int d = 1; d < kThreads; d <<= 1) {
        const int64_t v = tid >= d ? sn[tid - d] + sn[tid] : sn[tid];
        __syncthreads();
        sn[tid] = v;
        __syncthreads();
    }
    int64_t nex = tid ? sn[tid - 1] : 0;
    const S st0 = state ? *state : F::identity();
    __syncthreads();
    ex = F::cat(st0, ex);
    for (int64_t c = lo; c < hi; ++c) {
        carry[c] = ex;
        off[c] = nex;
        const S v = sums[c];
        ex = F::cat(ex, v);
        nex += v.n;
    }
    if (tid == kThreads - 1) {
        const int64_t total = sn[kThreads - 1];
        off[n_chunks] = total;
        if (n_out) *n_out = total;
        if (total > cap) atomicOr(err, 2);
        if (state) {
            S ns = F::cat(st0, tot);
            ns.n = 0;
            *state = ns;
        }
    }
}

template <class F>
__global__ void __launch_bounds__(kThreads)
evt_decode_kernel(const typename F::Word *__restrict__ words, int64_t n_words, const typename F::S *__restrict__ carry,
                  const int64_t *__restrict__ off, uint32_t *__restrict__ xy, int64_t *__restrict__ t,
                  uint8_t *__restrict__ p, int64_t cap) {
    using S = typename F::S;
    __shared__ S sh[kThreads];
    uint32_t w[kPer];
    int nw;
    load_words<F>(words, n_words, blockIdx.x, w, nw);
    S s = F::identity();
#pragma unroll
    for (int e = 0; e < kPer; ++e)
        if (e < nw) F::fold(s, w[e]);
    const S ex = F::cat(carry[blockIdx.x], block_excl_scan<F>(s, sh, nullptr));
    int64_t pos = off[blockIdx.x] + (ex.n - carry[blockIdx.x].n);
    typename F::Regs r = F::regs(ex);
    auto emit = [&](uint32_t v, int64_t ts, uint8_t pol) {
        if (pos < cap) {
            if (xy) xy[pos] = v;
            if (t) t[pos] = ts;
            if (p) p[pos] = pol;
        }
        ++pos;
    };
    for (int e = 0; e < nw; ++e) F::step(r, w[e], emit);
}

template <class F>
int decode(ecc_ctx *ctx, const void *words_v, int64_t n_words, uint32_t *xy, int64_t *t, uint8_t *p, int64_t cap,
           int64_t *n_out, void *state, hipStream_t s) {
    using S = typename F::S;
    const auto *words = static_cast<const typename F::Word *>(words_v);
    const int64_t n_chunks = (n_words + kChunk - 1) / kChunk;
    if (n_chunks > INT32_MAX) return ECC_ERR_INVALID;
    const size_t off_carry = ecc::align_up((size_t)n_chunks * sizeof(S), 256);
    const size_t off_off = off_carry + ecc::align_up((size_t)n_chunks * sizeof(S), 256);
    int rc = ecc::ws_reserve(ctx, off_off + (size_t)(n_chunks + 1) * 8);
    if (rc) return rc;
    char *ws = static_cast<char *>(ctx->ws);
    S *sums = reinterpret_cast<S *>(ws);
    S *carry = reinterpret_cast<S *>(ws + off_carry);
    int64_t *off = reinterpret_cast<int64_t *>(ws + off_off);
    int32_t *err = ctx->flags + kFlagWord;
    ECC_CHECK_HIP(ctx, hipMemsetAsync(err, 0, 4, s), "memset(evt err)");
    if (n_chunks == 0) {
        if (n_out) ECC_CHECK_HIP(ctx, hipMemsetAsync(n_out, 0, 8, s), "memset(n_out)");
        return ECC_OK;
    }
    {
        ECC_TIMED(ctx, s, "evt_summary_kernel");
        hipLaunchKernelGGL(evt_summary_kernel<F>, dim3((unsigned)n_chunks), dim3(kThreads), 0, s, words, n_words, sums);
    }
    {
        ECC_TIMED(ctx, s, "evt_carry_kernel");
        hipLaunchKernelGGL(evt_carry_kernel<F>, dim3(1), dim3(kThreads), 0, s, sums, n_chunks, carry, off,
                           static_cast<S *>(state), n_out, cap, err);
    }
    {
        ECC_TIMED(ctx, s, "evt_decode_kernel");
        hipLaunchKernelGGL(evt_decode_kernel<F>, dim3((unsigned)n_chunks), dim3(kThreads), 0, s, words, n_words, carry,
                           off, xy, t, p, cap);
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
