// Native multi-GPU exchanges of the time-window-sharded pipeline over RCCL (SURVEY.md §8e,
// BASELINE config C5).  One process per GPU; rank r owns the stream's r-th time
// window.  The three data-path exchanges of a step:
//   * k-means:  ONE in-place SUM all-reduce of the shards' per-pixel count images (int32[H*W]);
//               every rank then runs the Lloyd passes over the global image (ecc_kmeans_run_counts)
//   * SAE:      an all-gather of the shards' own last-timestamp images (int64[H*W], written by
//               ecc_fast_detect_prepare) and, fused, rank r's initial SAE = the element-wise max
//               over ranks < r (ecc_sae_max_combine; time is non-decreasing across shards)
//   * tracks:   the shards' packed per-slice NMS lists (ecc_corner_pack) gathered in rank order =
//               global slice order, with each slice's (start, count) for ONE
//               ecc_tracker_update_lists (the reference's slice loop, FCT/…group_track.cpp:832-850)
// The reference has no multi-device code; these restate its sequential slice loop exactly.
//
// librccl is opened on first use (dlopen, RTLD_LOCAL) rather than linked: libecc keeps no
// link-time dependence on it, and its symbols never interpose the RCCL copy a host process (e.g.
// PyTorch) may already have loaded.  Collectives are enqueued on the caller's stream, so they
// order against libecc's kernels like any other launch (no host synchronisation, except the
// corner gather's one size exchange).
#include <dlfcn.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>

#include <rccl/rccl.h>

#include "ecc_internal.hpp"

namespace {

struct RcclApi {
    bool ok = false;
    std::string err;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
};

RcclApi &rccl() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        const char *env = std::getenv("ECC_RCCL_LIB");
        const char *names[] = {env, "librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        void *h = nullptr;
        for (const char *n : names)
            if (n && (h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) {
            const char *e = dlerror();
            api.err = std::string("dlopen(librccl): ") + (e ? e : "not found");
            return;
        }
        auto sym = [&](const char *name) { return dlsym(h, name); };
        api.get_unique_id = reinterpret_cast<decltype(api.get_unique_id)>(sym("ncclGetUniqueId"));
        api.comm_init_rank = reinterpret_cast<decltype(api.comm_init_rank)>(sym("ncclCommInitRank"));
        api.comm_destroy = reinterpret_cast<decltype(api.comm_destroy)>(sym("ncclCommDestroy"));
        api.all_reduce = reinterpret_cast<decltype(api.all_reduce)>(sym("ncclAllReduce"));
        api.all_gather = reinterpret_cast<decltype(api.all_gather)>(sym("ncclAllGather"));
        api.error_string = reinterpret_cast<decltype(api.error_string)>(sym("ncclGetErrorString"));
        api.ok = api.get_unique_id && api.comm_init_rank && api.comm_destroy && api.all_reduce && api.all_gather &&
                 api.error_string;
        if (!api.ok) api.err = "librccl lacks an nccl* entry point";
    });
    return api;
}

// (start, count) per slice of the gathered lists: rank r's slices follow ranks < r.
// offs: [n_ranks][ns_max + 1] gathered offsets (exclusive scans of the shards' counts).
__global__ void corner_slices_kernel(const int64_t *__restrict__ offs, const int64_t *__restrict__ meta,
                                     int32_t n_ranks, int64_t ns_max, int64_t t_max, int64_t *__restrict__ starts,
                                     int32_t *__restrict__ counts) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // i = r * ns_max + s
    if (i >= (int64_t)n_ranks * ns_max) return;
    const int32_t r = (int32_t)(i / ns_max);
    const int64_t s = i - (int64_t)r * ns_max;
    const int64_t ns_r = meta[2 * r + 1];
    if (s >= ns_r) return;
    int64_t base = 0;  // slices of the lower ranks (n_ranks is small: a short serial sum)
    for (int32_t q = 0; q < r; ++q) base += meta[2 * q + 1];
    const int64_t *o = offs + (int64_t)r * (ns_max + 1);
    starts[base + s] = (int64_t)r * t_max + o[s];
    counts[base + s] = (int32_t)(o[s + 1] - o[s]);
}

__global__ void corner_meta_kernel(const int64_t *__restrict__ offsets, int32_t n_slices, int64_t *__restrict__ meta) {
    if (threadIdx.x == 0) {
        meta[0] = n_slices > 0 ? offsets[n_slices] : 0;
        meta[1] = n_slices;
    }
}

}  // namespace

struct ecc_dist {
    ecc_ctx *ctx = nullptr;
    ncclComm_t comm = nullptr;
    int32_t n_ranks = 0, rank = 0;
    // corner-gather scratch (device): meta [2], gathered metas [2 n_ranks], padded send lists and
    // offsets, gathered offsets; grown on demand
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
};

static int dist_fail(ecc_dist *d, ncclResult_t r, const char *what) {
    if (d && d->ctx) d->ctx->last_error = std::string(what) + ": " + rccl().error_string(r);
    return ECC_ERR_HIP;
}

#define ECC_CHECK_RCCL(d, call, what)                     \
    do {                                                  \
        ncclResult_t _r = (call);                         \
        if (_r != ncclSuccess) return dist_fail(d, _r, what); \
    } while (0)

ECC_API int ecc_dist_available(void) { return rccl().ok ? 1 : 0; }

ECC_API int ecc_dist_get_unique_id(uint8_t *id) {
    if (!id) return ECC_ERR_INVALID;
    if (!rccl().ok) return ECC_ERR_NO_DEVICE;
    ncclUniqueId u;
    if (rccl().get_unique_id(&u) != ncclSuccess) return ECC_ERR_HIP;
    static_assert(sizeof(u) == ECC_DIST_ID_BYTES, "ncclUniqueId size");
    std::memcpy(id, &u, sizeof(u));
    return ECC_OK;
}

ECC_API int ecc_dist_init(ecc_dist **out, ecc_ctx *ctx, const uint8_t *id, int32_t n_ranks, int32_t rank) {
    if (!out || !ctx || !id || n_ranks < 1 || rank < 0 || rank >= n_ranks) return ECC_ERR_INVALID;
    *out = nullptr;
    if (!rccl().ok) {
        ctx->last_error = rccl().err;
        return ECC_ERR_NO_DEVICE;
    }
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    auto *d = new ecc_dist();
    d->ctx = ctx;
    d->n_ranks = n_ranks;
    d->rank = rank;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    const ncclResult_t r = rccl().comm_init_rank(&d->comm, n_ranks, u, rank);
    if (r != ncclSuccess) {
        dist_fail(d, r, "ncclCommInitRank");
        delete d;
        return ECC_ERR_HIP;
    }
    *out = d;
    return ECC_OK;
}

ECC_API int ecc_dist_destroy(ecc_dist *d) {
    if (!d) return ECC_OK;
    if (d->comm) rccl().comm_destroy(d->comm);
    if (d->scratch) {
        hipSetDevice(d->ctx->device);
        hipFree(d->scratch);
    }
    delete d;
    return ECC_OK;
}

ECC_API int ecc_dist_rank(const ecc_dist *d, int32_t *rank, int32_t *n_ranks) {
    if (!d) return ECC_ERR_INVALID;
    if (rank) *rank = d->rank;
    if (n_ranks) *n_ranks = d->n_ranks;
    return ECC_OK;
}

ECC_API int ecc_dist_allreduce_counts(ecc_dist *d, uint32_t *counts, int64_t n, ecc_stream_t stream) {
    if (!d || n < 0 || (n > 0 && !counts)) return ECC_ERR_INVALID;
    if (n == 0) return ECC_OK;
    ECC_CHECK_HIP(d->ctx, hipSetDevice(d->ctx->device), "hipSetDevice");
    ECC_CHECK_RCCL(d, rccl().all_reduce(counts, counts, (size_t)n, ncclUint32, ncclSum, d->comm, ecc::as_stream(stream)),
                   "ncclAllReduce(counts)");
    return ECC_OK;
}

ECC_API int ecc_dist_allreduce_f64_max(ecc_dist *d, double *values, int64_t n, ecc_stream_t stream) {
    if (!d || n < 0 || (n > 0 && !values)) return ECC_ERR_INVALID;
    if (n == 0) return ECC_OK;
    ECC_CHECK_HIP(d->ctx, hipSetDevice(d->ctx->device), "hipSetDevice");
    ECC_CHECK_RCCL(d, rccl().all_reduce(values, values, (size_t)n, ncclFloat64, ncclMax, d->comm, ecc::as_stream(stream)),
                   "ncclAllReduce(max)");
    return ECC_OK;
}

ECC_API int ecc_dist_sae_handoff(ecc_dist *d, const int64_t *local_last, int64_t hw, int64_t *all, int64_t *sae,
                                 ecc_stream_t stream) {
    if (!d || hw < 0 || (hw > 0 && (!local_last || !all || !sae))) return ECC_ERR_INVALID;
    if (hw == 0) return ECC_OK;
    ECC_CHECK_HIP(d->ctx, hipSetDevice(d->ctx->device), "hipSetDevice");
    ECC_CHECK_RCCL(d, rccl().all_gather(local_last, all, (size_t)hw, ncclInt64, d->comm, ecc::as_stream(stream)),
                   "ncclAllGather(sae)");
    // rank r starts from the max over ranks < r (zeros for rank 0)
    return ecc_sae_max_combine(d->ctx, all, d->rank, hw, sae, stream);
}

ECC_API int ecc_dist_gather_corners(ecc_dist *d, const ecc_corner *packed, const int64_t *offsets, int32_t n_slices,
                                    ecc_corner *all, int64_t all_cap, int64_t *starts, int32_t *counts,
                                    int64_t slices_cap, int64_t *n_slices_total, int64_t *corners_stride,
                                    ecc_stream_t stream) {
    if (!d || n_slices < 0 || !n_slices_total || (n_slices > 0 && (!packed || !offsets))) return ECC_ERR_INVALID;
    ecc_ctx *ctx = d->ctx;
    hipStream_t s = ecc::as_stream(stream);
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    const int R = d->n_ranks;
    // 1. sizes: {corners, slices} of every rank (the one host synchronisation of the exchange)
    const size_t meta_b = ecc::align_up(2 * 8, 256), metas_b = ecc::align_up((size_t)R * 16, 256);
    if (!d->scratch || d->scratch_bytes < meta_b + metas_b) {
        if (d->scratch) hipFree(d->scratch);
        d->scratch = nullptr;
        d->scratch_bytes = 0;
        ECC_CHECK_HIP(ctx, hipMalloc(&d->scratch, meta_b + metas_b), "hipMalloc(dist scratch)");
        d->scratch_bytes = meta_b + metas_b;
    }
    int64_t *meta = static_cast<int64_t *>(d->scratch);
    int64_t *metas = reinterpret_cast<int64_t *>(static_cast<char *>(d->scratch) + meta_b);
    if (n_slices > 0) {
        hipLaunchKernelGGL(corner_meta_kernel, dim3(1), dim3(64), 0, s, offsets, n_slices, meta);
    } else {
        ECC_CHECK_HIP(ctx, hipMemsetAsync(meta, 0, 16, s), "memset(meta)");
    }
    ECC_CHECK_LAUNCH(ctx, "corner_meta");
    ECC_CHECK_RCCL(d, rccl().all_gather(meta, metas, 2, ncclInt64, d->comm, s), "ncclAllGather(meta)");
    std::vector<int64_t> h((size_t)R * 2);
    ECC_CHECK_HIP(ctx, hipMemcpyAsync(h.data(), metas, h.size() * 8, hipMemcpyDeviceToHost, s), "d2h(meta)");
    ECC_CHECK_HIP(ctx, hipStreamSynchronize(s), "sync(meta)");
    int64_t t_max = 1, ns_max = 1, ns_tot = 0;
    for (int r = 0; r < R; ++r) {
        t_max = std::max(t_max, h[2 * r]);
        ns_max = std::max(ns_max, h[2 * r + 1]);
        ns_tot += h[2 * r + 1];
    }
    *n_slices_total = ns_tot;
    if (corners_stride) *corners_stride = t_max;
    if (!all && !starts && !counts) return ECC_OK;  // a size query (itself a collective call)
    if (!all || !starts || !counts) return ECC_ERR_INVALID;
    if ((int64_t)R * t_max > all_cap || ns_tot > slices_cap) return ECC_ERR_CAPACITY;
    // 2. lists padded to the largest rank's, offsets padded to the most slices; one all-gather each
    const size_t pk_b = ecc::align_up((size_t)t_max * sizeof(ecc_corner), 256);
    const size_t off_b = ecc::align_up((size_t)(ns_max + 1) * 8, 256);
    const size_t offs_b = ecc::align_up((size_t)R * (ns_max + 1) * 8, 256);
    const size_t need = meta_b + metas_b + pk_b + off_b + offs_b;
    if (d->scratch_bytes < need) {
        ECC_CHECK_HIP(ctx, hipStreamSynchronize(s), "sync(grow)");
        hipFree(d->scratch);
        d->scratch = nullptr;
        d->scratch_bytes = 0;
        ECC_CHECK_HIP(ctx, hipMalloc(&d->scratch, need), "hipMalloc(dist scratch)");
        d->scratch_bytes = need;
        meta = static_cast<int64_t *>(d->scratch);
        metas = reinterpret_cast<int64_t *>(static_cast<char *>(d->scratch) + meta_b);
        ECC_CHECK_HIP(ctx, hipMemcpyAsync(metas, h.data(), h.size() * 8, hipMemcpyHostToDevice, s), "h2d(meta)");
    }
    char *base = static_cast<char *>(d->scratch) + meta_b + metas_b;
    ecc_corner *pk = reinterpret_cast<ecc_corner *>(base);
    int64_t *off = reinterpret_cast<int64_t *>(base + pk_b);
    int64_t *offs = reinterpret_cast<int64_t *>(base + pk_b + off_b);
    const int64_t my_t = h[2 * d->rank];
    if (my_t > 0) ECC_CHECK_HIP(ctx, hipMemcpyAsync(pk, packed, my_t * sizeof(ecc_corner), hipMemcpyDeviceToDevice, s), "pack");
    ECC_CHECK_HIP(ctx, hipMemsetAsync(off, 0, (size_t)(ns_max + 1) * 8, s), "memset(off)");
    if (n_slices > 0)
        ECC_CHECK_HIP(ctx, hipMemcpyAsync(off, offsets, (size_t)(n_slices + 1) * 8, hipMemcpyDeviceToDevice, s), "offs");
    ECC_CHECK_RCCL(d, rccl().all_gather(pk, all, (size_t)t_max * 3, ncclInt32, d->comm, s), "ncclAllGather(corners)");
    ECC_CHECK_RCCL(d, rccl().all_gather(off, offs, (size_t)ns_max + 1, ncclInt64, d->comm, s), "ncclAllGather(offsets)");
    const int64_t items = (int64_t)R * ns_max;
    hipLaunchKernelGGL(corner_slices_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s, offs, metas, R,
                       ns_max, t_max, starts, counts);
    ECC_CHECK_LAUNCH(ctx, "corner_slices");
    return ECC_OK;
}
