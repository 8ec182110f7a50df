// Context, status strings and workspace management for libecc.
// Reference counterpart: create_device()/clCreateContext/clCreateCommandQueue
// (SMP/metavision_sdk_get_started5_opencl_store.cpp:51-79, 233-270).  Unlike the reference,
// which re-creates (and leaks) a cl_mem per slice (DSA/…opencl_store.cpp:389, Q5), all
// scratch lives in one workspace owned by the context.
#include "ecc_internal.hpp"

namespace ecc {

int hip_fail(ecc_ctx *ctx, hipError_t e, const char *what) {
    if (ctx) {
        ctx->last_error = std::string(what) + ": " + hipGetErrorString(e);
    }
    return ECC_ERR_HIP;
}

int ws_reserve(ecc_ctx *ctx, size_t bytes) {
    if (!ctx) return ECC_ERR_INVALID;
    if (bytes <= ctx->ws_bytes) return ECC_OK;
    ECC_CHECK_HIP(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (ctx->ws) {
        // Work already queued on any stream may still use the old buffer.
        ECC_CHECK_HIP(ctx, hipDeviceSynchronize(), "hipDeviceSynchronize(ws grow)");
        ECC_CHECK_HIP(ctx, hipFree(ctx->ws), "hipFree(ws)");
        ctx->ws = nullptr;
        ctx->ws_bytes = 0;
    }
    size_t want = align_up(bytes, 1 << 20);
    hipError_t e = hipMalloc(&ctx->ws, want);
    if (e != hipSuccess) {
        ctx->ws = nullptr;
        hip_fail(ctx, e, "hipMalloc(ws)");
        return ECC_ERR_NOMEM;
    }
    ctx->ws_bytes = want;
    return ECC_OK;
}

static hipEvent_t pool_get(ecc_ctx *ctx) {
    if (!ctx->event_pool.empty()) {
        hipEvent_t e = ctx->event_pool.back();
        ctx->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

TimedLaunch::TimedLaunch(ecc_ctx *c, hipStream_t st, const char *n) : ctx(c), s(st), name(n) {
    if (!ctx || !ctx->timing) return;
    a = pool_get(ctx);
    if (a) hipEventRecord(a, s);
}

TimedLaunch::~TimedLaunch() {
    if (!a) return;
    hipEvent_t b = pool_get(ctx);
    if (!b) return;
    hipEventRecord(b, s);
    ctx->pending.push_back(EccTimingPair{name, a, b});
}

static void timing_collect(ecc_ctx *ctx) {
    if (ctx->pending.empty()) return;
    hipDeviceSynchronize();
    for (auto &p : ctx->pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            auto &st = ctx->stats[p.name];
            st.total_ms += ms;
            st.launches += 1;
        }
        ctx->event_pool.push_back(p.a);
        ctx->event_pool.push_back(p.b);
    }
    ctx->pending.clear();
}

}  // namespace ecc

ECC_API int ecc_ctx_set_timing(ecc_ctx *ctx, int enable) {
    if (!ctx) return ECC_ERR_INVALID;
    ctx->timing = enable != 0;
    return ECC_OK;
}

ECC_API int ecc_ctx_timing_reset(ecc_ctx *ctx) {
    if (!ctx) return ECC_ERR_INVALID;
    ecc::timing_collect(ctx);
    ctx->stats.clear();
    return ECC_OK;
}

ECC_API int ecc_ctx_timing_report(ecc_ctx *ctx, char *buf, size_t cap) {
    if (!ctx || !buf || cap == 0) return ECC_ERR_INVALID;
    ecc::timing_collect(ctx);
    std::string out = "{";
    bool first = true;
    for (auto &kv : ctx->stats) {
        char tmp[256];
        snprintf(tmp, sizeof(tmp), "%s\"%s\": {\"launches\": %lld, \"total_ms\": %.6f}",
                 first ? "" : ", ", kv.first.c_str(), (long long)kv.second.launches, kv.second.total_ms);
        out += tmp;
        first = false;
    }
    out += "}";
    if (out.size() + 1 > cap) return ECC_ERR_CAPACITY;
    memcpy(buf, out.c_str(), out.size() + 1);
    return ECC_OK;
}

ECC_API int ecc_version(void) { return ECC_VERSION; }

ECC_API const char *ecc_status_string(int s) {
    switch (s) {
        case ECC_OK: return "ok";
        case ECC_ERR_INVALID: return "invalid argument";
        case ECC_ERR_HIP: return "HIP runtime error";
        case ECC_ERR_UNSORTED_TIME: return "event timestamps are not non-decreasing";
        case ECC_ERR_CAPACITY: return "output capacity exceeded";
        case ECC_ERR_NOMEM: return "out of memory";
        case ECC_ERR_NO_DEVICE: return "no GPU device";
        default: return "unknown status";
    }
}

ECC_API int ecc_ctx_create(ecc_ctx **out, int device) {
    if (!out) return ECC_ERR_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ECC_ERR_NO_DEVICE;
    if (device < 0 || device >= n) return ECC_ERR_INVALID;
    ecc_ctx *ctx = new (std::nothrow) ecc_ctx();
    if (!ctx) return ECC_ERR_NOMEM;
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess || hipMalloc(&ctx->flags, 256) != hipSuccess ||
        hipMemset(ctx->flags, 0, 256) != hipSuccess) {
        delete ctx;
        return ECC_ERR_HIP;
    }
    int n_cu = 0;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && n_cu > 0)
        ctx->n_cu = n_cu;
    *out = ctx;
    return ECC_OK;
}

ECC_API int ecc_ctx_destroy(ecc_ctx *ctx) {
    if (!ctx) return ECC_ERR_INVALID;
    hipSetDevice(ctx->device);
    hipDeviceSynchronize();
    for (auto &p : ctx->pending) { hipEventDestroy(p.a); hipEventDestroy(p.b); }
    for (auto e : ctx->event_pool) hipEventDestroy(e);
    ecc::corner_state_release(ctx);
    ecc::nms_state_release(ctx);
    if (ctx->ws) hipFree(ctx->ws);
    if (ctx->flags) hipFree(ctx->flags);
    delete ctx;
    return ECC_OK;
}

ECC_API const char *ecc_ctx_last_error(const ecc_ctx *ctx) {
    return ctx ? ctx->last_error.c_str() : "";
}

ECC_API int ecc_stream_sync(ecc_stream_t stream) {
    return hipStreamSynchronize(ecc::as_stream(stream)) == hipSuccess ? ECC_OK : ECC_ERR_HIP;
}

// ---- runtime plumbing ---------------------------------------------------------------------
#define ECC_RT(call) return (call) == hipSuccess ? ECC_OK : ECC_ERR_HIP

ECC_API int ecc_device_count(int *n) {
    if (!n) return ECC_ERR_INVALID;
    *n = 0;
    if (hipGetDeviceCount(n) != hipSuccess) { *n = 0; return ECC_ERR_NO_DEVICE; }
    return ECC_OK;
}
ECC_API int ecc_set_device(int device) { ECC_RT(hipSetDevice(device)); }
ECC_API int ecc_dev_alloc(void **ptr, size_t bytes) {
    if (!ptr) return ECC_ERR_INVALID;
    if (hipMalloc(ptr, bytes ? bytes : 16) != hipSuccess) { *ptr = nullptr; return ECC_ERR_NOMEM; }
    return ECC_OK;
}
ECC_API int ecc_dev_free(void *ptr) { ECC_RT(hipFree(ptr)); }
ECC_API int ecc_memset_async(void *dst, int value, size_t bytes, ecc_stream_t s) {
    ECC_RT(hipMemsetAsync(dst, value, bytes, ecc::as_stream(s)));
}
ECC_API int ecc_device_sync(void) {
    ECC_RT(hipDeviceSynchronize());
}
ECC_API int ecc_memcpy_h2d(void *dst, const void *src, size_t bytes, ecc_stream_t s) {
    ECC_RT(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ecc::as_stream(s)));
}
ECC_API int ecc_memcpy_d2h(void *dst, const void *src, size_t bytes, ecc_stream_t s) {
    if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ecc::as_stream(s)) != hipSuccess)
        return ECC_ERR_HIP;
    ECC_RT(hipStreamSynchronize(ecc::as_stream(s)));
}
ECC_API int ecc_memcpy_d2d(void *dst, const void *src, size_t bytes, ecc_stream_t s) {
    ECC_RT(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ecc::as_stream(s)));
}
ECC_API int ecc_stream_create(ecc_stream_t *stream) {
    if (!stream) return ECC_ERR_INVALID;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return ECC_ERR_HIP;
    *stream = reinterpret_cast<ecc_stream_t>(s);
    return ECC_OK;
}
ECC_API int ecc_stream_destroy(ecc_stream_t stream) { ECC_RT(hipStreamDestroy(ecc::as_stream(stream))); }
ECC_API int ecc_event_create(void **event) {
    if (!event) return ECC_ERR_INVALID;
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return ECC_ERR_HIP;
    *event = reinterpret_cast<void *>(e);
    return ECC_OK;
}
ECC_API int ecc_event_destroy(void *event) { ECC_RT(hipEventDestroy(reinterpret_cast<hipEvent_t>(event))); }
ECC_API int ecc_event_record(void *event, ecc_stream_t s) {
    ECC_RT(hipEventRecord(reinterpret_cast<hipEvent_t>(event), ecc::as_stream(s)));
}
ECC_API int ecc_stream_wait_event(ecc_stream_t s, void *event) {
    if (!event) return ECC_ERR_INVALID;
    ECC_RT(hipStreamWaitEvent(ecc::as_stream(s), reinterpret_cast<hipEvent_t>(event), 0));
}
ECC_API int ecc_event_elapsed_ms(float *ms, void *start, void *stop) {
    if (!ms) return ECC_ERR_INVALID;
    if (hipEventSynchronize(reinterpret_cast<hipEvent_t>(stop)) != hipSuccess) return ECC_ERR_HIP;
    ECC_RT(hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start), reinterpret_cast<hipEvent_t>(stop)));
}

namespace {
__global__ void util_sqrt_kernel(const float *__restrict__ in, float *__restrict__ out, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        out[i] = ecc::sqrt_rn(in[i]);
}
}  // namespace

ECC_API int ecc_util_sqrt_f32(ecc_ctx *ctx, const float *in, float *out, int64_t n, ecc_stream_t stream) {
    if (!ctx || n < 0 || (n > 0 && (!in || !out))) return ECC_ERR_INVALID;
    if (n == 0) return ECC_OK;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(util_sqrt_kernel, dim3((unsigned)blocks), dim3(256), 0, ecc::as_stream(stream), in, out, n);
    ECC_CHECK_LAUNCH(ctx, "util_sqrt_kernel");
    return ECC_OK;
}

// ---- step capture (HIP graphs) --------------------------------------------------------------
struct ecc_graph {
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
};

ECC_API int ecc_graph_begin(ecc_stream_t stream) {
    if (!stream) return ECC_ERR_INVALID;
    return hipStreamBeginCapture(ecc::as_stream(stream), hipStreamCaptureModeRelaxed) == hipSuccess ? ECC_OK
                                                                                                  : ECC_ERR_HIP;
}

ECC_API int ecc_graph_end(ecc_stream_t stream, ecc_graph **out) {
    if (!stream || !out) return ECC_ERR_INVALID;
    *out = nullptr;
    auto *g = new ecc_graph();
    if (hipStreamEndCapture(ecc::as_stream(stream), &g->graph) != hipSuccess || !g->graph ||
        hipGraphInstantiate(&g->exec, g->graph, nullptr, nullptr, 0) != hipSuccess) {
        if (g->graph) (void)hipGraphDestroy(g->graph);
        delete g;
        return ECC_ERR_HIP;
    }
    *out = g;
    return ECC_OK;
}

ECC_API int ecc_graph_launch(ecc_graph *graph, ecc_stream_t stream) {
    if (!graph) return ECC_ERR_INVALID;
    return hipGraphLaunch(graph->exec, ecc::as_stream(stream)) == hipSuccess ? ECC_OK : ECC_ERR_HIP;
}

ECC_API int ecc_graph_destroy(ecc_graph *graph) {
    if (!graph) return ECC_OK;
    if (graph->exec) (void)hipGraphExecDestroy(graph->exec);
    if (graph->graph) (void)hipGraphDestroy(graph->graph);
    delete graph;
    return ECC_OK;
}
