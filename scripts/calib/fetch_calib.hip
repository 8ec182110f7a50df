// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths libecc's
// corner kernels use.  MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of a 16-B/lane
// coalesced read; other widths are uncalibrated.  Each kernel below moves a known number of bytes
// from a 512 MiB buffer (beyond the 256 MiB Infinity Cache, cold between kernels); the printed
// byte counts are compared with the counters by scripts/calib_report.py.
//
// build: hipcc -O3 --offload-arch=gfx950 -o scripts/calib/bin/fetch_calib scripts/calib/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            return 1;                                                               \
        }                                                                           \
    } while (0)

// coalesced reads, W bytes per lane per access, grid-strided over n_words W-byte words
template <typename T>
__device__ __forceinline__ void read_body(const T *__restrict__ p, int64_t n, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const T v = p[i];
        const uint32_t *w = reinterpret_cast<const uint32_t *>(&v);
#pragma unroll
        for (int k = 0; k < (int)(sizeof(T) / 4); ++k) acc ^= w[k];
    }
    if (acc == 0x12345678u) sink[0] = acc;  // keeps the loads
}

// gathers: one 8-B element per lane at a hashed index (a different 64-B line per lane)
__global__ void __launch_bounds__(256) gather8(const uint2 *__restrict__ p, int64_t n_elems, int64_t n_loads,
                                                      uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_loads; i += (int64_t)gridDim.x * 256) {
        const uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
        const int64_t j = (int64_t)((h >> 20) % (uint64_t)(n_elems / 8)) * 8;  // first element of a 64-B line
        const uint2 v = p[j];
        acc ^= v.x ^ v.y;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <typename T>
__device__ __forceinline__ void write_body(T *__restrict__ p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        T v;
        uint32_t *w = reinterpret_cast<uint32_t *>(&v);
#pragma unroll
        for (int k = 0; k < (int)(sizeof(T) / 4); ++k) w[k] = (uint32_t)i + k;
        p[i] = v;
    }
}

// plain kernel names (rocprofv3 prints them as they are)
__global__ void __launch_bounds__(256) read16(const uint4 *p, int64_t n, uint32_t *sink) { read_body(p, n, sink); }
__global__ void __launch_bounds__(256) read8(const uint2 *p, int64_t n, uint32_t *sink) { read_body(p, n, sink); }
__global__ void __launch_bounds__(256) read4(const uint32_t *p, int64_t n, uint32_t *sink) { read_body(p, n, sink); }
__global__ void __launch_bounds__(256) write16(uint4 *p, int64_t n) { write_body(p, n); }
__global__ void __launch_bounds__(256) write8(uint2 *p, int64_t n) { write_body(p, n); }
__global__ void __launch_bounds__(256) write4(uint32_t *p, int64_t n) { write_body(p, n); }

// one 1-B store per lane, coalesced (the corner flags are written 4 per lane instead)
__global__ void __launch_bounds__(256) write1(uint8_t *__restrict__ p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = (uint8_t)i;
}

int main() {
    const int64_t bytes = 512ll << 20;
    void *buf = nullptr, *flush = nullptr;
    uint32_t *sink = nullptr;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&flush, bytes));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(buf, 1, bytes));
    const dim3 grid(2048), block(256);
    auto flush_caches = [&]() { return hipMemset(flush, 2, bytes); };  // evicts buf from L2/MALL
    // name, algorithmic bytes
    CHECK(flush_caches());
    hipLaunchKernelGGL(read16, grid, block, 0, 0, (const uint4 *)buf, bytes / 16, sink);
    std::printf("read16 %lld\n", (long long)bytes);
    CHECK(flush_caches());
    hipLaunchKernelGGL(read8, grid, block, 0, 0, (const uint2 *)buf, bytes / 8, sink);
    std::printf("read8 %lld\n", (long long)bytes);
    CHECK(flush_caches());
    hipLaunchKernelGGL(read4, grid, block, 0, 0, (const uint32_t *)buf, bytes / 4, sink);
    std::printf("read4 %lld\n", (long long)bytes);
    CHECK(flush_caches());
    const int64_t n_loads = 1 << 22;  // 4 M gathers, one 64-B line each (some lines repeat)
    hipLaunchKernelGGL(gather8, grid, block, 0, 0, (const uint2 *)buf, bytes / 8, n_loads, sink);
    {  // distinct 64-B lines the gathers touch (the same hash on the host)
        std::vector<uint8_t> seen((size_t)(bytes / 64), 0);
        long long distinct = 0;
        for (int64_t i = 0; i < n_loads; ++i) {
            const uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
            const int64_t line = (int64_t)((h >> 20) % (uint64_t)(bytes / 64));
            distinct += seen[line] ? 0 : 1;
            seen[line] = 1;
        }
        std::printf("gather8 %lld\n", distinct * 64);
    }
    CHECK(flush_caches());
    hipLaunchKernelGGL(write16, grid, block, 0, 0, (uint4 *)buf, bytes / 16);
    std::printf("write16 %lld\n", (long long)bytes);
    CHECK(flush_caches());
    hipLaunchKernelGGL(write8, grid, block, 0, 0, (uint2 *)buf, bytes / 8);
    std::printf("write8 %lld\n", (long long)bytes);
    CHECK(flush_caches());
    hipLaunchKernelGGL(write4, grid, block, 0, 0, (uint32_t *)buf, bytes / 4);
    std::printf("write4 %lld\n", (long long)bytes);
    CHECK(flush_caches());
    hipLaunchKernelGGL(write1, grid, block, 0, 0, (uint8_t *)buf, bytes);
    std::printf("write1 %lld\n", (long long)bytes);
    CHECK(hipDeviceSynchronize());
    CHECK(hipFree(buf));
    CHECK(hipFree(flush));
    CHECK(hipFree(sink));
    return 0;
}
