// Device exclusive scan int32 -> int64 (offsets with a trailing total), shared by the
// eps-list and corner-binning paths: block sums -> single-WG scan of the sums -> finish.
#include "ecc_internal.hpp"

namespace {
// ---- exclusive scan int32 -> int64 (3 kernels: block sums, scan of sums, finish) ----------
constexpr int kThreads = 256;
constexpr int kScanBlock = 1024;  // elements per block (4 per thread)

__global__ void __launch_bounds__(kThreads)
scan_block_sums(const int32_t *__restrict__ in, int64_t n, int64_t *__restrict__ bsum) {
    __shared__ int64_t red[kThreads / 64];
    const int64_t b0 = (int64_t)blockIdx.x * kScanBlock;
    int64_t s = 0;
    for (int k = 0; k < 4; ++k) {
        const int64_t i = b0 + threadIdx.x * 4 + k;
        if (i < n) s += in[i];
    }
    s = ecc::wave_sum_i64(s);  // DPP
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) bsum[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(kThreads)
scan_sums(int64_t *__restrict__ bsum, int64_t nb) {
    // single workgroup: exclusive scan in place, chunks of kThreads
    __shared__ int64_t wtot[kThreads / 64];
    int64_t carry = 0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t c0 = 0; c0 < nb; c0 += kThreads) {
        const int64_t i = c0 + threadIdx.x;
        const int64_t v = i < nb ? bsum[i] : 0;
        const int64_t inc = ecc::wave_incl_scan_i64(v);  // DPP
        if (lane == 63) wtot[wave] = inc;
        __syncthreads();
        int64_t off = carry + inc - v, tot = 0;
        for (int w = 0; w < kThreads / 64; ++w) {
            if (w < wave) off += wtot[w];
            tot += wtot[w];
        }
        if (i < nb) bsum[i] = off;
        carry += tot;
        __syncthreads();
    }
}

__global__ void __launch_bounds__(kThreads)
scan_finish(const int32_t *__restrict__ in, int64_t n, const int64_t *__restrict__ bsum,
            int64_t *__restrict__ out) {
    __shared__ int64_t wtot[kThreads / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t b0 = (int64_t)blockIdx.x * kScanBlock;
    int64_t v[4], s = 0;
    for (int k = 0; k < 4; ++k) {
        const int64_t i = b0 + threadIdx.x * 4 + k;
        v[k] = i < n ? in[i] : 0;
        s += v[k];
    }
    const int64_t inc = ecc::wave_incl_scan_i64(s);  // DPP
    if (lane == 63) wtot[wave] = inc;
    __syncthreads();
    int64_t off = bsum[blockIdx.x] + inc - s;
    for (int w = 0; w < wave; ++w) off += wtot[w];
    for (int k = 0; k < 4; ++k) {
        const int64_t i = b0 + threadIdx.x * 4 + k;
        if (i < n) out[i] = off;
        off += v[k];
        if (i == n - 1) out[n] = off;  // total
    }
}

}  // namespace

namespace ecc {

size_t scan_scratch_bytes(int64_t n) { return (size_t)((n + kScanBlock - 1) / kScanBlock) * 8 + 256; }

int exclusive_scan_i32_i64(ecc_ctx *ctx, const int32_t *in, int64_t n, int64_t *out, int64_t *scratch,
                           hipStream_t s) {
    if (n <= 0) {
        if (n == 0) ECC_CHECK_HIP(ctx, hipMemsetAsync(out, 0, 8, s), "scan(empty)");
        return ECC_OK;
    }
    const int64_t nb = (n + kScanBlock - 1) / kScanBlock;
    {
        ECC_TIMED(ctx, s, "scan_block_sums");
        hipLaunchKernelGGL(scan_block_sums, dim3((unsigned)nb), dim3(kThreads), 0, s, in, n, scratch);
    }
    {
        ECC_TIMED(ctx, s, "scan_sums");
        hipLaunchKernelGGL(scan_sums, dim3(1), dim3(kThreads), 0, s, scratch, nb);
    }
    {
        ECC_TIMED(ctx, s, "scan_finish");
        hipLaunchKernelGGL(scan_finish, dim3((unsigned)nb), dim3(kThreads), 0, s, in, n, scratch, out);
    }
    ECC_CHECK_LAUNCH(ctx, "exclusive_scan");
    return ECC_OK;
}

}  // namespace ecc
