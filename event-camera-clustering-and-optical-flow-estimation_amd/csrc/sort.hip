// rocPRIM device sorts behind sort_internal.hpp (one translation unit: rocPRIM's templates are
// heavy to compile, so every caller shares these instantiations).
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "sort_internal.hpp"

namespace ecc {

size_t sort_pairs_u64_i32_temp_bytes(int64_t n, int end_bit) {
    size_t bytes = 0;
    rocprim::radix_sort_pairs(nullptr, bytes, (uint64_t *)nullptr, (uint64_t *)nullptr, (int32_t *)nullptr,
                              (int32_t *)nullptr, (size_t)n, 0u, (unsigned)end_bit, hipStream_t(0));
    return bytes;
}

int sort_pairs_u64_i32(ecc_ctx *ctx, void *tmp, size_t tmp_bytes, const uint64_t *keys_in, uint64_t *keys_out,
                       const int32_t *vals_in, int32_t *vals_out, int64_t n, int end_bit, hipStream_t s) {
    ECC_TIMED(ctx, s, "radix_sort_pairs");
    ECC_CHECK_HIP(ctx,
                  rocprim::radix_sort_pairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out, (size_t)n, 0u,
                                            (unsigned)end_bit, s),
                  "rocprim::radix_sort_pairs");
    return ECC_OK;
}

size_t segsort_i32_temp_bytes(int64_t total, int64_t n_segs, bool with_f64) {
    size_t bytes = 0;
    if (with_f64)
        rocprim::segmented_radix_sort_pairs(nullptr, bytes, (int32_t *)nullptr, (int32_t *)nullptr, (double *)nullptr,
                                            (double *)nullptr, (unsigned)total, (unsigned)n_segs,
                                            (const int64_t *)nullptr, (const int64_t *)nullptr, 0u, 32u, hipStream_t(0));
    else
        rocprim::segmented_radix_sort_keys(nullptr, bytes, (int32_t *)nullptr, (int32_t *)nullptr, (unsigned)total,
                                           (unsigned)n_segs, (const int64_t *)nullptr, (const int64_t *)nullptr, 0u,
                                           32u, hipStream_t(0));
    return bytes;
}

int segsort_i32(ecc_ctx *ctx, void *tmp, size_t tmp_bytes, const int32_t *keys_in, int32_t *keys_out,
                const double *vals_in, double *vals_out, int64_t total, int64_t n_segs, const int64_t *offsets,
                hipStream_t s) {
    ECC_TIMED(ctx, s, "segmented_radix_sort");
    if (vals_in)
        ECC_CHECK_HIP(ctx,
                      rocprim::segmented_radix_sort_pairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out,
                                                          (unsigned)total, (unsigned)n_segs, offsets, offsets + 1, 0u,
                                                          32u, s),
                      "rocprim::segmented_radix_sort_pairs");
    else
        ECC_CHECK_HIP(ctx,
                      rocprim::segmented_radix_sort_keys(tmp, tmp_bytes, keys_in, keys_out, (unsigned)total,
                                                         (unsigned)n_segs, offsets, offsets + 1, 0u, 32u, s),
                      "rocprim::segmented_radix_sort_keys");
    return ECC_OK;
}

}  // namespace ecc
