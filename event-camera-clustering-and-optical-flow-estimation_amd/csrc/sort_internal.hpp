// Device sorts shared by libecc's translation units (rocPRIM, sort.hip): the stable radix sort
// the any-N DBSCAN orders its clusters with, and the segmented sort that puts eps-neighbour lists
// into ascending index order (the order of DBSCAN_precomp.h's adjacency rows).
#pragma once

#include "ecc_internal.hpp"

namespace ecc {

size_t sort_pairs_u64_i32_temp_bytes(int64_t n, int end_bit);
// stable ascending sort of (keys, vals) over key bits [0, end_bit)
int sort_pairs_u64_i32(ecc_ctx *ctx, void *tmp, size_t tmp_bytes, const uint64_t *keys_in, uint64_t *keys_out,
                       const int32_t *vals_in, int32_t *vals_out, int64_t n, int end_bit, hipStream_t s);

size_t segsort_i32_temp_bytes(int64_t total, int64_t n_segs, bool with_f64);
// every segment [offsets[k], offsets[k+1]) of keys (and, if given, f64 values) sorted ascending
int segsort_i32(ecc_ctx *ctx, void *tmp, size_t tmp_bytes, const int32_t *keys_in, int32_t *keys_out,
                const double *vals_in, double *vals_out, int64_t total, int64_t n_segs, const int64_t *offsets,
                hipStream_t s);

}  // namespace ecc
