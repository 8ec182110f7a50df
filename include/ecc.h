/*
 * ecc.h — C ABI of the MI355X-native event-camera clustering / corner pipeline.
 *
 * Drop-in boundary for the hot path of
 * LogicTronixInc/Event-Camera-Clustering-and-Optical-Flow-Estimation:
 *
 *   hash-map downsample -> k-means / DBSCAN / OPTICS eps-neighbour -> SAE + FAST arc corners
 *   -> box NMS -> predictor-corrector corner tracker
 *
 * Every compute entry point takes DEVICE pointers (hipMalloc'd memory on the context's GPU)
 * plus an opaque stream (a hipStream_t passed as void*, NULL = default stream) and enqueues
 * work asynchronously, mirroring the OpenCL clEnqueueNDRangeKernel boundary the reference
 * uses.  Return value: ECC_OK (0) or a negative ecc_status, mirroring the reference's
 * `if (err < 0) { perror(...); exit(1); }` convention (SMP/…opencl_store.cpp:256-260).
 *
 * Canonical data layout in HBM (SoA): xy = packed u32 (x | y << 16), t = int64 µs,
 * p = u8.  The reference copies EventCD{u16 x,u16 y,i16 p,i64 t} into int arrays.
 *
 * Reference interface each entry point replaces is cited on the declaration.
 * Quirk decisions (ref_compat vs fixed) follow SURVEY.md Appendix A.
 */
#ifndef ECC_H
#define ECC_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ECC_VERSION 1

typedef void *ecc_stream_t; /* hipStream_t */

typedef enum ecc_status {
    ECC_OK = 0,
    ECC_ERR_INVALID = -1,       /* bad argument / shape */
    ECC_ERR_HIP = -2,           /* HIP runtime error (launch, memcpy, malloc) */
    ECC_ERR_UNSORTED_TIME = -3, /* event timestamps decrease inside a batch */
    ECC_ERR_CAPACITY = -4,      /* an output capacity was exceeded (result truncated) */
    ECC_ERR_NOMEM = -5,         /* host / device allocation failed */
    ECC_ERR_NO_DEVICE = -6      /* no GPU visible */
} ecc_status;

typedef struct ecc_ctx ecc_ctx; /* per-stream context: device id + scratch workspace */

/* Reference: create_device()/clCreateContext (SMP/…opencl_store.cpp:51-79, 233-240). */
int ecc_ctx_create(ecc_ctx **out, int device);
int ecc_ctx_destroy(ecc_ctx *ctx);
const char *ecc_status_string(int status);
int ecc_version(void);
/* Last HIP error string recorded by this context (for ECC_ERR_HIP). */
const char *ecc_ctx_last_error(const ecc_ctx *ctx);
/* Blocks until all work queued by this library on `stream` has finished. */
int ecc_stream_sync(ecc_stream_t stream);
/* Blocks until all work on the current device (every stream) has finished. */
int ecc_device_sync(void);

/* Runtime plumbing (the reference's clCreateBuffer / clEnqueueRead/WriteBuffer /
 * clGetEventProfilingInfo, SMP/…opencl_store.cpp:264-268, 406-422) so hosts and tests need
 * no other GPU runtime.  Copies are stream-ordered; *_sync variants block. */
int ecc_device_count(int *n);
int ecc_set_device(int device);
int ecc_dev_alloc(void **ptr, size_t bytes);
int ecc_dev_free(void *ptr);
int ecc_memset_async(void *dst, int value, size_t bytes, ecc_stream_t stream);
int ecc_memcpy_h2d(void *dst, const void *src, size_t bytes, ecc_stream_t stream);
int ecc_memcpy_d2h(void *dst, const void *src, size_t bytes, ecc_stream_t stream);
int ecc_memcpy_d2d(void *dst, const void *src, size_t bytes, ecc_stream_t stream);
int ecc_stream_create(ecc_stream_t *stream);
int ecc_stream_destroy(ecc_stream_t stream);
int ecc_event_create(void **event);
int ecc_event_destroy(void *event);
int ecc_event_record(void *event, ecc_stream_t stream);
int ecc_event_elapsed_ms(float *ms, void *start, void *stop); /* synchronises `stop` */
int ecc_stream_wait_event(ecc_stream_t stream, void *event); /* stream waits for `event` */

/* Per-kernel timing (the reference's CL_QUEUE_PROFILING_ENABLE + clGetEventProfilingInfo,
 * SMP/…opencl_store.cpp:263-264, 406-412): when enabled, every kernel this context launches
 * is bracketed by HIP events on its stream.  The report (JSON object
 * {"<kernel>": {"launches": n, "total_ms": t}, ...}) synchronises the device first. */
int ecc_ctx_set_timing(ecc_ctx *ctx, int enable);
int ecc_ctx_timing_reset(ecc_ctx *ctx);
int ecc_ctx_timing_report(ecc_ctx *ctx, char *buf, size_t cap);

/* Step capture with HIP graphs (no reference counterpart: the reference re-issues every OpenCL
 * command per slice, SMP/…opencl_store.cpp:370-459).  Work issued on `stream` between
 * ecc_graph_begin and ecc_graph_end is recorded, not run; ecc_graph_launch replays it with the
 * same pointers and sizes.  Run the sequence once eagerly first (workspaces are allocated
 * outside the capture) and keep per-kernel timing off while capturing.  `stream` must be a
 * created stream, not the null stream. */
typedef struct ecc_graph ecc_graph;
int ecc_graph_begin(ecc_stream_t stream);
int ecc_graph_end(ecc_stream_t stream, ecc_graph **out);
int ecc_graph_launch(ecc_graph *graph, ecc_stream_t stream);
int ecc_graph_destroy(ecc_graph *graph);

/* Numerics self-check: out[i] = correctly rounded fp32 sqrt(in[i]) as used by every bit-exact
 * kernel of this library (device pointers).  Lets tests pin the device arithmetic against
 * IEEE sqrtf on the host. */
int ecc_util_sqrt_f32(ecc_ctx *ctx, const float *in, float *out, int64_t n, ecc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * 1. Hash-map downsample
 * Reference: __kernel process_coordinates(input_coords, repeated_coords, unique_coords,
 *            repeated_count, unique_count, total_coords, width, height)
 *            SMP/build/coordinate_processor.cl:3-14 (hash), :16-89 (kernel);
 *            host launch SMP/…opencl_store.cpp:250-312, DSA/…opencl_store.cpp:370-445.
 * Events are cut into contiguous windows of `window` events (reference ring: 8192 pairs).
 * Per window: bucket h = (x*mult_x + y*mult_y) % n_buckets for events with
 * 0<=x<=x_max && 0<=y<=y_max (inclusive, coordinate_processor.cl:56); the first hit of a
 * bucket (canonical: LOWEST event index, Appendix A Q2) is the representative; a bucket's
 * second hit increments `repeated`.  Outputs (any may be NULL):
 *   rep_xy [n_windows*window]  packed xy of representatives of window w at w*window + k,
 *                              k < win_unique[w], ascending event index;
 *   rep_idx[n_windows*window]  global event index of the same representatives;
 *   win_unique[n_windows], win_repeated[n_windows] per-window counts (Q4: not cumulative).
 * n_windows = ceil(n / window).  Bit-exact vs oracle/ and the reference kernel's counts.
 * ------------------------------------------------------------------------------------- */
typedef struct ecc_hash_cfg {
    int32_t window;    /* events per window, 1..16384 (reference 8192) */
    int32_t x_max;     /* inclusive bound (reference 1280) */
    int32_t y_max;     /* inclusive bound (reference 720) */
    int32_t mult_x;    /* 1619 */
    int32_t mult_y;    /* 31 */
    int32_t n_buckets; /* 8192 (fixed: LDS table size) */
} ecc_hash_cfg;

void ecc_hash_cfg_default(ecc_hash_cfg *cfg);
int ecc_downsample_hash(ecc_ctx *ctx, const uint32_t *xy, int64_t n, const ecc_hash_cfg *cfg,
                        uint32_t *rep_xy, uint32_t *rep_idx, int32_t *win_unique,
                        int32_t *win_repeated, ecc_stream_t stream);

/* Exact (x, y) deduplication per window.
 * Reference: analyzeCoordinates / findCoordinate FCT/metavision_time_surface_periodic.cpp:56-120
 *   (linear search over the unique list: first-occurrence order, a count per coordinate; it
 *   prints the unique count).  Windows of `window` events (<= 8192 pairs: ARRAY_SIZE 16384 ints),
 *   the last one partial.  Outputs, per window w (base = w * window):
 *   n_unique[w] = the number of distinct (x, y) in the window (the reference's uniqueCount);
 *   uniq_idx[base + k] = global index of the k-th distinct coordinate's first event (ascending);
 *   uniq_cnt[base + k] = how many events of the window carry it (the reference's count).
 *   Any output may be NULL. */
int ecc_dedup_exact(ecc_ctx *ctx, const uint32_t *xy, int64_t n, int32_t window, uint32_t *uniq_idx,
                    int32_t *uniq_cnt, int32_t *n_unique, ecc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * 2. k-means (2-D, k <= 64)
 * Reference: __kernel assign_to_centers / assign_data_cluster / reduction_scalar
 *            KM/assign_to_centers.cl:1-34, :36-119, :121-140; host loop
 *            KM/assign_to_centers2.c:184-548.
 * Assignment (a5, Q10): d_c = sqrtf(dx*dx + dy*dy) in fp32 with dx = cx - px, first
 * minimum with strict `<` starting from `threshold` (50); no centre closer => label 255.
 * Update ("fixed" mode, Q7-Q9): c = (sum x / n, sum y / n) over assigned points (exact
 * integer / fp64 sums), unchanged when n == 0; stop after `max_iters` updates or once the
 * largest per-coordinate centroid shift <= tol (tol < 0: never).  After the loop, labels
 * (if non-NULL) are the assignment against the FINAL centroids.
 * Points: packed u16 xy (the downsample output) or interleaved float xy.
 * Segmented input (downsample layout): point j of segment s is at s*seg_stride + j,
 * j < seg_counts[s] (device int32[n_segs]); pass seg_counts = NULL for a dense array of
 * n_points (= n_segs*seg_stride is then ignored; use n_segs = 1, seg_stride = n_points).
 * centroids: DEVICE float[2k] (x0,y0,x1,y1,...) in/out.  iters_out: DEVICE int32[1] or NULL.
 * ------------------------------------------------------------------------------------- */
typedef struct ecc_kmeans_cfg {
    int32_t k;         /* number of centres, 1..64 */
    int32_t max_iters; /* >= 0 */
    float threshold;   /* 50.0f */
    float tol;         /* convergence tolerance on centroid shift; < 0 disables */
} ecc_kmeans_cfg;

void ecc_kmeans_cfg_default(ecc_kmeans_cfg *cfg);
int ecc_kmeans_run_xy16(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                        const int32_t *seg_counts, const ecc_kmeans_cfg *cfg, float *centroids,
                        uint8_t *labels, int32_t *iters_out, ecc_stream_t stream);
int ecc_kmeans_run_f32(ecc_ctx *ctx, const float *xy, int64_t n_points, const ecc_kmeans_cfg *cfg,
                       float *centroids, uint8_t *labels, int32_t *iters_out, ecc_stream_t stream);
/* ecc_kmeans_run_xy16 with the sensor frame known (1 <= frame_w, frame_h <= 2048): the per-pixel
 * counts cover [0, frame_w) x [0, frame_h) with no bounding-box pass; points outside the frame
 * are still assigned (listed and added point by point).  Same results as ecc_kmeans_run_xy16. */
int ecc_kmeans_run_xy16_frame(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                              const int32_t *seg_counts, int32_t frame_w, int32_t frame_h,
                              const ecc_kmeans_cfg *cfg, float *centroids, uint8_t *labels,
                              int32_t *iters_out, ecc_stream_t stream);
/* The same with an explicit assignment engine for k <= 32 (BASELINE config C3): 0 = default
 * (the vector engine), 1 = vector (centres in scalar registers, exact fp32 d^2 per centre),
 * 2 = matrix cores (d^2 - |p|^2 from v_mfma_f32_4x4x1f32, exact fallback near ties, the
 * winner's exact d^2 against the threshold), 3 = matrix cores in the streaming form (16 centres x
 * 32 points per v_mfma_f32_32x32x2f32, same margin and fallback; k <= 16 with 16-byte aligned xy,
 * otherwise engine 2).  All return the reference's labels; sums are fp64 (exact for
 * integer-valued coordinates).  xy must be 8-byte aligned. */
int ecc_kmeans_run_f32_engine(ecc_ctx *ctx, const float *xy, int64_t n_points, const ecc_kmeans_cfg *cfg,
                              int32_t engine, float *centroids, uint8_t *labels, int32_t *iters_out,
                              ecc_stream_t stream);
/* The reference's k-means host loop in "ref_compat" mode (KM/assign_to_centers2.c:184-548 over
 * KM/assign_to_centers.cl): 8 centres, n <= 16384 float (x, y)
 * points in 8 bins of 2048 (a point past its bin's 2048th is counted, not stored); the bins are
 * zeroed once and never cleared (Q8: a bin keeps earlier passes' values past its count; filled
 * here in point-index order, where the reference's kernel appends in atomic order); each
 * 1024-float chunk summed as reduction_scalar's pairwise tree; the update's partial-sum indexing
 * ss[j], ss[j+1] / ss[j+2], ss[j+3] for j = 2c (Q7), C's int abs of the float shift with the
 * running-maximum selective update, and the restart while that maximum is > 10 (Q9), at most
 * max_passes passes.  centroids16: DEVICE float[16] (x0, y0, .., x7, y7) in/out; passes_out
 * DEVICE int32[1], bin_counts_out DEVICE int32[8] (cluster_index) and partial_sums_out DEVICE
 * float[32] (the chunk sums) of the last pass, each may be NULL.  Bit-exact vs the oracle's
 * orc_kmeans_refcompat, whose passes are pinned against the reference's kernels.  The product's
 * default is the "fixed" loop above (ecc_kmeans_run_*). */
int ecc_kmeans_refcompat_f32(ecc_ctx *ctx, const float *xy, int64_t n, float *centroids16, int32_t max_passes,
                             int32_t *passes_out, int32_t *bin_counts_out, float *partial_sums_out,
                             ecc_stream_t stream);
/* Split form of one Lloyd iteration, for multi-GPU: each rank accumulates its shard's exact
 * integer partial sums into acc (DEVICE uint64[3k]: count, sum x, sum y per centre; added to,
 * so zero it first), the ranks all-reduce acc (SUM), then every rank applies the identical
 * update (which also zeroes acc).  state: DEVICE int32[2] = {done, iterations}, zeroed by the
 * caller before the first iteration; once done, further accumulate/update calls are no-ops. */
int ecc_kmeans_accumulate_xy16(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                               const int32_t *seg_counts, const float *centroids, int32_t k,
                               float threshold, uint64_t *acc, const int32_t *state,
                               ecc_stream_t stream);
int ecc_kmeans_update(ecc_ctx *ctx, uint64_t *acc, float *centroids, int32_t k, float tol,
                      int32_t *state, ecc_stream_t stream);
/* Final labels against given centroids (packed u16 points, segmented). */
int ecc_kmeans_labels_xy16(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                           const int32_t *seg_counts, const float *centroids, int32_t k,
                           float threshold, uint8_t *labels, ecc_stream_t stream);
/* Count-image form (multi-GPU: ONE all-reduce per k-means instead of one per Lloyd pass).
 * ecc_kmeans_counts_xy16 writes counts[y*frame_w + x] (u32) = the number of points at (x, y)
 * (a point outside the frame sets the flag ecc_kmeans_counts_status reports as
 * ECC_ERR_INVALID).  Count images are additive over shards; ecc_kmeans_run_counts runs the
 * Lloyd passes ("fixed" mode, k <= 32) over a (summed) image: the same integer sums, hence the
 * same centroids, as ecc_kmeans_run_xy16 over all the points.  Labels: ecc_kmeans_labels_xy16. */
int ecc_kmeans_counts_xy16(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                           const int32_t *seg_counts, int32_t frame_w, int32_t frame_h, uint32_t *counts,
                           ecc_stream_t stream);
int ecc_kmeans_counts_status(ecc_ctx *ctx, ecc_stream_t stream);
int ecc_kmeans_run_counts(ecc_ctx *ctx, const uint32_t *counts, int32_t frame_w, int32_t frame_h,
                          const ecc_kmeans_cfg *cfg, float *centroids, int32_t *iters_out, ecc_stream_t stream);
/* One assignment pass only (assign_to_centers): labels[i] in [0,k) or 255. */
int ecc_kmeans_assign_f32(ecc_ctx *ctx, const float *xy, int64_t n_points, const float *centroids,
                          int32_t k, float threshold, uint8_t *labels, ecc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * 3. SAE (time surface) + FAST/arc corner detection
 * Reference: FCT/metavision_time_surface_periodic_group_track.cpp:884-1063 (aggregate lambda:
 *            batch SAE update :900-923, arc test :948-1063, circles :44-45), slices of
 *            16384 events (make_n_events, :772-774), detection from the 2nd slice on (:926).
 * Semantics per slice s (events [s*slice, (s+1)*slice)): first ALL events of the slice write
 * sae[y][x] = t (Q14, batch), then every event is tested: border events
 * (x<m || x>=W-m || y<m || y>=H-m, m = margin 4, W/H = sensor size: Q12) are skipped
 * (border_mode 0 = fixed) or end the slice's tests (border_mode 1 = ref_compat `break`,
 * Q11); corner = circle3 streak (len 3..6 of 16) AND circle4 streak (len 4..8 of 20).
 * Slices with global index < first_detect_slice are not tested (Q15: pass 1 for a fresh
 * stream, 0 when continuing a stream).
 * sae: DEVICE int64[H*W], row-major, holds the initial SAE on entry and the final SAE on
 * exit (stream continuation / multi-GPU hand-off).  Timestamps must be non-decreasing
 * (Metavision stream order) -> ECC_ERR_UNSORTED_TIME otherwise (flag checked on device,
 * reported by ecc_fast_detect_status()).
 * corner_flags: DEVICE uint8[n], 1 = corner.  Bit-exact vs oracle/.
 * ------------------------------------------------------------------------------------- */
typedef struct ecc_corner_cfg {
    int32_t width, height;      /* sensor size */
    int32_t slice_events;       /* 16384 */
    int32_t margin;             /* 4 */
    int32_t border_mode;        /* 0 fixed (continue), 1 ref_compat (break) */
    int32_t first_detect_slice; /* 1 */
    int32_t any_order;          /* 0: timestamps non-decreasing (checked: ECC_ERR_UNSORTED_TIME);
                                 * 1: any order - the SAE keeps the LAST writer in stream order
                                 * (Q14) and every arc test takes the exact path; ecc_fast_detect
                                 * only (the multi-GPU hand-off combines shards by max time) */
} ecc_corner_cfg;

void ecc_corner_cfg_default(ecc_corner_cfg *cfg);
int ecc_fast_detect(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n,
                    const ecc_corner_cfg *cfg, int64_t *sae, uint8_t *corner_flags,
                    ecc_stream_t stream);
/* The same in two calls, for the multi-GPU SAE hand-off: prepare sorts the batch and writes
 * local_last[H*W] = the batch's own last timestamp per pixel (0 where untouched; no SAE input
 * needed), finish then runs the detection from the initial SAE `sae` (updated in place) with
 * the same xy/t/n/cfg on the same context.  prepare + finish == ecc_fast_detect. */
int ecc_fast_detect_prepare(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n,
                            const ecc_corner_cfg *cfg, int64_t *local_last, ecc_stream_t stream);
int ecc_fast_detect_finish(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n,
                           const ecc_corner_cfg *cfg, int64_t *sae, uint8_t *corner_flags,
                           ecc_stream_t stream);
/* Synchronises `stream` and reports the verdict of the LAST detection call on this context:
 * ECC_ERR_UNSORTED_TIME if its batch had decreasing timestamps, else ECC_OK.
 *  - ecc_fast_detect / _nms: that call's batch.
 *  - ecc_fast_detect_prepare: the prepared batch (known as soon as the sort phase ran).
 *  - ecc_fast_detect_finish / _finish_nms: the batch of the prepare it finishes.
 *  - a call with n == 0: ECC_OK.
 * Every sort phase carries its own tag, so a verdict never leaks into a later call: a prepare
 * that is abandoned (never finished) affects only itself; the next prepare or full call starts
 * clean.  A finish reports (and consumes) the verdict of the most recent prepare on the
 * context. */
int ecc_fast_detect_status(ecc_ctx *ctx, ecc_stream_t stream);
/* Diagnostics of the last ecc_fast_detect / _finish on this context (synchronises `stream`):
 * out[0] = (group of 32 slices, 14x14 tile) work items, out[1] = items tested by the dense-plane
 * kernel (windows holding more values than the compact per-pixel lists take, and items whose
 * clamped 32-bit keys could not decide a test: those take the exact int64 path), out[2] =
 * slices, out[3] = groups.  Writes min(n_out, 4). */
int ecc_fast_detect_stats(ecc_ctx *ctx, int64_t *out, int32_t n_out, ecc_stream_t stream);
/* Multi-GPU SAE hand-off: out[q] = max over images[i*hw + q], i < n_images (the shards'
 * local final SAEs of all LOWER ranks give a rank its exact initial SAE; max == last writer
 * because time is non-decreasing across shards). */
int ecc_sae_max_combine(ecc_ctx *ctx, const int64_t *images, int32_t n_images, int64_t hw,
                        int64_t *out, ecc_stream_t stream);
/* Final-SAE-only pass (used for the multi-GPU hand-off: per-shard local SAE). */
int ecc_sae_scatter(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n, int32_t width,
                    int32_t height, int64_t *sae, ecc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * 4. Greedy box NMS per slice
 * Reference: CornerFilter::filterCorners(corners, W, H, box_size=15, threshold)
 *            FCT/…group_track.cpp:69-153, called per slice at :832-837.
 * Corners of slice s are the events with corner_flags==1 in event order; a corner is kept
 * iff its clipped box [x±box/2]×[y±box/2] touches no box of an earlier kept corner; kept
 * corner label = its rank in the kept list (":140").  out: DEVICE ecc_corner[n_slices*cap],
 * slice s at s*cap; out_count: DEVICE int32[n_slices] (counts are clamped to cap).
 * Corners must lie inside the image (ecc_fast_detect never flags border events).
 * ------------------------------------------------------------------------------------- */
typedef struct ecc_corner { int32_t x, y, label; } ecc_corner; /* reference struct Corner */

int ecc_corner_nms(ecc_ctx *ctx, const uint32_t *xy, const uint8_t *corner_flags, int64_t n,
                   int32_t slice_events, int32_t width, int32_t height, int32_t box_size,
                   int32_t cap, ecc_corner *out, int32_t *out_count, ecc_stream_t stream);
/* Synchronises `stream`; ECC_ERR_CAPACITY if a slice kept more than `cap` corners in the last
 * ecc_corner_nms / ecc_fast_detect_nms, ECC_ERR_INVALID if a flagged event lay outside the image
 * (it was skipped). */
int ecc_corner_nms_status(ecc_ctx *ctx, ecc_stream_t stream);
/* Detection followed by the per-slice NMS, as the reference's slice loop runs them
 * (FCT/…group_track.cpp:832-837: detect, then filterCorners on the slice's corners):
 * == ecc_fast_detect(ctx, xy, t, n, cfg, sae, corner_flags) then ecc_corner_nms(ctx, xy,
 * corner_flags, n, cfg->slice_events, cfg->width, cfg->height, box_size, cap, out, out_count),
 * same outputs and status calls.  With slices of at most 16384 events (a multiple of 4) the
 * flag pass writes the NMS candidate lists itself, so NMS does not re-read the flags. */
int ecc_fast_detect_nms(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n,
                        const ecc_corner_cfg *cfg, int64_t *sae, uint8_t *corner_flags, int32_t box_size,
                        int32_t cap, ecc_corner *out, int32_t *out_count, ecc_stream_t stream);
/* The finish half of ecc_fast_detect_nms after ecc_fast_detect_prepare on the same context:
 * prepare + finish_nms == ecc_fast_detect_nms.  Time-window shards of one stream (several
 * GPUs, or several contexts and streams on one GPU) each prepare their shard, take their
 * initial SAE as the ecc_sae_max_combine of the lower shards' local_last images, and finish. */
int ecc_fast_detect_finish_nms(ecc_ctx *ctx, const uint32_t *xy, const int64_t *t, int64_t n,
                               const ecc_corner_cfg *cfg, int64_t *sae, uint8_t *corner_flags,
                               int32_t box_size, int32_t cap, ecc_corner *out, int32_t *out_count,
                               ecc_stream_t stream);
/* Dense form of ecc_corner_nms' per-slice lists (multi-GPU corner gather): with
 * counts[s] <= cap as ecc_corner_nms writes them, offsets[0..n_slices] (DEVICE int64) = the
 * exclusive scan of counts (offsets[n_slices] = total) and out[offsets[s] + d] = in[s*cap + d]. */
int ecc_corner_pack(ecc_ctx *ctx, const ecc_corner *in, const int32_t *counts, int32_t n_slices,
                    int32_t cap, ecc_corner *out, int64_t *offsets, ecc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * 5. Corner tracker (damped predictor-corrector + grouping)
 * Reference: class CornerTracker FCT/…group_track.cpp:163-537 (updateTrackedCorners
 *            :421-530, predictPosition :304-319, calculateDirection :233-271,
 *            estimateVelocity :273-302, updateCornerGroups :321-398), constructed with
 *            (30, 30, 10, 5, 0.8, 0.3, 100) at :805-813.  fp32 arithmetic in the
 *            reference's operation order; miss path truncates to int (Q16).
 * A tracker lives on the device; ecc_tracker_update consumes n_slices NMS outputs in order
 * (one updateTrackedCorners call per slice) in a single launch.  A slice's working set is
 * held in LDS, so max_tracks <= ECC_TRACKER_MAX_TRACKS and max_detections <=
 * ECC_TRACKER_MAX_DETECTIONS (ECC_ERR_INVALID otherwise); tracks or detections beyond
 * the tracker's capacities are dropped and reported as ECC_ERR_CAPACITY.
 * ------------------------------------------------------------------------------------- */
#define ECC_TRACK_HIST_MAX 16
#define ECC_TRACKER_MAX_TRACKS 4096
#define ECC_TRACKER_MAX_DETECTIONS 4096

typedef struct ecc_tracker_cfg {
    float max_distance;     /* 30 */
    int32_t max_frames;     /* 30 */
    int32_t history_size;   /* 10 (<= ECC_TRACK_HIST_MAX) */
    int32_t frames_to_skip; /* 5 */
    float damping;          /* 0.8 */
    float smoothing;        /* 0.3 */
    float group_radius;     /* 100 */
} ecc_tracker_cfg;

typedef struct ecc_track { /* reference struct TrackedCorner (:177-190) */
    int32_t x, y, label, frame_count;
    int32_t is_matched, frames_since_last_detection;
    int32_t hist_len;
    int32_t hist_x[ECC_TRACK_HIST_MAX], hist_y[ECC_TRACK_HIST_MAX]; /* [0] = most recent */
    float vx, vy;
    float dir_cur_x, dir_cur_y, dir_tgt_x, dir_tgt_y;
    int32_t group_id;
} ecc_track;

typedef struct ecc_group { /* reference struct CornerGroup (:193-199), keyed by group id */
    int32_t id, n_labels, first_label_offset; /* labels in ecc_tracker_get_groups' label array */
    float avg_vx, avg_vy, cx, cy, radius;
} ecc_group;

typedef struct ecc_tracker ecc_tracker;

void ecc_tracker_cfg_default(ecc_tracker_cfg *cfg);
int ecc_tracker_create(ecc_ctx *ctx, const ecc_tracker_cfg *cfg, int32_t max_tracks,
                       int32_t max_detections, ecc_tracker **out);
int ecc_tracker_destroy(ecc_tracker *tr);
int ecc_tracker_update(ecc_tracker *tr, const ecc_corner *corners, const int32_t *counts,
                       int32_t n_slices, int32_t cap, ecc_stream_t stream);
/* The same over explicit lists: slice s = corners[starts[s] .. starts[s] + counts[s]) (DEVICE
 * int64 starts, int32 counts), e.g. ecc_corner_pack outputs of several shards gathered in global
 * slice order (the multi-GPU track merge).  Counts above max_detections: ECC_ERR_CAPACITY. */
int ecc_tracker_update_lists(ecc_tracker *tr, const ecc_corner *corners, const int64_t *starts,
                             const int32_t *counts, int32_t n_slices, ecc_stream_t stream);
/* Host copies of the current state (synchronises stream). */
int ecc_tracker_get_tracks(ecc_tracker *tr, ecc_track *out, int32_t cap, int32_t *n_out,
                           ecc_stream_t stream);
int ecc_tracker_get_groups(ecc_tracker *tr, ecc_group *out, int32_t cap, int32_t *n_out,
                           int32_t *labels, int32_t labels_cap, ecc_stream_t stream);
/* 0 = OK, otherwise an ecc_status (capacity overflow inside the device loop). */
int ecc_tracker_status(ecc_tracker *tr, ecc_stream_t stream);
/* Checkpoint / restore and rank->rank hand-over of the tracker state (the reference's
 * CornerTracker is a copyable value, FCT/…group_track.cpp:163-199): the next label a new track
 * gets, and a replacement track list (HOST tracks, e.g. from ecc_tracker_get_tracks) with that
 * next label.  After set_tracks, updates continue exactly as the tracker the state came from;
 * the groups read as empty until the next update rebuilds them (:321-398).  Synchronous.
 * n > max_tracks: ECC_ERR_CAPACITY. */
int ecc_tracker_next_label(ecc_tracker *tr, int32_t *next_label, ecc_stream_t stream);
int ecc_tracker_set_tracks(ecc_tracker *tr, const ecc_track *tracks, int32_t n, int32_t next_label,
                           ecc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * 6. eps-neighbourhoods for DBSCAN / OPTICS over 2-D integer points (pixels)
 * Reference: DBSCANSimpleCluster::radiusSearch PCC/DBSCAN_simple.h:118-142 and
 *            DBSCANPrecompCluster::precomp PCC/DBSCAN_precomp.h:22-44 (d^2 <= eps^2 in double,
 *            self included); kdt::KDTree::radius_search OPT/include/optics/kdTree.hpp:307-422;
 *            optics::compute_core_dist OPT/include/optics/optics.hpp:286-299.
 * Points are packed u16 xy, segmented like ecc_kmeans_run_xy16 (one independent
 * neighbourhood problem per segment, <= 16384 points each, e.g. one downsample window);
 * duplicates allowed.  Arrays are indexed by the flattened point index p = s*seg_stride + j
 * (entries with j >= seg_counts[s] are left untouched, except offsets which stay monotone).
 *   counts[p]    = |{j in seg : (xi-xj)^2 + (yi-yj)^2 <= eps^2}| (self included);
 *   core_dist[p] = sqrt of the (min_pts-1)-th smallest d^2 of that set (fp64), or -1 when
 *                  counts[p] < min_pts (optics.hpp:292-298).  NULL to skip.
 * ecc_eps_lists: offsets[n_segs*seg_stride + 1] = exclusive scan of counts (computed here);
 *   nbr[offsets[p] .. offsets[p+1]) = segment-local neighbour indices in ascending order
 *   (the order of DBSCAN_precomp.h's adjacency lists).  ECC_ERR_CAPACITY if nbr_cap is too
 *   small (call ecc_eps_counts + read offsets' last entry to size it).
 * ------------------------------------------------------------------------------------- */
int ecc_eps_counts(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                   const int32_t *seg_counts, double eps, int32_t min_pts, int32_t *counts,
                   double *core_dist, ecc_stream_t stream);
int ecc_eps_lists(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                  const int32_t *seg_counts, double eps, const int32_t *counts, int64_t *offsets,
                  int32_t *nbr, int64_t nbr_cap, ecc_stream_t stream);
/* Host helper: synchronises `stream`, returns offsets[n] (total list length) via *total. */
int ecc_eps_total(ecc_ctx *ctx, const int64_t *offsets, int64_t n, int64_t *total,
                  ecc_stream_t stream);

/* Radius neighbourhoods of ONE fp64 (or fp32) point set of any size in 1-3 dimensions (the OPTICS
 * library's radius search, §8a rows a11-a12, beyond the int 2-D windows above).
 * Reference: kdt::KDTree::radius_search OPT/include/optics/kdTree.hpp:407-422 (keep i iff
 *   square_distance(points[i], p) <= radius*radius, square_distance = sum of d*d in double with
 *   d = p1[i] - p2[i], :180-192; self included); optics::compute_core_dist optics.hpp:286-299.
 * pts: DEVICE double[n*dim] row-major.  counts[i] = |ball(i)|; core_dist[i] = sqrt of the
 * (min_pts-1)-th smallest squared distance in the ball, or -1 below min_pts (NULL to skip).
 * ecc_radius_lists_f64: offsets[n+1] = exclusive scan of counts (computed here); with nbr ==
 * NULL only the offsets (offsets[n] = entries needed); else nbr[offsets[i]..offsets[i+1]) = the
 * ball's indices in grid order (the OPTICS expansion does not depend on it) and, when nbr_dist
 * is not NULL, their distances sqrt(square_distance) (geom::dist, optics.hpp:326);
 * ecc_radius_status reports ECC_ERR_CAPACITY if nbr_cap was too small.  Deterministic counts
 * and core distances. */
int ecc_radius_counts_f64(ecc_ctx *ctx, const double *pts, int64_t n, int32_t dim, double eps,
                          int32_t min_pts, int32_t *counts, double *core_dist, ecc_stream_t stream);
int ecc_radius_lists_f64(ecc_ctx *ctx, const double *pts, int64_t n, int32_t dim, double eps,
                         const int32_t *counts, int64_t *offsets, int32_t *nbr, double *nbr_dist,
                         int64_t nbr_cap, ecc_stream_t stream);
/* fp32 points (pcl::PointXYZ fields; DBSCAN_simple.h:132-135 / DBSCAN_precomp.h:31-34): the
 * per-axis difference is taken in float, then widened: d^2 = dx*dx + dy*dy + dz*dz in double.
 * Same outputs as the f64 forms; ecc_radius_lists_f32 is DBSCANPrecompCluster::precomp's
 * adjacency (ecc_lists_sort_ascending gives its row order). */
int ecc_radius_counts_f32(ecc_ctx *ctx, const float *pts, int64_t n, int32_t dim, double eps,
                          int32_t min_pts, int32_t *counts, double *core_dist, ecc_stream_t stream);
int ecc_radius_lists_f32(ecc_ctx *ctx, const float *pts, int64_t n, int32_t dim, double eps,
                         const int32_t *counts, int64_t *offsets, int32_t *nbr, double *nbr_dist,
                         int64_t nbr_cap, ecc_stream_t stream);
/* min_pts has no upper bound (compute_core_dist has none): above 64 the core distance comes from
 * a per-point radix select.  ECC_ERR_CAPACITY: nbr_cap too small; ECC_ERR_INVALID: a non-finite
 * coordinate in the last call's points. */
int ecc_radius_status(ecc_ctx *ctx, ecc_stream_t stream);
/* Sorts every list nbr[offsets[i] .. offsets[i+1]) (i < n) ascending in place (nbr_dist, when not
 * NULL, permuted alongside): the row order of DBSCAN_precomp.h:22-44's adjacency.  total =
 * offsets[n] (host value). */
int ecc_lists_sort_ascending(ecc_ctx *ctx, int64_t n, const int64_t *offsets, int64_t total,
                             int32_t *nbr, double *nbr_dist, ecc_stream_t stream);

/* OPTICS ordering (optics::compute_reachability_dists, optics.hpp:413-565): HOST pts[n*dim]
 * (dim 1-3) in; the GPU radius search above, then the ordered seed-set expansion on the host.
 * eps <= 0: epsilon_estimation (:369-387).  order[i] = point index of the i-th ordered point,
 * reach[i] = its reachability (-1 undefined).  Synchronises `stream`. */
int ecc_optics_f64(ecc_ctx *ctx, const double *pts, int64_t n, int32_t dim, int32_t min_pts, double eps,
                   int64_t *order, double *reach, ecc_stream_t stream);

/* DBSCAN cluster extraction over the eps-lists.
 * Reference: DBSCANSimpleCluster::extract PCC/DBSCAN_simple.h:27-90 (seed-queue expansion in
 *   point order, clusters kept when min_cluster_size <= size <= max_cluster_size, each
 *   cluster's indices sorted, clusters sorted by size descending :89; equal sizes: by first
 *   index, then creation order — the reference's std::sort leaves ties unspecified).
 * Consumes ecc_eps_lists' offsets / nbr for the same segments (core <=> count >= min_pts).
 * The seed-queue result is computed without the queue: clusters are the core-connected
 * components (union-find), created in order of their smallest core index (= the seed); a
 * border point joins the first cluster with a core neighbour AND every later cluster whose
 * seed is its neighbour (the seed's neighbours are queued unconditionally, :43-48).
 * Outputs per point p (flattened s*seg_stride + j, j < seg_counts[s]):
 *   labels[p] = index within segment s's output list of the cluster that claimed p first, or
 *               -1 (noise, or that cluster was filtered out by size);
 * n_clusters[s] = clusters kept for segment s;
 * dups[2*i], dups[2*i+1] = (p, cluster index) for every further membership (unordered),
 *   *n_dups (device int64) = their number; only dup_cap pairs are written.
 * nbr_len = entries of nbr (a segment whose offsets run past it is rejected, not read).
 * ecc_dbscan_status: ECC_ERR_CAPACITY if dups overflowed, a segment had more than 4096
 * core-connected components, or its lists exceed nbr_len (that segment's labels are then
 * all -1 and n_clusters 0); ECC_ERR_INVALID if a list entry lies outside [0, seg_counts[s])
 * (the entry is ignored; the segment's result is then unspecified). */
int ecc_dbscan_extract(ecc_ctx *ctx, int64_t n_segs, int64_t seg_stride, const int32_t *seg_counts,
                       const int64_t *offsets, const int32_t *nbr, int64_t nbr_len, int32_t min_pts,
                       int32_t min_cluster_size, int32_t max_cluster_size, int32_t *labels,
                       int32_t *n_clusters, int64_t *dups, int64_t dup_cap, int64_t *n_dups,
                       ecc_stream_t stream);
/* ecc_dbscan_grid: the same extraction (same outputs, same status) straight from the points,
 * with no neighbour lists: the segment is binned into an LDS cell grid and every phase walks the
 * 3x3 cells around a point (exact integer eps test, as ecc_eps_counts).  This is the whole of
 * DBSCANSimpleCluster::extract (:27-90) including its radiusSearch (:118-142) in one launch.
 * seg_stride <= 8192 (one downsample window). */
int ecc_dbscan_grid(ecc_ctx *ctx, const uint32_t *xy, int64_t n_segs, int64_t seg_stride,
                    const int32_t *seg_counts, double eps, int32_t min_pts, int32_t min_cluster_size,
                    int32_t max_cluster_size, int32_t *labels, int32_t *n_clusters, int64_t *dups,
                    int64_t dup_cap, int64_t *n_dups, ecc_stream_t stream);
int ecc_dbscan_status(ecc_ctx *ctx, ecc_stream_t stream);

/* DBSCAN over ONE point cloud of any size in 1-3 dimensions: DBSCANSimpleCluster::extract
 * (PCC/DBSCAN_simple.h:27-90) with its radiusSearch (:118-142) on the reference's own input type,
 * a float pcl::PointXYZ cloud (ecc_dbscan_cloud_f32, dim 3 = x,y,z; the differences in float as
 * ecc_radius_counts_f32) — or fp64 points (ecc_dbscan_cloud_f64).  The driver's parameters:
 * eps 20, min_pts 20, sizes 100..25000 (PCC/pcl_cluster.cpp:112-123).  pts: DEVICE row-major
 * [n*dim].  A negative eps acts as |eps| (radius_square = radius*radius, :127).  Outputs as
 * ecc_dbscan_extract for a single segment: labels[n] (cluster index in output order or -1),
 * *n_clusters (device int32), dups / *n_dups (device) further memberships.  No size cap and no
 * component cap (global union-find, clusters ordered by a device radix sort).
 * ecc_dbscan_cloud_status: ECC_ERR_CAPACITY if dups overflowed (*n_dups holds the number needed),
 * ECC_ERR_INVALID if a coordinate was not finite. */
int ecc_dbscan_cloud_f32(ecc_ctx *ctx, const float *pts, int64_t n, int32_t dim, double eps,
                         int32_t min_pts, int32_t min_cluster_size, int32_t max_cluster_size,
                         int32_t *labels, int32_t *n_clusters, int64_t *dups, int64_t dup_cap,
                         int64_t *n_dups, ecc_stream_t stream);
int ecc_dbscan_cloud_f64(ecc_ctx *ctx, const double *pts, int64_t n, int32_t dim, double eps,
                         int32_t min_pts, int32_t min_cluster_size, int32_t max_cluster_size,
                         int32_t *labels, int32_t *n_clusters, int64_t *dups, int64_t dup_cap,
                         int64_t *n_dups, ecc_stream_t stream);
int ecc_dbscan_cloud_status(ecc_ctx *ctx, ecc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * 7. Host-side helpers (no GPU): synthetic event streams and event-file I/O.
 * Reference ingress is Metavision's Camera::from_file(argv[1]) (FCT/…group_track.cpp:756-760);
 * here: CSV "x,y,t,p" (OPT/test/event_raw_data8.csv layout) or the binary SoA .ecc file.
 * ------------------------------------------------------------------------------------- */
typedef struct ecc_gen_cfg {
    uint64_t seed;
    int32_t width, height;
    double rate_mev_s;     /* events per µs of sensor time (10 = 10 Mev/s) */
    int64_t t0;            /* first timestamp (µs) */
    int32_t n_polygons;    /* 8 moving convex polygons (70 % of events) */
    int32_t n_blobs;       /* 16 Gaussian blobs sigma 4 (20 %) */
    float frac_edges, frac_blobs; /* remaining = uniform noise */
} ecc_gen_cfg;

void ecc_gen_cfg_default(ecc_gen_cfg *cfg);
/* Fills host arrays (any may be NULL) with events [first, first+n) of the stream. */
int ecc_gen_events(const ecc_gen_cfg *cfg, int64_t first, int64_t n, uint32_t *xy, int64_t *t,
                   uint8_t *p);
/* CSV reader: returns the number of events read (<= cap) or a negative status. */
int64_t ecc_read_csv(const char *path, uint32_t *xy, int64_t *t, uint8_t *p, int64_t cap);
int64_t ecc_count_csv(const char *path);

/* ---------------------------------------------------------------------------------------
 * 8. Event ingest: Prophesee/Metavision RAW files (EVT 2.0 / EVT 3.0) and the reslicer.
 * Reference: every host program opens its input with Metavision::Camera::from_file(argv[1])
 *   (FCT/…group_track.cpp:756-760, SMP/…opencl_store.cpp:336) and cuts the decoded stream
 *   with EventBufferReslicerAlgorithm make_n_events(16384) (FCT/…group_track.cpp:772-774) or
 *   make_n_us(50000) (DSA/…opencl_store.cpp:351).  Metavision/OpenEB is not vendored: the
 *   decoders restate the published EVT 2.0 / EVT 3.0 word formats,
 *   parity "unpinned" against OpenEB itself.
 *
 * A RAW file is an ASCII header of lines starting with '%' (ended by "% end" or by the first
 * line not starting with '%'), then little-endian words: u32 for EVT 2.0, u16 for EVT 3.0.
 * The format comes from "% evt 2.0|3.0" or "% format EVT2|EVT3;height=H;width=W"; the
 * geometry from "% geometry WxH" or the format line's width/height keys.
 * ------------------------------------------------------------------------------------- */
typedef enum ecc_raw_format { ECC_RAW_UNKNOWN = 0, ECC_RAW_EVT2 = 2, ECC_RAW_EVT3 = 3 } ecc_raw_format;

typedef struct ecc_raw_info {
    int32_t format;        /* ecc_raw_format */
    int32_t width, height; /* 0 when the header does not say */
    int32_t word_bytes;    /* 4 (EVT2) or 2 (EVT3) */
    int64_t header_bytes;  /* payload starts here */
    int64_t n_words;       /* whole words in the payload */
} ecc_raw_info;

/* Host: parses the header.  ECC_ERR_INVALID if unreadable or of an unsupported format. */
int ecc_raw_probe(const char *path, ecc_raw_info *info);
/* Host: reads payload words [first_word, first_word + n) into buf; returns words read or < 0. */
int64_t ecc_raw_read_words(const char *path, const ecc_raw_info *info, int64_t first_word,
                           int64_t n, void *buf);

/* Host: RAW writer — encodes events (x, y < 2048, non-decreasing t) into EVT 2.0 (u32) or
 * EVT 3.0 (u16) words; EVT 3.0 runs of >= 3 events with equal (t, y, p) and increasing x
 * within 12 px go out as VECT_BASE_X + VECT_12.  Returns the number of words (<= cap written)
 * or a negative status.  Word bound: EVT 2.0 2n + 1, EVT 3.0 4n + 2 * (t_last >> 24) + 4. */
int64_t ecc_evt_encode(int32_t format, const uint32_t *xy, const int64_t *t, const uint8_t *p, int64_t n,
                       void *out, int64_t cap);

/* Decoder carry state (device memory, ECC_EVT_STATE_BYTES, zeroed = stream start).  Passing
 * the same state to consecutive calls decodes a long recording in pieces exactly as if it
 * were one buffer; NULL = decode `words` as a complete stream. */
#define ECC_EVT_STATE_BYTES 64

/* GPU: decodes n_words device-resident words (format ECC_RAW_EVT2: const uint32_t*,
 * ECC_RAW_EVT3: const uint16_t*) into CD events in stream order:
 *   xy[i] = x | y << 16, t[i] = timestamp (µs), p[i] = polarity (0 = OFF, 1 = ON).
 * Event words carry 11-bit x/y; EVT 3.0 vector words expand to one event per set mask bit at
 * x = base + bit.  EVT 3.0 timestamps are 24-bit; each decrease of TIME_HIGH adds 2^24
 * (one loop).  Trigger / OTHERS / CONTINUED words produce no CD event.  Events before the
 * first TIME_HIGH word take time-high 0.
 * *n_out (device int64) = number of events in the buffer; only the first `cap` are written
 * (ecc_evt_status reports ECC_ERR_CAPACITY when n_out > cap).  Any of xy/t/p may be NULL. */
int ecc_evt_decode(ecc_ctx *ctx, int32_t format, const void *words, int64_t n_words, uint32_t *xy,
                   int64_t *t, uint8_t *p, int64_t cap, int64_t *n_out, void *state,
                   ecc_stream_t stream);
/* Host helper: synchronises `stream`; ECC_ERR_CAPACITY if the last decode on ctx truncated. */
int ecc_evt_status(ecc_ctx *ctx, ecc_stream_t stream);

/* GPU reslicer, n-µs condition (EventBufferReslicerAlgorithm::Condition::make_n_us):
 * slice k holds the events with t in [t_base + k*period_us, t_base + (k+1)*period_us), where
 * t_base = floor(t[0] / period_us) * period_us; bounds[k] = index of its first event
 * (bounds[n_slices] = n).  Slices without events are kept (empty ranges), as the reslicer
 * emits one on_new_slice per elapsed period.  t must be non-decreasing.
 * *n_slices (device int64) = ceil-count of periods spanned; bounds has max_slices + 1 entries
 * and only slices < max_slices are written (ECC_ERR_CAPACITY through ecc_evt_status).
 * The n-events condition (make_n_events(N)) needs no kernel: bounds[k] = min(k*N, n). */
int ecc_reslice_n_us(ecc_ctx *ctx, const int64_t *t, int64_t n, int64_t period_us,
                     int64_t *bounds, int64_t max_slices, int64_t *n_slices, ecc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * 9. Multi-GPU time-window shards over RCCL (xGMI) — SURVEY.md §8e, BASELINE config C5.
 * Reference: none (the reference is single-device); the exchanges restate its sequential slice
 *            loop FCT/…group_track.cpp:832-850 exactly.
 * One process per GPU; rank r owns the r-th time window of the stream (windows are multiples
 * of the 16384-event slice).  Rank 0 calls ecc_dist_get_unique_id and ships the 128 bytes to
 * the other ranks over any channel (pipe, file, socket, MPI); every rank then calls
 * ecc_dist_init with its own context (its GPU).  Collectives are enqueued on `stream` and
 * ordered with libecc's kernels; only ecc_dist_gather_corners synchronises `stream` (one
 * size exchange).  librccl is opened on first use (dlopen): ecc_dist_available() == 0 when it
 * cannot be, and ecc_dist_init then returns ECC_ERR_NO_DEVICE.
 * The sharded step (apps/ecc_sharded_step.cpp):
 *   ecc_downsample_hash -> ecc_kmeans_counts_xy16 -> ecc_dist_allreduce_counts ->
 *   ecc_kmeans_run_counts -> ecc_kmeans_labels_xy16            (global centroids, bit-exact)
 *   ecc_fast_detect_prepare -> ecc_dist_sae_handoff -> ecc_fast_detect_finish_nms (exact SAE)
 *   ecc_corner_pack -> ecc_dist_gather_corners -> (rank 0) ecc_tracker_update_lists
 * ------------------------------------------------------------------------------------- */
#define ECC_DIST_ID_BYTES 128
typedef struct ecc_dist ecc_dist;
int ecc_dist_available(void);
int ecc_dist_get_unique_id(uint8_t *id /* [ECC_DIST_ID_BYTES] */);
int ecc_dist_init(ecc_dist **out, ecc_ctx *ctx, const uint8_t *id, int32_t n_ranks, int32_t rank);
int ecc_dist_destroy(ecc_dist *d);
int ecc_dist_rank(const ecc_dist *d, int32_t *rank, int32_t *n_ranks);
/* k-means: in-place SUM over ranks of the per-pixel count images (DEVICE uint32[n],
 * ecc_kmeans_counts_xy16). */
int ecc_dist_allreduce_counts(ecc_dist *d, uint32_t *counts, int64_t n, ecc_stream_t stream);
/* In-place MAX over ranks of DEVICE doubles (e.g. per-rank step times). */
int ecc_dist_allreduce_f64_max(ecc_dist *d, double *values, int64_t n, ecc_stream_t stream);
/* SAE hand-off: all[n_ranks*hw] (DEVICE scratch) = every rank's local_last image
 * (ecc_fast_detect_prepare), then sae[hw] = element-wise max over ranks < this rank (zeros on
 * rank 0) = this shard's exact initial SAE for ecc_fast_detect_finish(_nms). */
int ecc_dist_sae_handoff(ecc_dist *d, const int64_t *local_last, int64_t hw, int64_t *all,
                         int64_t *sae, ecc_stream_t stream);
/* Track-merge exchange: packed/offsets = this rank's ecc_corner_pack output (n_slices slices).
 * On every rank: all[r * stride + i] = rank r's packed corner i (stride = the largest rank's
 * corner count, *corners_stride), and slice k of the global order (ranks in order) is
 * all[starts[k] .. starts[k] + counts[k]) (DEVICE int64 / int32 arrays, k < *n_slices_total)
 * — exactly the arguments of ecc_tracker_update_lists.  ECC_ERR_CAPACITY (with
 * *n_slices_total / *corners_stride set) if n_ranks * stride > all_cap or the slices exceed
 * slices_cap.  With all, starts and counts all NULL it only returns the sizes (the size
 * exchange is itself collective: every rank makes the same calls). */
int ecc_dist_gather_corners(ecc_dist *d, const ecc_corner *packed, const int64_t *offsets,
                            int32_t n_slices, ecc_corner *all, int64_t all_cap, int64_t *starts,
                            int32_t *counts, int64_t slices_cap, int64_t *n_slices_total,
                            int64_t *corners_stride, ecc_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* ECC_H */
