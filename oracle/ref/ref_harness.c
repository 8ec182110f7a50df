/* OpenCL host harness for the reference kernels — TEST INFRASTRUCTURE ONLY.
 *
 * Runs the reference's own, unmodified OpenCL kernels (compiled from /root/reference by
 * oracle/ref/Makefile into the oracle/_ref code objects) on the GPU box's OpenCL device, the way the
 * reference hosts launch them, and writes the raw outputs for tests/test_ref_opencl.py:
 *
 *   ref_harness downsample <co> <in.i32> <out.i32> [lanes]
 *       process_coordinates (coordinate_processor.cl:16-89) as in SMP/…opencl_store.cpp:
 *       297-326: ONE work-group, total_coords = number of (x,y) pairs, width 1280, height 720.
 *       in: int32 pairs x,y.  out: [unique_count, repeated_count, unique_coords[2*unique]].
 *       The single work-group has `lanes` lanes (default 64 = one wave).  The reference
 *       launches 1024, but its lane 0 adds the LDS counters to the globals with no barrier
 *       (:80-81 commented out), so with more than one wave the counts race (quirk Q21);
 *       with one wave they are final.  The unique_coords buffer is pre-filled with -1.
 *   ref_harness assign <co> <in.f32> <centers.f32> <out.i32>
 *       assign_to_centers (assign_to_centers.cl:1-34): in = float x,y pairs (padded by the
 *       caller to a multiple of 256 points), centers = 8 (x,y); out = assignments (2c or 255).
 *   ref_harness kmeans_loop <co> <max_passes> <out.bin>
 *       The three kernels of assign_to_centers.cl in the pass loop of KM/assign_to_centers2.c
 *       (:184-548; that program itself reads the .cl SOURCE at run time, :2/:61, so it cannot
 *       run where the reference is absent): the demo data data[i] = i % 100 (:123-129), the demo
 *       centroids (:131), output zeroed once (:133-137) and re-uploaded from the previous
 *       readback every pass (:195, :348), cluster_index zeroed per pass (:186-188),
 *       assign_to_centers / assign_data_cluster over 2048 points (:233, :318),
 *       reduction_scalar over 32768 floats -> 32 sums of 1024 (:404-455); then the
 *       reference's host update restated (:505-548: the y_offset index, C int abs() on
 *       float, the running-max update, restart while error_max > 10).  out: int32 passes, then
 *       per pass int32 cluster_index[8], float scalar_sum[32], new_centroids[16],
 *       centroids[16] (after the update), then per pass the output buffer read back after
 *       assign_data_cluster (float[32768]: the bins with the stale tails the next pass keeps).
 *       Work-groups are 256 lanes, not the reference's 1024: clang compiles an OpenCL kernel
 *       without a work-group-size attribute for at most 256 lanes (ROCm's OpenCL device also
 *       reports 256), and the sources may not be edited.  assign_to_centers and
 *       assign_data_cluster index by global id only; reduction_scalar is size-generic, so its
 *       128 sums of 256 are added four at a time into the reference's 32 sums of 1024 — exact
 *       here, since the demo data are integer-valued floats far below 2^24.
 */
#include <math.h>
#define CL_TARGET_OPENCL_VERSION 200
#include <CL/cl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void die(const char *what, cl_int err) {
    fprintf(stderr, "ref_harness: %s failed (%d)\n", what, (int)err);
    exit(1);
}

static void *slurp(const char *path, size_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    fseek(f, 0, SEEK_END);
    *len = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    void *buf = malloc(*len ? *len : 1);
    if (*len && fread(buf, 1, *len, f) != *len) { perror("fread"); exit(1); }
    fclose(f);
    return buf;
}

static void spit(const char *path, const void *p, size_t len) {
    FILE *f = fopen(path, "wb");
    if (!f || fwrite(p, 1, len, f) != len) { perror(path); exit(1); }
    fclose(f);
}

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: ref_harness downsample|assign|kmeans_loop <co> <in> [...] <out>\n");
        return 2;
    }
    cl_int err;
    cl_platform_id plat;
    cl_device_id dev;
    if ((err = clGetPlatformIDs(1, &plat, NULL)) != CL_SUCCESS) die("clGetPlatformIDs", err);
    if ((err = clGetDeviceIDs(plat, CL_DEVICE_TYPE_GPU, 1, &dev, NULL)) != CL_SUCCESS) die("clGetDeviceIDs", err);
    cl_context ctx = clCreateContext(NULL, 1, &dev, NULL, NULL, &err);
    if (err) die("clCreateContext", err);
    cl_command_queue q = clCreateCommandQueueWithProperties(ctx, dev, NULL, &err);
    if (err) die("clCreateCommandQueue", err);
    size_t blen;
    unsigned char *bin = slurp(argv[2], &blen);
    const unsigned char *bins[1] = {bin};
    cl_int bstat;
    cl_program prog = clCreateProgramWithBinary(ctx, 1, &dev, &blen, bins, &bstat, &err);
    if (err) die("clCreateProgramWithBinary", err);
    if ((err = clBuildProgram(prog, 1, &dev, "", NULL, NULL)) != CL_SUCCESS) die("clBuildProgram", err);

    if (!strcmp(argv[1], "downsample")) {
        size_t ilen;
        int *in = slurp(argv[3], &ilen);
        const int pairs = (int)(ilen / 8);
        cl_kernel k = clCreateKernel(prog, "process_coordinates", &err);
        if (err) die("clCreateKernel", err);
        int zero = 0;
        cl_mem bin_ = clCreateBuffer(ctx, CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR, ilen ? ilen : 8, in, &err);
        cl_mem brep = clCreateBuffer(ctx, CL_MEM_READ_WRITE, 16384 * sizeof(int), NULL, &err);
        int *init = malloc(2 * 8192 * sizeof(int));
        for (int i = 0; i < 2 * 8192; ++i) init[i] = -1;
        cl_mem buni = clCreateBuffer(ctx, CL_MEM_READ_WRITE | CL_MEM_COPY_HOST_PTR, 2 * 8192 * sizeof(int), init, &err);
        cl_mem brc = clCreateBuffer(ctx, CL_MEM_READ_WRITE | CL_MEM_COPY_HOST_PTR, sizeof(int), &zero, &err);
        cl_mem buc = clCreateBuffer(ctx, CL_MEM_READ_WRITE | CL_MEM_COPY_HOST_PTR, sizeof(int), &zero, &err);
        if (err) die("clCreateBuffer", err);
        int w = 1280, h = 720;
        clSetKernelArg(k, 0, sizeof(cl_mem), &bin_);
        clSetKernelArg(k, 1, sizeof(cl_mem), &brep);
        clSetKernelArg(k, 2, sizeof(cl_mem), &buni);
        clSetKernelArg(k, 3, sizeof(cl_mem), &brc);
        clSetKernelArg(k, 4, sizeof(cl_mem), &buc);
        clSetKernelArg(k, 5, sizeof(int), &pairs);
        clSetKernelArg(k, 6, sizeof(int), &w);
        clSetKernelArg(k, 7, sizeof(int), &h);
        size_t g = argc > 5 ? (size_t)atoi(argv[5]) : 64, l = g;
        if ((err = clEnqueueNDRangeKernel(q, k, 1, NULL, &g, &l, 0, NULL, NULL)) != CL_SUCCESS) die("clEnqueueNDRangeKernel", err);
        clFinish(q);
        int counts[2];
        clEnqueueReadBuffer(q, buc, CL_TRUE, 0, sizeof(int), &counts[0], 0, NULL, NULL);
        clEnqueueReadBuffer(q, brc, CL_TRUE, 0, sizeof(int), &counts[1], 0, NULL, NULL);
        /* the whole coordinate buffer: entries past the final local counter stay -1 */
        int *out = malloc((2 + 2 * 8192) * sizeof(int));
        out[0] = counts[0];
        out[1] = counts[1];
        clEnqueueReadBuffer(q, buni, CL_TRUE, 0, 2 * 8192 * sizeof(int), out + 2, 0, NULL, NULL);
        spit(argv[4], out, (2 + 2 * 8192) * sizeof(int));
    } else if (!strcmp(argv[1], "assign")) {
        if (argc < 6) return 2;
        size_t ilen, clen;
        float *in = slurp(argv[3], &ilen);
        float *cen = slurp(argv[4], &clen);
        const size_t npts = ilen / 8;
        cl_kernel k = clCreateKernel(prog, "assign_to_centers", &err);
        if (err) die("clCreateKernel", err);
        cl_mem bd = clCreateBuffer(ctx, CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR, ilen, in, &err);
        cl_mem bc = clCreateBuffer(ctx, CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR, clen, cen, &err);
        cl_mem ba = clCreateBuffer(ctx, CL_MEM_READ_WRITE, npts * sizeof(int), NULL, &err);
        if (err) die("clCreateBuffer", err);
        clSetKernelArg(k, 0, sizeof(cl_mem), &bd);
        clSetKernelArg(k, 1, sizeof(cl_mem), &bc);
        clSetKernelArg(k, 2, sizeof(cl_mem), &ba);
        size_t g = npts, l = 256;
        if ((err = clEnqueueNDRangeKernel(q, k, 1, NULL, &g, &l, 0, NULL, NULL)) != CL_SUCCESS) die("clEnqueueNDRangeKernel", err);
        clFinish(q);
        int *out = malloc(npts * sizeof(int));
        clEnqueueReadBuffer(q, ba, CL_TRUE, 0, npts * sizeof(int), out, 0, NULL, NULL);
        spit(argv[5], out, npts * sizeof(int));
    } else if (!strcmp(argv[1], "kmeans_loop")) {
        enum { N = 4096 };
        const int max_passes = atoi(argv[3]);
        static float data[N], output[N * 8], out_rec[64 * 72], out_buf[64][N * 8];
        for (int i = 0; i < N; ++i) data[i] = (float)(i % 100);
        float centroids[16] = {1, 1, 10, 10, 20, 20, 30, 30, 50, 50, 60, 60, 70, 70, 80, 80};
        cl_kernel k1 = clCreateKernel(prog, "assign_to_centers", &err);
        if (err) die("clCreateKernel 1", err);
        cl_kernel k2 = clCreateKernel(prog, "assign_data_cluster", &err);
        if (err) die("clCreateKernel 2", err);
        cl_kernel k3 = clCreateKernel(prog, "reduction_scalar", &err);
        if (err) die("clCreateKernel 3", err);
        cl_mem bd = clCreateBuffer(ctx, CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR, sizeof(data), data, &err);
        if (err) die("clCreateBuffer data", err);
        int passes = 0;
        for (;;) {
            int cluster_index[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            unsigned int assign[N / 2];
            memset(assign, 0, sizeof(assign));
            float scalar_sum[32], part[128];
            cl_mem bc = clCreateBuffer(ctx, CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR, sizeof(centroids), centroids, &err);
            cl_mem ba = clCreateBuffer(ctx, CL_MEM_READ_WRITE | CL_MEM_COPY_HOST_PTR, sizeof(assign), assign, &err);
            cl_mem bo = clCreateBuffer(ctx, CL_MEM_READ_WRITE | CL_MEM_COPY_HOST_PTR, sizeof(output), output, &err);
            cl_mem bi = clCreateBuffer(ctx, CL_MEM_READ_WRITE | CL_MEM_COPY_HOST_PTR, sizeof(cluster_index), cluster_index, &err);
            cl_mem bs = clCreateBuffer(ctx, CL_MEM_READ_WRITE, sizeof(part), NULL, &err);
            if (err) die("clCreateBuffer pass", err);
            size_t g = N / 2, l = 256;
            clSetKernelArg(k1, 0, sizeof(cl_mem), &bd);
            clSetKernelArg(k1, 1, sizeof(cl_mem), &bc);
            clSetKernelArg(k1, 2, sizeof(cl_mem), &ba);
            if ((err = clEnqueueNDRangeKernel(q, k1, 1, NULL, &g, &l, 0, NULL, NULL)) != CL_SUCCESS) die("assign_to_centers", err);
            clSetKernelArg(k2, 0, sizeof(cl_mem), &bd);
            clSetKernelArg(k2, 1, sizeof(cl_mem), &ba);
            clSetKernelArg(k2, 2, sizeof(cl_mem), &bi);
            clSetKernelArg(k2, 3, sizeof(cl_mem), &bo);
            if ((err = clEnqueueNDRangeKernel(q, k2, 1, NULL, &g, &l, 0, NULL, NULL)) != CL_SUCCESS) die("assign_data_cluster", err);
            clFinish(q);
            clEnqueueReadBuffer(q, bo, CL_TRUE, 0, sizeof(output), output, 0, NULL, NULL);
            clEnqueueReadBuffer(q, bi, CL_TRUE, 0, sizeof(cluster_index), cluster_index, 0, NULL, NULL);
            memcpy(out_buf[passes], output, sizeof(output));
            size_t g3 = (size_t)N * 8, l3 = 256;
            clSetKernelArg(k3, 0, sizeof(cl_mem), &bo);
            clSetKernelArg(k3, 1, l3 * sizeof(float), NULL);
            clSetKernelArg(k3, 2, sizeof(cl_mem), &bs);
            if ((err = clEnqueueNDRangeKernel(q, k3, 1, NULL, &g3, &l3, 0, NULL, NULL)) != CL_SUCCESS) die("reduction_scalar", err);
            clFinish(q);
            clEnqueueReadBuffer(q, bs, CL_TRUE, 0, sizeof(part), part, 0, NULL, NULL);
            for (int j = 0; j < 32; ++j)
                scalar_sum[j] = (part[4 * j] + part[4 * j + 1]) + (part[4 * j + 2] + part[4 * j + 3]);
            clReleaseMemObject(bc); clReleaseMemObject(ba); clReleaseMemObject(bo);
            clReleaseMemObject(bi); clReleaseMemObject(bs);
            float nc[16], error[16], error_max = 0.0f;
            for (int j = 0; j < 16; j += 2) {
                nc[j] = (scalar_sum[j] + scalar_sum[j + 1]) / cluster_index[j / 2];
                nc[j + 1] = (scalar_sum[j + 2] + scalar_sum[j + 3]) / cluster_index[j / 2];
            }
            for (int j = 0; j < 16; ++j) error[j] = nc[j] - centroids[j];
            for (int j = 0; j < 16; ++j) {
                if (abs((int)error[j]) > error_max) {  /* C int abs() of a float argument */
                    error_max = (float)abs((int)error[j]);
                    centroids[j] = nc[j];
                }
            }
            float *rec = out_rec + 72 * passes;
            memcpy(rec, cluster_index, 8 * 4);
            memcpy(rec + 8, scalar_sum, 32 * 4);
            memcpy(rec + 40, nc, 16 * 4);
            memcpy(rec + 56, centroids, 16 * 4);
            ++passes;
            if (!(error_max > 10) || passes >= max_passes || passes >= 64) break;
        }
        FILE *f = fopen(argv[4], "wb");
        if (!f) { perror(argv[4]); return 1; }
        fwrite(&passes, 4, 1, f);
        fwrite(out_rec, 4, (size_t)72 * passes, f);
        for (int p = 0; p < passes; ++p) fwrite(out_buf[p], 4, (size_t)N * 8, f);
        fclose(f);
    } else {
        fprintf(stderr, "unknown mode %s\n", argv[1]);
        return 2;
    }
    return 0;
}
