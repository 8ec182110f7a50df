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
 */
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
        fprintf(stderr, "usage: ref_harness downsample|assign <co> <in> [...] <out>\n");
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
    } else {
        fprintf(stderr, "unknown mode %s\n", argv[1]);
        return 2;
    }
    return 0;
}
