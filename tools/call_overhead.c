/* call_overhead.c -- where the time of a small eager fused reduce goes, from C:
 * back-to-back calls of inccl_reduce_f32 (R = 2, fixed scale) and of a
 * prepared op (inccl_op_run) on one stream, host wall time per call (the
 * stream is synchronised once at the end), against an empty HIP kernel
 * launched the same way (hipLaunchKernel's floor, from tools/tune/tune_small).
 * One JSON line per bucket size.  Run under `rocprofv3 --hip-trace
 * --kernel-trace --stats` to split each call into HIP API time and kernel time.
 * Build (tools/gpu_call_overhead.sh):
 *   gcc -O2 -std=c11 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude tools/call_overhead.c \
 *       -Lcontainer_inc_amd -linccl_amd -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,... -o tools/call_overhead */
#define _GNU_SOURCE
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "inccl_amd.h"

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

#define CHECK(x)                                                                  \
    do {                                                                          \
        if ((x) != 0) {                                                           \
            fprintf(stderr, "%s:%d: %s (%s)\n", __FILE__, __LINE__, #x, inccl_last_error()); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    const size_t sizes[] = {4u << 10, 64u << 10, 1u << 20, 4u << 20};
    hipStream_t st;
    CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (size_t si = 0; si < sizeof(sizes) / sizeof(sizes[0]); ++si) {
        const size_t n = sizes[si] / 4;
        float *x0, *x1, *y;
        CHECK(hipMalloc((void **)&x0, n * 4));
        CHECK(hipMalloc((void **)&x1, n * 4));
        CHECK(hipMalloc((void **)&y, n * 4));
        CHECK(hipMemset(x0, 0, n * 4));
        CHECK(hipMemset(x1, 0, n * 4));
        const float *srcs[2] = {x0, x1};
        struct inccl_op *op = inccl_op_create(INCCL_KIND_F32, INCCL_KIND_F32, (const void *const *)srcs, 2, y, n, 25, 2, st);
        if (!op) {
            fprintf(stderr, "inccl_op_create: %s\n", inccl_last_error());
            return 1;
        }
        double t_call = 0, t_op = 0;
        for (int pass = 0; pass < 2; ++pass) {   /* pass 0 warms up */
            CHECK(hipStreamSynchronize(st));
            double t0 = now_s();
            for (int i = 0; i < iters; ++i) CHECK(inccl_reduce_f32(srcs, 2, y, n, 25, st));
            CHECK(hipStreamSynchronize(st));
            t_call = (now_s() - t0) / iters;
            t0 = now_s();
            for (int i = 0; i < iters; ++i) CHECK(inccl_op_run(op));
            CHECK(hipStreamSynchronize(st));
            t_op = (now_s() - t0) / iters;
        }
        printf("{\"bucket_bytes\": %zu, \"R\": 2, \"c_call_us\": %.3f, \"c_prepared_us\": %.3f, \"iters\": %d}\n",
               sizes[si], t_call * 1e6, t_op * 1e6, iters);
        fflush(stdout);
        inccl_op_destroy(op);
        hipFree(x0);
        hipFree(x1);
        hipFree(y);
    }
    hipStreamDestroy(st);
    return 0;
}
