/* big_ipc.c -- the IPC engines on a bucket whose IPC buffer exceeds 2 GiB, in
 * a C process (which maps /opt/rocm's HSA runtime, where importing such a
 * buffer works; DESIGN.md "2 GiB per IPC export").  One process per rank, rank
 * 0 the TCP master, every rank on GPU 0 (RCCL refuses a shared GPU, so the
 * ranks agree on the p2p engine), exactly as host.c is run.
 *
 *   big_ipc <world> <rank> <elements> <engine: p2p|mesh>
 *
 * Inputs are exact in fixed point: x_r[i] = ((i % 4093) - 2046) / 1024 *
 * (r + 1), so the sum is ((i % 4093) - 2046) / 1024 * W(W+1)/2 exactly, and
 * every lane of two calls (the second with the inputs negated) is checked.
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "api.h"
#include "inccl_amd.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "rank %d: %s: %s\n", rank, #x, hipGetErrorString(e_)); return 2; } } while (0)

int main(int argc, char **argv)
{
    if (argc != 5) {
        fprintf(stderr, "usage: big_ipc <world> <rank> <elements> <engine>\n");
        return 9;
    }
    const int world = atoi(argv[1]), rank = atoi(argv[2]);
    const size_t n = (size_t)strtoull(argv[3], NULL, 0);
    const char *engine = argv[4];
    struct inccl_group *g = inccl_group_create(world, rank, "127.0.0.1");
    if (!g) {
        fprintf(stderr, "rank %d: group: %s\n", rank, inccl_last_error());
        return 3;
    }
    printf("rank %d: process IPC bound %zu bytes, group bound %zu bytes\n", rank, inccl_ipc_max_bytes(),
           inccl_group_ipc_max_bytes(g));
    struct inccl_communicator *c = inccl_communicator_create(g, 0);
    if (!c || inccl_comm_set_engine(c, engine) != INCCL_OK) {
        fprintf(stderr, "rank %d: communicator / engine %s: %s\n", rank, engine, inccl_last_error());
        return 4;
    }
    float *h = (float *)malloc(n * sizeof(float));
    float *d_in = NULL, *d_out = NULL;
    if (!h) return 5;
    CK(hipMalloc((void **)&d_in, n * sizeof(float)));
    CK(hipMalloc((void **)&d_out, n * sizeof(float)));
    const float tri = (float)(world * (world + 1) / 2);
    int bad_calls = 0;
    for (int call = 0; call < 2; ++call) {
        const float sign = call ? -1.0f : 1.0f;
        for (size_t i = 0; i < n; ++i) h[i] = sign * (float)((int)(i % 4093) - 2046) / 1024.0f * (float)(rank + 1);
        CK(hipMemcpy(d_in, h, n * sizeof(float), hipMemcpyHostToDevice));
        const float *bufs[1] = {d_in};
        int rc = inccl_allreduce_f32(c, bufs, 1, d_out, n, 25, NULL);
        if (rc == INCCL_OK) CK(hipStreamSynchronize((hipStream_t)inccl_comm_stream(c)));
        if (rc != INCCL_OK) {
            fprintf(stderr, "rank %d: call %d: %s\n", rank, call, inccl_last_error());
            return 6;
        }
        CK(hipMemcpy(h, d_out, n * sizeof(float), hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < n; ++i)
            bad += h[i] != sign * (float)((int)(i % 4093) - 2046) / 1024.0f * tri;
        printf("rank %d: engine %s, %zu elements (%zu-byte IPC buffer), call %d: %zu bad lanes\n", rank, engine, n,
               n * sizeof(int32_t), call, bad);
        bad_calls += bad != 0;
    }
    free(h);
    hipFree(d_in);
    hipFree(d_out);
    inccl_communicator_destroy(c);
    inccl_group_destroy(g);
    if (bad_calls) return 7;
    printf("result ok\n");
    return 0;
}
