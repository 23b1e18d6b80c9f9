/* host_stress.c -- the host-memory entry points through the C ABI alone, on
 * buffers large enough for many pipeline chunks: inccl_allreduce_write on
 * pageable and on registered memory (api.c:403-452's path as host.c calls it,
 * plus the ibv_reg_mr analogue) and inccl_allreduce_f32_host on pageable
 * memory.  Meant to run under ASan/UBSan (tools/asan_host.sh) as well as
 * plainly.  Inputs are chosen so every result is exact and known in closed form.
 *
 *   host_stress <world_size> <master_ip|local> [rank] [elements] [calls]
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "inccl_amd.h"

struct rank_arg {
    int world, rank;
    const char *master;
    size_t n;
    int calls;
    long failures;
};

static int32_t in_q(size_t i, int rank) { return (int32_t)((i * 2654435761u) ^ (uint32_t)rank * 0x9E3779B9u); }

static void *run_rank(void *p)
{
    struct rank_arg *a = (struct rank_arg *)p;
    const size_t n = a->n, m = n / 1024 * 1024;   /* whole messages only (api.c:406) */
    int32_t *src = malloc(n * sizeof(int32_t)), *dst = malloc(n * sizeof(int32_t));
    float *xf = malloc(n * sizeof(float)), *yf = malloc(n * sizeof(float));
    if (!src || !dst || !xf || !yf) {
        a->failures = -1;
        return NULL;
    }
    for (size_t i = 0; i < n; ++i) {
        src[i] = in_q(i, a->rank);
        /* multiples of 2^-10 below 2^11: exact at k = 20, and their sums too */
        xf[i] = (float)((int)(i % 4093) - 2046) / 1024.0f * (float)(a->rank + 1);
    }
    struct inccl_group *g = strcmp(a->master, "local") == 0
                                ? inccl_group_create_local(a->world, a->rank, "host_stress", -1)
                                : inccl_group_create(a->world, a->rank, a->master);
    if (!g) {
        fprintf(stderr, "rank %d: group: %s\n", a->rank, inccl_last_error());
        a->failures = -1;
        return NULL;
    }
    struct inccl_communicator *c = inccl_communicator_create(g, 1 << 20);
    if (!c) {
        fprintf(stderr, "rank %d: communicator: %s\n", a->rank, inccl_last_error());
        a->failures = -1;
        return NULL;
    }
    for (int reg = 0; reg < 2; ++reg) {
        if (reg && (inccl_host_register(c, src, n * sizeof(int32_t)) || inccl_host_register(c, dst, n * sizeof(int32_t)))) {
            fprintf(stderr, "rank %d: host_register: %s\n", a->rank, inccl_last_error());
            a->failures++;
            break;
        }
        for (int call = 0; call < a->calls; ++call) {
            for (size_t i = 0; i < n; ++i) dst[i] = -7 - call;
            inccl_allreduce_write(c, src, (uint32_t)n, dst);
            for (size_t i = 0; i < m; ++i) {
                uint32_t want = 0;
                for (int r = 0; r < a->world; ++r) want += (uint32_t)in_q(i, r);
                if ((uint32_t)dst[i] != want) a->failures++;
            }
            for (size_t i = m; i < n; ++i)
                if (dst[i] != -7 - call) a->failures++;
        }
        if (reg) {
            inccl_host_deregister(c, src);
            inccl_host_deregister(c, dst);
        }
    }
    const float mult = (float)(a->world * (a->world + 1) / 2);
    for (int call = 0; call < a->calls; ++call) {
        for (size_t i = 0; i < n; ++i) yf[i] = -1.0f;
        if (inccl_allreduce_f32_host(c, xf, yf, n, 20, (size_t)3 << 20)) {
            fprintf(stderr, "rank %d: allreduce_f32_host: %s\n", a->rank, inccl_last_error());
            a->failures++;
            break;
        }
        for (size_t i = 0; i < n; ++i)
            if (yf[i] != (float)((int)(i % 4093) - 2046) / 1024.0f * mult) a->failures++;
    }
    inccl_communicator_destroy(c);
    inccl_group_destroy(g);
    free(src);
    free(dst);
    free(xf);
    free(yf);
    return NULL;
}

int main(int argc, char **argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s <world_size> <master_ip|local> [rank] [elements] [calls]\n", argv[0]);
        return 2;
    }
    const int world = atoi(argv[1]);
    const char *master = argv[2];
    const size_t n = argc > 4 ? (size_t)atoll(argv[4]) : (size_t)(9 << 22) + 1000;
    const int calls = argc > 5 ? atoi(argv[5]) : 3;
    long failures = 0;
    if (strcmp(master, "local") == 0) {
        pthread_t th[INCCL_MAX_LOCAL_INPUTS];
        struct rank_arg args[INCCL_MAX_LOCAL_INPUTS];
        if (world < 1 || world > INCCL_MAX_LOCAL_INPUTS) return 2;
        for (int r = 0; r < world; ++r) {
            args[r] = (struct rank_arg){world, r, master, n, calls, 0};
            pthread_create(&th[r], NULL, run_rank, &args[r]);
        }
        for (int r = 0; r < world; ++r) {
            pthread_join(th[r], NULL);
            failures += args[r].failures < 0 ? 1 : args[r].failures;
        }
    } else {
        struct rank_arg a = {world, argc > 3 ? atoi(argv[3]) : 0, master, n, calls, 0};
        run_rank(&a);
        failures = a.failures < 0 ? 1 : a.failures;
    }
    if (failures) {
        printf("result WRONG (%ld mismatches)\n", failures);
        return 1;
    }
    printf("result ok\n");
    return 0;
}
