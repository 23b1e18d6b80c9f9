/* host_example.c -- the reference's example program (repository/src/host.c:28-59)
 * rewritten against include/api.h: same inputs (in[i] = i*(rank+1), host.c:20-25),
 * same communicator size (host.c:41) and the same known answer (host.c:51-55),
 * here with `world_size` ranks as threads over the in-process transport.
 *
 *   host_example <world_size> <master_ip|local> [rank]
 *
 * With master_ip "local" all ranks run as threads of this process on one GPU
 * and the expected value becomes i * world*(world+1)/2 (3*i for the
 * reference's two ranks).  With an IP the process is one rank, as in host.c. */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "inccl_amd.h"

#define IN_DATA_COUNT 4096

struct rank_arg {
    int world, rank;
    const char *master;
    int failures;
};

static void *run_rank(void *p)
{
    struct rank_arg *a = (struct rank_arg *)p;
    int32_t *in_data = malloc(IN_DATA_COUNT * sizeof(int32_t));
    int32_t *dst_data = malloc(IN_DATA_COUNT * sizeof(int32_t));
    for (int i = 0; i < IN_DATA_COUNT; ++i) in_data[i] = i * (a->rank + 1);
    memset(dst_data, 0, IN_DATA_COUNT * sizeof(int32_t));
    struct inccl_group *group = strcmp(a->master, "local") == 0
                                    ? inccl_group_create_local(a->world, a->rank, "host_example", -1)
                                    : inccl_group_create(a->world, a->rank, a->master);
    if (!group) {
        fprintf(stderr, "rank %d: group create failed: %s\n", a->rank, inccl_last_error());
        a->failures = -1;
        return NULL;
    }
    struct inccl_communicator *comm = inccl_communicator_create(group, IN_DATA_COUNT * 4);
    if (!comm) {
        fprintf(stderr, "rank %d: communicator create failed: %s\n", a->rank, inccl_last_error());
        a->failures = -1;
        return NULL;
    }
    inccl_allreduce_write(comm, in_data, IN_DATA_COUNT, dst_data);
    const long long mult = (long long)a->world * (a->world + 1) / 2;
    for (int i = 0; i < IN_DATA_COUNT; ++i)
        if (dst_data[i] != (int32_t)(mult * i)) a->failures++;
    /* and once more through the send/recv variant (api.c:330-401) */
    memset(dst_data, 0, IN_DATA_COUNT * sizeof(int32_t));
    inccl_allreduce_sendrecv(comm, in_data, IN_DATA_COUNT, dst_data);
    for (int i = 0; i < IN_DATA_COUNT; ++i)
        if (dst_data[i] != (int32_t)(mult * i)) a->failures++;
    inccl_communicator_destroy(comm);
    inccl_group_destroy(group);
    free(in_data);
    free(dst_data);
    return NULL;
}

int main(int argc, char **argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s <world_size> <master_ip|local> [rank]\n", argv[0]);
        return 2;
    }
    const int world = atoi(argv[1]);
    const char *master = argv[2];
    int failures = 0;
    if (strcmp(master, "local") == 0) {
        pthread_t th[INCCL_MAX_LOCAL_INPUTS];
        struct rank_arg args[INCCL_MAX_LOCAL_INPUTS];
        if (world < 1 || world > INCCL_MAX_LOCAL_INPUTS) return 2;
        for (int r = 0; r < world; ++r) {
            args[r] = (struct rank_arg){world, r, master, 0};
            pthread_create(&th[r], NULL, run_rank, &args[r]);
        }
        for (int r = 0; r < world; ++r) {
            pthread_join(th[r], NULL);
            failures += args[r].failures < 0 ? 1 : args[r].failures;
        }
    } else {
        struct rank_arg a = {world, argc > 3 ? atoi(argv[3]) : 0, master, 0};
        run_rank(&a);
        failures = a.failures < 0 ? 1 : a.failures;
    }
    if (failures) {
        printf("result WRONG (%d mismatches)\n", failures);
        return 1;
    }
    printf("result ok\n");
    return 0;
}
