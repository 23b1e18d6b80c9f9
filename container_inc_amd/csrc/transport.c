/* transport.c -- the exchange step of the allreduce, over one of two transports.
 *
 *  rccl   one process per GPU; RCCL (rccl.h, "nccl" on ROCm) over xGMI.  The
 *         reference's equivalent is the RoCE RC path to the software switch
 *         (repository/src/api.c:293-327, non_termination_switch.c:303-501).
 *  local  the ranks are threads of one process sharing one GPU; the GPU is the
 *         aggregation switch: the reduce-scatter runs this library's own sum
 *         kernel over every rank's buffer (the nts.c:361-363 aggregate), the
 *         all-gather is device-to-device copies.  Used for the single-process
 *         loopback harness and for multi-rank tests on a one-GPU box.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <rccl/rccl.h>

#include "inccl_internal.h"
#include "inccl_kernels.h"

/* ------------------------------------------------------------------ */
/* rccl                                                                 */
/* ------------------------------------------------------------------ */
/* the result code's text and RCCL's own account of the failure
 * (ncclGetLastError: the calling thread's last error message, e.g. why
 * ncclCommInitRank refused -- "invalid usage" alone does not say) */
static int nccl_check(ncclResult_t r, const char *what)
{
    if (r == ncclSuccess) return 0;
    const char *last = ncclGetLastError(NULL);
    return inccl_set_error(INCCL_ERR_NCCL, "%s: %s%s%s", what, ncclGetErrorString(r), last && *last ? ": " : "",
                           last && *last ? last : "");
}

/* a collective's own return code, then the communicator's asynchronous error
 * (a peer that died, a network failure): RCCL reports those only this way */
static int nccl_call(struct inccl_communicator *c, ncclResult_t r, const char *what)
{
    int rc = nccl_check(r, what);
    if (rc) return rc;
    ncclResult_t ae = ncclSuccess;
    if (c->nccl && ncclCommGetAsyncError((ncclComm_t)c->nccl, &ae) == ncclSuccess && ae != ncclSuccess &&
        ae != ncclInProgress)
        return inccl_set_error(INCCL_ERR_NCCL, "%s: asynchronous RCCL error: %s", what, ncclGetErrorString(ae));
    return 0;
}

int inccl_rccl_comm_init(struct inccl_communicator *c)
{
    struct inccl_group *g = c->group;
    /* rank 0 broadcasts even when it has no id, so that no peer waits on it */
    struct {
        int32_t ok;
        ncclUniqueId id;
    } u;
    memset(&u, 0, sizeof(u));
    int rc0 = 0;
    if (g->rank == 0) {
        rc0 = nccl_check(ncclGetUniqueId(&u.id), "ncclGetUniqueId");
        u.ok = rc0 == 0;
    }
    int rc = inccl_boot_bcast(g, &u, sizeof(u));
    if (rc) return rc;
    if (rc0) return rc0;
    if (!u.ok) return inccl_set_error(INCCL_ERR_NCCL, "ncclGetUniqueId failed on rank 0");
    ncclComm_t comm = NULL;
    rc = nccl_check(ncclCommInitRank(&comm, g->world_size, u.id, g->rank), "ncclCommInitRank");
    if (rc) return rc;
    c->nccl = comm;
    return 0;
}

void inccl_rccl_comm_destroy(struct inccl_communicator *c)
{
    if (c->nccl) {
        ncclCommDestroy((ncclComm_t)c->nccl);
        c->nccl = NULL;
    }
}

int inccl_rccl_reduce_scatter_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t shard,
                                  hipStream_t st)
{
    return nccl_call(c, ncclReduceScatter(send, recv, shard, ncclInt32, ncclSum, (ncclComm_t)c->nccl, st),
                      "ncclReduceScatter");
}

int inccl_rccl_all_gather_f32(struct inccl_communicator *c, const float *send, float *recv, size_t shard,
                              hipStream_t st)
{
    return nccl_call(c, ncclAllGather(send, recv, shard, ncclFloat32, (ncclComm_t)c->nccl, st), "ncclAllGather");
}

int inccl_rccl_all_gather_bf16(struct inccl_communicator *c, const uint16_t *send, uint16_t *recv, size_t shard,
                               hipStream_t st)
{
    return nccl_call(c, ncclAllGather(send, recv, shard, ncclBfloat16, (ncclComm_t)c->nccl, st), "ncclAllGather(bf16)");
}

int inccl_rccl_allreduce_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t n,
                             hipStream_t st)
{
    return nccl_call(c, ncclAllReduce(send, recv, n, ncclInt32, ncclSum, (ncclComm_t)c->nccl, st), "ncclAllReduce");
}

int inccl_rccl_allreduce_max_u32(struct inccl_communicator *c, uint32_t *buf, size_t n, hipStream_t st)
{
    return nccl_call(c, ncclAllReduce(buf, buf, n, ncclUint32, ncclMax, (ncclComm_t)c->nccl, st),
                      "ncclAllReduce(max)");
}

int inccl_rccl_alltoall_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t shard,
                            hipStream_t st)
{
    const int W = c->group->world_size, me = c->group->rank;
    if (!c->nccl && W > 1) {
        int rc = inccl_rccl_comm_init(c);
        if (rc) return rc;
    }
    if (W == 1) return 0;
    int rc = nccl_check(ncclGroupStart(), "ncclGroupStart");
    for (int j = 0; rc == 0 && j < W; ++j) {
        if (j == me) continue;
        rc = nccl_check(ncclSend(send + (size_t)j * shard, shard, ncclInt32, j, (ncclComm_t)c->nccl, st), "ncclSend");
        if (rc == 0)
            rc = nccl_check(ncclRecv(recv + (size_t)j * shard, shard, ncclInt32, j, (ncclComm_t)c->nccl, st),
                            "ncclRecv");
    }
    int rc2 = nccl_call(c, ncclGroupEnd(), "ncclGroupEnd");
    return rc ? rc : rc2;
}

/* ------------------------------------------------------------------ */
/* local hub                                                            */
/* ------------------------------------------------------------------ */
struct inccl_local_hub {
    char name[64];
    int world_size;
    int refs;
    pthread_barrier_t bar;
    const void *send[INCCL_MAX_LOCAL_INPUTS];
    uint32_t words[INCCL_MAX_LOCAL_INPUTS];
    struct inccl_local_hub *next;
};

static pthread_mutex_t g_hub_mu = PTHREAD_MUTEX_INITIALIZER;
static struct inccl_local_hub *g_hubs;

struct inccl_local_hub *inccl_hub_attach(const char *name, int world_size)
{
    if (world_size < 1 || world_size > INCCL_MAX_LOCAL_INPUTS) {
        inccl_set_error(INCCL_ERR_ARG, "local transport supports 1..%d ranks", INCCL_MAX_LOCAL_INPUTS);
        return NULL;
    }
    pthread_mutex_lock(&g_hub_mu);
    struct inccl_local_hub *h = g_hubs;
    while (h && strncmp(h->name, name, sizeof(h->name)) != 0) h = h->next;
    if (h && h->world_size != world_size) {
        pthread_mutex_unlock(&g_hub_mu);
        inccl_set_error(INCCL_ERR_ARG, "hub '%s' exists with world_size %d", name, h->world_size);
        return NULL;
    }
    if (!h) {
        h = (struct inccl_local_hub *)calloc(1, sizeof(*h));
        if (!h) {
            pthread_mutex_unlock(&g_hub_mu);
            return NULL;
        }
        snprintf(h->name, sizeof(h->name), "%s", name);
        h->world_size = world_size;
        pthread_barrier_init(&h->bar, NULL, (unsigned)world_size);
        h->next = g_hubs;
        g_hubs = h;
    }
    h->refs++;
    pthread_mutex_unlock(&g_hub_mu);
    return h;
}

void inccl_hub_detach(struct inccl_local_hub *hub)
{
    if (!hub) return;
    pthread_mutex_lock(&g_hub_mu);
    if (--hub->refs == 0) {
        struct inccl_local_hub **pp = &g_hubs;
        while (*pp && *pp != hub) pp = &(*pp)->next;
        if (*pp) *pp = hub->next;
        pthread_barrier_destroy(&hub->bar);
        free(hub);
    }
    pthread_mutex_unlock(&g_hub_mu);
}

int inccl_local_barrier(struct inccl_communicator *c)
{
    pthread_barrier_wait(&c->group->hub->bar);
    return 0;
}

/* publish this rank's buffer once its producers on `st` have finished */
static int hub_publish(struct inccl_communicator *c, const void *p, hipStream_t st)
{
    INCCL_HIP(hipStreamSynchronize(st));
    c->group->hub->send[c->group->rank] = p;
    pthread_barrier_wait(&c->group->hub->bar);
    return 0;
}

static int hub_release(struct inccl_communicator *c, hipStream_t st)
{
    hipError_t e = hipStreamSynchronize(st);
    pthread_barrier_wait(&c->group->hub->bar);   /* nobody reads a peer buffer after this */
    return e == hipSuccess ? 0 : inccl_hip_check(e, "hipStreamSynchronize");
}

int inccl_local_reduce_scatter_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t shard,
                                   hipStream_t st)
{
    struct inccl_local_hub *h = c->group->hub;
    const int W = h->world_size, me = c->group->rank;
    int rc = hub_publish(c, send, st);
    if (rc) return rc;
    const void *srcs[INCCL_MAX_LOCAL_INPUTS];
    for (int j = 0; j < W; ++j) srcs[j] = (const int32_t *)h->send[j] + (size_t)me * shard;
    rc = inccl_k_stream(INCCL_KIND_Q32, INCCL_KIND_Q32, srcs, W, recv, shard, 0, NULL, W, st);
    int rc2 = hub_release(c, st);
    return rc ? inccl_set_error(INCCL_ERR_HIP, "local reduce-scatter kernel failed (%d)", rc) : rc2;
}

/* shards of `esize`-byte elements */
static int local_all_gather(struct inccl_communicator *c, const void *send, void *recv, size_t shard, size_t esize,
                            hipStream_t st)
{
    struct inccl_local_hub *h = c->group->hub;
    const int W = h->world_size;
    int rc = hub_publish(c, send, st);
    if (rc) return rc;
    for (int j = 0; j < W && rc == 0; ++j) {
        char *d = (char *)recv + (size_t)j * shard * esize;
        if ((const void *)d == h->send[j]) continue;   /* in-place own shard */
        hipError_t e = hipMemcpyAsync(d, h->send[j], shard * esize, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) rc = inccl_hip_check(e, "hipMemcpyAsync(all-gather)");
    }
    int rc2 = hub_release(c, st);
    return rc ? rc : rc2;
}

int inccl_local_all_gather_f32(struct inccl_communicator *c, const float *send, float *recv, size_t shard,
                               hipStream_t st)
{
    return local_all_gather(c, send, recv, shard, sizeof(float), st);
}

int inccl_local_allreduce_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t n,
                              hipStream_t st)
{
    struct inccl_local_hub *h = c->group->hub;
    const int W = h->world_size;
    /* sum into private scratch first: recv may alias a buffer a peer is still reading */
    int rc = inccl_ws_claim(c, st);
    if (rc) return rc;
    rc = inccl_ensure_dev(&c->d_q32, &c->d_q32_bytes, n * sizeof(int32_t));
    if (rc) return rc;
    rc = hub_publish(c, send, st);
    if (rc) return rc;
    const void *srcs[INCCL_MAX_LOCAL_INPUTS];
    for (int j = 0; j < W; ++j) srcs[j] = h->send[j];
    rc = inccl_k_stream(INCCL_KIND_Q32, INCCL_KIND_Q32, srcs, W, c->d_q32, n, 0, NULL, W, st);
    int rc2 = hub_release(c, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "local allreduce kernel failed (%d)", rc);
    if (rc2) return rc2;
    INCCL_HIP(hipMemcpyAsync(recv, c->d_q32, n * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    return 0;
}

int inccl_local_allreduce_max_u32(struct inccl_communicator *c, uint32_t *buf, size_t n, hipStream_t st)
{
    struct inccl_local_hub *h = c->group->hub;
    const int W = h->world_size, me = c->group->rank;
    if (n != 1) return inccl_set_error(INCCL_ERR_ARG, "local max-allreduce handles one word");
    uint32_t v = 0;
    INCCL_HIP(hipMemcpyAsync(&v, buf, sizeof(v), hipMemcpyDeviceToHost, st));
    INCCL_HIP(hipStreamSynchronize(st));
    h->words[me] = v;
    pthread_barrier_wait(&h->bar);
    uint32_t m = 0;
    for (int j = 0; j < W; ++j) m = h->words[j] > m ? h->words[j] : m;
    pthread_barrier_wait(&h->bar);
    INCCL_HIP(hipMemcpyAsync(buf, &m, sizeof(m), hipMemcpyHostToDevice, st));
    INCCL_HIP(hipStreamSynchronize(st));
    return 0;
}

/* ------------------------------------------------------------------ */
/* dispatch                                                             */
/* ------------------------------------------------------------------ */
static int is_local(const struct inccl_communicator *c) { return c->group->transport == INCCL_TRANSPORT_LOCAL; }

/* RCCL communicator on first use when the engine skipped the eager init (p2p) */
static int ensure_rccl(struct inccl_communicator *c)
{
    if (c->nccl || c->group->world_size == 1) return 0;
    return inccl_rccl_comm_init(c);
}

/* 4-byte max over the group on the host (the IPC engines): the node's shared
 * memory segment once the engine has set it up, else the bootstrap sockets */
static int host_allreduce_max_u32(struct inccl_communicator *c, uint32_t *buf, hipStream_t st)
{
    uint32_t v = 0;
    INCCL_HIP(hipMemcpyAsync(&v, buf, sizeof(v), hipMemcpyDeviceToHost, st));
    INCCL_HIP(hipStreamSynchronize(st));
    int rc = inccl_group_allreduce_max_u32(c->group, &v);
    if (rc) return rc;
    const uint32_t m = v;
    INCCL_HIP(hipMemcpyAsync(buf, &m, sizeof(m), hipMemcpyHostToDevice, st));
    INCCL_HIP(hipStreamSynchronize(st));
    return 0;
}

int inccl_tp_reduce_scatter_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t shard,
                                hipStream_t st)
{
    if (is_local(c)) return inccl_local_reduce_scatter_q32(c, send, recv, shard, st);
    int rc = ensure_rccl(c);
    if (rc) return rc;
    if (!c->nccl) {   /* world 1 without RCCL: the reduce-scatter is a copy */
        if (send != recv) INCCL_HIP(hipMemcpyAsync(recv, send, shard * 4, hipMemcpyDeviceToDevice, st));
        return 0;
    }
    return inccl_rccl_reduce_scatter_q32(c, send, recv, shard, st);
}

int inccl_tp_all_gather_f32(struct inccl_communicator *c, const float *send, float *recv, size_t shard,
                            hipStream_t st)
{
    if (is_local(c)) return inccl_local_all_gather_f32(c, send, recv, shard, st);
    int rc = ensure_rccl(c);
    if (rc) return rc;
    if (!c->nccl) {
        if (send != recv) INCCL_HIP(hipMemcpyAsync(recv, send, shard * 4, hipMemcpyDeviceToDevice, st));
        return 0;
    }
    return inccl_rccl_all_gather_f32(c, send, recv, shard, st);
}

int inccl_tp_all_gather_bf16(struct inccl_communicator *c, const uint16_t *send, uint16_t *recv, size_t shard,
                             hipStream_t st)
{
    if (is_local(c)) return local_all_gather(c, send, recv, shard, sizeof(uint16_t), st);
    int rc = ensure_rccl(c);
    if (rc) return rc;
    if (!c->nccl) {
        if (send != recv) INCCL_HIP(hipMemcpyAsync(recv, send, shard * 2, hipMemcpyDeviceToDevice, st));
        return 0;
    }
    return inccl_rccl_all_gather_bf16(c, send, recv, shard, st);
}

int inccl_tp_allreduce_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t n,
                           hipStream_t st)
{
    if (is_local(c)) return inccl_local_allreduce_q32(c, send, recv, n, st);
    /* the IPC engines carry the int32 allreduce without RCCL */
    if ((c->engine == INCCL_ENGINE_P2P || c->engine == INCCL_ENGINE_LL || c->engine == INCCL_ENGINE_MESH) &&
        c->group->world_size > 1)
        return inccl_p2p_allreduce_q32(c, send, recv, n, st);
    int rc = ensure_rccl(c);
    if (rc) return rc;
    if (!c->nccl) {
        if (send != recv) INCCL_HIP(hipMemcpyAsync(recv, send, n * 4, hipMemcpyDeviceToDevice, st));
        return 0;
    }
    return inccl_rccl_allreduce_q32(c, send, recv, n, st);
}

int inccl_tp_allreduce_max_u32(struct inccl_communicator *c, uint32_t *buf, size_t n, hipStream_t st)
{
    if (is_local(c)) return inccl_local_allreduce_max_u32(c, buf, n, st);
    if ((c->engine == INCCL_ENGINE_P2P || c->engine == INCCL_ENGINE_LL || c->engine == INCCL_ENGINE_MESH) && n == 1)
        return host_allreduce_max_u32(c, buf, st);
    int rc = ensure_rccl(c);
    if (rc) return rc;
    if (!c->nccl) return 0;
    return inccl_rccl_allreduce_max_u32(c, buf, n, st);
}

int inccl_tp_barrier(struct inccl_communicator *c)
{
    if (is_local(c)) return inccl_local_barrier(c);
    return inccl_group_barrier(c->group);
}
