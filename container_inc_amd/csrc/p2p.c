/* p2p.c -- the "p2p" exchange engine: reduce-scatter and all-gather as direct
 * peer reads over xGMI with this library's own kernels (no RCCL on the data path).
 *
 * Every rank owns two library-allocated device buffers whose HIP IPC handles are
 * exchanged once over the group's bootstrap sockets:
 *   part  int32 [W * shard]  this rank's quantised local sums (W shards)
 *   res   fp32  [W * shard]  this rank's dequantised result shard at rank * shard
 * One bucket piece:
 *   1. quant + local sum of the R buckets -> part            (HBM, local)
 *   2. stream sync + group barrier                            (all parts ready)
 *   3. res[me] = dequant( sum_j part_j[me] )  -- one kernel reading the W
 *      peers' shard me concurrently (W-1 of them over xGMI): the reference's
 *      switch aggregate (non_termination_switch.c:361-363) fused with the new
 *      dequantise stage
 *   4. stream sync + group barrier                            (all shards ready)
 *   5. dst[j] = res_j[j] for every j -- one gather kernel pulling all W shards
 * Buffer reuse is safe without a third barrier: a rank reaches the next
 * call's step-2 barrier only after its own step 5 has drained (the sync in 2),
 * so nobody still reads a `part` or `res` that the next call overwrites.
 * Host barriers cost tens of microseconds; the step moves hundreds of MB.
 *
 * Asynchronous mode (default; INCCL_P2P_SYNC=1 selects the synchronous one):
 * no stream synchronisation at all.  Each rank records interprocess events
 * after steps 1, 3 and 5, and before steps 1, 3 and 5 its stream waits on the
 * peers' events that guard the buffers it reads or overwrites:
 *   before 1 (overwrite own part):   peers' "reduced"  of the previous call
 *   before 3 (read peers' part,      peers' "ready"    of this call
 *             overwrite own res):    peers' "gathered" of the previous call
 *   before 5 (read peers' res):      peers' "reduced"  of this call
 * A wait binds to the event's latest record at the time of the wait, so the two
 * host barriers (shared-memory, same node) only have to guarantee that every
 * record of this phase has been ENQUEUED before anyone enqueues a wait on it --
 * the host never waits for the GPU. */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "inccl_internal.h"
#include "inccl_kernels.h"

typedef struct {
    hipIpcMemHandle_t part, res;
    hipIpcEventHandle_t ev[3];
    int32_t async;   /* this rank could export its events */
} p2p_handles;

void inccl_p2p_release(struct inccl_communicator *c)
{
    const int W = c->group->world_size, me = c->group->rank;
    if (c->p2p_cap == 0 && !c->p2p_part) return;
    hipDeviceSynchronize();
    for (int j = 0; j < W && j < INCCL_MAX_LOCAL_INPUTS; ++j) {
        if (j == me) continue;
        if (c->p2p_peer_part[j]) hipIpcCloseMemHandle(c->p2p_peer_part[j]);
        if (c->p2p_peer_res[j]) hipIpcCloseMemHandle(c->p2p_peer_res[j]);
        c->p2p_peer_part[j] = NULL;
        c->p2p_peer_res[j] = NULL;
    }
    if (c->p2p_part) hipFree(c->p2p_part);
    if (c->p2p_res) hipFree(c->p2p_res);
    c->p2p_part = NULL;
    c->p2p_res = NULL;
    c->p2p_cap = 0;
    for (int j = 0; j < W && j < INCCL_MAX_LOCAL_INPUTS; ++j)
        for (int e = 0; e < 3; ++e) {
            if (j != me && c->p2p_peer_ev[j][e]) hipEventDestroy(c->p2p_peer_ev[j][e]);
            c->p2p_peer_ev[j][e] = NULL;
        }
    for (int e = 0; e < 3; ++e) {
        if (c->p2p_ev[e]) hipEventDestroy(c->p2p_ev[e]);
        c->p2p_ev[e] = NULL;
    }
}

/* collective: every rank calls it with the same `elems` */
static int p2p_ensure(struct inccl_communicator *c, size_t elems)
{
    struct inccl_group *g = c->group;
    const int W = g->world_size, me = g->rank;
    if (c->p2p_cap >= elems && c->p2p_part) return 0;
    /* peers may still read the old buffers: drain our own GPU work, then wait
     * until every rank has drained its own (async mode queues peer reads) */
    INCCL_HIP(hipDeviceSynchronize());
    int rc = inccl_boot_barrier(g);
    if (rc) return rc;
    rc = inccl_boot_shm_init(g);   /* same-node fast barrier for the per-call syncs */
    if (rc) return rc;
    inccl_p2p_release(c);
    size_t cap = (elems + (1u << 19) - 1) & ~(size_t)((1u << 19) - 1);   /* 2 MiB granules */
    p2p_handles mine, *all = (p2p_handles *)calloc((size_t)W, sizeof(p2p_handles));
    if (!all) return inccl_set_error(INCCL_ERR_NOMEM, "p2p: out of memory");
    memset(&mine, 0, sizeof(mine));
    /* local failures are carried to the collective outcome check below */
    hipError_t e = hipMalloc((void **)&c->p2p_part, cap * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&c->p2p_res, cap * sizeof(float));
    if (e == hipSuccess) {
        c->p2p_cap = cap;
        e = hipIpcGetMemHandle(&mine.part, c->p2p_part);
        if (e == hipSuccess) e = hipIpcGetMemHandle(&mine.res, c->p2p_res);
    }
    if (e != hipSuccess) rc = inccl_hip_check(e, "p2p: hipMalloc/hipIpcGetMemHandle");
    /* interprocess events for the asynchronous mode (falls back to synchronous
     * mode on every rank if any rank cannot export them) */
    const char *sync_env = getenv("INCCL_P2P_SYNC");
    mine.async = !(sync_env && atoi(sync_env) != 0);
    for (int k = 0; mine.async && k < 3; ++k) {
        if (hipEventCreateWithFlags(&c->p2p_ev[k], hipEventInterprocess | hipEventDisableTiming) != hipSuccess ||
            hipIpcGetEventHandle(&mine.ev[k], c->p2p_ev[k]) != hipSuccess ||
            hipEventRecord(c->p2p_ev[k], c->stream) != hipSuccess)   /* a first record: waits are then valid */
            mine.async = 0;
    }
    if (mine.async && hipStreamSynchronize(c->stream) != hipSuccess) mine.async = 0;
    int rc_x = inccl_boot_allgather(g, &mine, all, sizeof(p2p_handles));
    if (rc_x) {
        free(all);
        return rc_x;
    }
    int async = 1;
    for (int j = 0; j < W; ++j) async = async && all[j].async;
    for (int j = 0; rc == 0 && j < W; ++j) {
        if (j == me) {
            c->p2p_peer_part[j] = c->p2p_part;
            c->p2p_peer_res[j] = c->p2p_res;
            for (int k = 0; k < 3; ++k) c->p2p_peer_ev[j][k] = c->p2p_ev[k];
            continue;
        }
        for (int k = 0; async && k < 3; ++k) {
            hipEvent_t pe = NULL;
            if (hipIpcOpenEventHandle(&pe, all[j].ev[k]) != hipSuccess) rc = inccl_set_error(INCCL_ERR_HIP,
                                                                                        "hipIpcOpenEventHandle");
            c->p2p_peer_ev[j][k] = pe;
        }
        void *pp = NULL, *pr = NULL;
        e = hipIpcOpenMemHandle(&pp, all[j].part, hipIpcMemLazyEnablePeerAccess);
        if (e == hipSuccess) e = hipIpcOpenMemHandle(&pr, all[j].res, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) rc = inccl_hip_check(e, "hipIpcOpenMemHandle");
        c->p2p_peer_part[j] = (int32_t *)pp;
        c->p2p_peer_res[j] = (float *)pr;
    }
    free(all);
    /* agree on the outcome: a rank whose IPC mapping failed must not leave its
     * peers waiting in a barrier it never reaches, and everyone must see the
     * failure so the caller can fall back on every rank alike */
    int32_t mine_rc = rc ? 1 : 0, all_rc[64];
    if (W > 64) return inccl_set_error(INCCL_ERR_ARG, "p2p: world too large");
    int rc2 = inccl_boot_allgather(g, &mine_rc, all_rc, sizeof(int32_t));
    if (rc2) return rc2;
    for (int j = 0; j < W; ++j)
        if (all_rc[j]) {
            if (!rc) rc = inccl_set_error(INCCL_ERR_HIP, "p2p: rank %d could not map the peer buffers", j);
            inccl_p2p_release(c);
            return rc;
        }
    /* probe: every rank must be able to enqueue a wait on every peer event */
    if (async) {
        int32_t ok = 1, all_ok[64];
        for (int j = 0; ok && j < W; ++j)
            for (int k = 0; ok && j != me && k < 3; ++k)
                ok = hipStreamWaitEvent(c->stream, c->p2p_peer_ev[j][k], 0) == hipSuccess;
        if (!ok) (void)hipGetLastError();
        if (hipStreamSynchronize(c->stream) != hipSuccess) ok = 0;
        rc2 = inccl_boot_allgather(g, &ok, all_ok, sizeof(ok));
        if (rc2) return rc2;
        for (int j = 0; j < W; ++j) async = async && all_ok[j];
    }
    c->p2p_async = async;
    return 0;
}

static int sync_and_barrier(struct inccl_communicator *c, hipStream_t st)
{
    INCCL_HIP(hipStreamSynchronize(st));
    return inccl_group_barrier(c->group);
}

static int wait_peers(struct inccl_communicator *c, hipStream_t st, int which)
{
    const int W = c->group->world_size, me = c->group->rank;
    for (int j = 0; j < W; ++j)
        if (j != me) INCCL_HIP(hipStreamWaitEvent(st, c->p2p_peer_ev[j][which], 0));
    return 0;
}

static void gather_plan(struct inccl_communicator *c, size_t n, size_t shard, const void **src, int64_t *off,
                        int64_t *cnt)
{
    const int W = c->group->world_size;
    for (int j = 0; j < W; ++j) {
        const size_t lo = (size_t)j * shard;
        src[j] = c->p2p_peer_res[j] + lo;
        off[j] = (int64_t)lo;
        cnt[j] = lo >= n ? 0 : (int64_t)((n - lo) < shard ? (n - lo) : shard);
    }
}

enum { EV_READY = 0, EV_REDUCED = 1, EV_GATHERED = 2 };

static int p2p_piece_async(struct inccl_communicator *c, const float *const *srcs, int R, float *dst, size_t n,
                           int k, const uint32_t *amax, int scale_R, hipStream_t st, size_t shard, size_t total)
{
    const int W = c->group->world_size, me = c->group->rank;
    /* 1. own partials, once every peer has finished reading the previous ones */
    int rc = wait_peers(c, st, EV_REDUCED);
    if (rc) return rc;
    rc = inccl_k_stream(INCCL_KIND_F32, INCCL_KIND_Q32, (const void *const *)srcs, R, c->p2p_part, n, k, amax,
                        scale_R, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p quant+sum launch failed (%d)", rc);
    if (total > n) INCCL_HIP(hipMemsetAsync(c->p2p_part + n, 0, (total - n) * sizeof(int32_t), st));
    INCCL_HIP(hipEventRecord(c->p2p_ev[EV_READY], st));
    rc = inccl_group_barrier(c->group);   /* every READY record enqueued */
    if (rc) return rc;
    /* 3. pull shard `me` from every peer once it is ready and our result shard is free */
    rc = wait_peers(c, st, EV_READY);
    if (rc == 0) rc = wait_peers(c, st, EV_GATHERED);
    if (rc) return rc;
    const void *peer[INCCL_MAX_LOCAL_INPUTS];
    for (int j = 0; j < W; ++j) peer[j] = c->p2p_peer_part[j] + (size_t)me * shard;
    rc = inccl_k_stream(INCCL_KIND_Q32, INCCL_KIND_F32, peer, W, c->p2p_res + (size_t)me * shard, shard, k, amax,
                        scale_R, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p reduce-scatter launch failed (%d)", rc);
    INCCL_HIP(hipEventRecord(c->p2p_ev[EV_REDUCED], st));
    rc = inccl_group_barrier(c->group);   /* every REDUCED record enqueued */
    if (rc) return rc;
    /* 5. gather every result shard once its owner has produced it */
    rc = wait_peers(c, st, EV_REDUCED);
    if (rc) return rc;
    const void *src[INCCL_MAX_LOCAL_INPUTS];
    int64_t off[INCCL_MAX_LOCAL_INPUTS], cnt[INCCL_MAX_LOCAL_INPUTS];
    gather_plan(c, n, shard, src, off, cnt);
    rc = inccl_k_gather(src, off, cnt, W, dst, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p gather launch failed (%d)", rc);
    INCCL_HIP(hipEventRecord(c->p2p_ev[EV_GATHERED], st));
    return 0;
}

int inccl_p2p_piece(struct inccl_communicator *c, const float *const *srcs, int R, float *dst, size_t n, int k,
                    const uint32_t *amax, int scale_R, hipStream_t st)
{
    const int W = c->group->world_size, me = c->group->rank;
    if (W > INCCL_MAX_LOCAL_INPUTS) return inccl_set_error(INCCL_ERR_ARG, "p2p engine supports up to %d GPUs",
                                                          INCCL_MAX_LOCAL_INPUTS);
    const size_t shard = inccl_shard_elems(n, W), total = shard * (size_t)W;
    int rc = p2p_ensure(c, total);
    if (rc) return rc;
    if (c->p2p_async) return p2p_piece_async(c, srcs, R, dst, n, k, amax, scale_R, st, shard, total);
    /* 1. local quantise + sum */
    rc = inccl_k_stream(INCCL_KIND_F32, INCCL_KIND_Q32, (const void *const *)srcs, R, c->p2p_part, n, k, amax,
                        scale_R, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p quant+sum launch failed (%d)", rc);
    if (total > n) INCCL_HIP(hipMemsetAsync(c->p2p_part + n, 0, (total - n) * sizeof(int32_t), st));
    rc = sync_and_barrier(c, st);
    if (rc) return rc;
    /* 3. pull shard `me` from every peer, sum, dequantise */
    const void *peer[INCCL_MAX_LOCAL_INPUTS];
    for (int j = 0; j < W; ++j) peer[j] = c->p2p_peer_part[j] + (size_t)me * shard;
    rc = inccl_k_stream(INCCL_KIND_Q32, INCCL_KIND_F32, peer, W, c->p2p_res + (size_t)me * shard, shard, k, amax,
                        scale_R, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p reduce-scatter launch failed (%d)", rc);
    rc = sync_and_barrier(c, st);
    if (rc) return rc;
    /* 5. gather every shard into dst (ragged last shard clamped to n) */
    const void *src[INCCL_MAX_LOCAL_INPUTS];
    int64_t off[INCCL_MAX_LOCAL_INPUTS], cnt[INCCL_MAX_LOCAL_INPUTS];
    gather_plan(c, n, shard, src, off, cnt);
    rc = inccl_k_gather(src, off, cnt, W, dst, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p gather launch failed (%d)", rc);
    return 0;
}
