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
 * Steps 3 and 5 read peer memory with system-coherent loads (inccl_peer.hip):
 * IPC-mapped remote VRAM may sit non-coherently in this GPU's L2 from the
 * previous call. */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "inccl_internal.h"
#include "inccl_kernels.h"

typedef struct {
    hipIpcMemHandle_t part, res;
} p2p_handles;

/* $INCCL_TRACE: every (re)growth logs, per rank, the FNV-1a hash of each
 * exported handle and the base address each peer's buffer mapped to, so that
 * a mapping that resolves to an earlier export (same base as before while the
 * handle changed) is visible in the log */
static uint64_t handle_hash(const hipIpcMemHandle_t *h)
{
    const unsigned char *b = (const unsigned char *)h;
    uint64_t x = 1469598103934665603ull;
    for (size_t i = 0; i < sizeof(*h); ++i) x = (x ^ b[i]) * 1099511628211ull;
    return x;
}

static void p2p_trace(const struct inccl_communicator *c, const char *what, const p2p_handles *all, int W)
{
    if (!getenv("INCCL_TRACE")) return;
    char line[2048];
    int k = snprintf(line, sizeof(line), "[inccl p2p rank %d] %s cap %zu own part %p res %p", c->group->rank, what,
                     c->p2p_cap, (void *)c->p2p_part, (void *)c->p2p_res);
    for (int j = 0; j < W && k > 0 && (size_t)k < sizeof(line); ++j)
        k += snprintf(line + k, sizeof(line) - (size_t)k, " | peer %d handle %016llx/%016llx -> part %p res %p", j,
                      all ? (unsigned long long)handle_hash(&all[j].part) : 0ull,
                      all ? (unsigned long long)handle_hash(&all[j].res) : 0ull, (void *)c->p2p_peer_part[j],
                      (void *)c->p2p_peer_res[j]);
    fprintf(stderr, "%s\n", line);   /* one write per line: ranks share the log */
}

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
}

/* collective: every rank calls it with the same `elems` */
static int p2p_ensure(struct inccl_communicator *c, size_t elems)
{
    struct inccl_group *g = c->group;
    const int W = g->world_size, me = g->rank;
    if (c->p2p_cap >= elems && c->p2p_part) return 0;
    if (elems * sizeof(int32_t) > g->ipc_max_bytes)   /* same sizes and bound on every rank: all refuse alike */
        return inccl_set_error(INCCL_ERR_ARG, "p2p: a %zu-element bucket needs %zu-byte IPC buffers; this group's stay "
                               "below %zu bytes (under PyTorch's bundled HSA runtime, importing a larger one hangs; "
                               "runtime.c)", elems, elems * sizeof(int32_t), g->ipc_max_bytes);
    /* this rank's queued reads of the peers' buffers (the previous call's gather)
     * drain before anyone may drop them */
    INCCL_HIP(hipDeviceSynchronize());
    int rc = inccl_boot_barrier(g);
    if (rc) return rc;
    rc = inccl_boot_shm_init(g);   /* same-node fast barrier for the per-call syncs */
    if (rc) return rc;
    /* Make before break: the new buffers are allocated, exported and mapped by
     * every peer while the old ones are still alive, and the old ones go only
     * after a barrier.  Freeing first lets a new export reuse the old one's
     * identity (a dmabuf fd number) while a peer's runtime may still resolve it
     * to the old import: a regrowth then, intermittently, left one rank reading
     * a peer's old buffer on every later call. */
    /* $INCCL_P2P_FREE_FIRST=1 restores the first version's order (free the old
     * buffers, then allocate and exchange the new ones) -- for the regrowth
     * regression test only */
    const char *ff = getenv("INCCL_P2P_FREE_FIRST");
    if (ff && atoi(ff) != 0 && c->p2p_part) {
        p2p_trace(c, "free-first: releasing", NULL, W);
        rc = inccl_boot_barrier(g);
        if (rc) return rc;
        inccl_p2p_release(c);
    }
    struct inccl_communicator old = *c;
    c->p2p_part = NULL;
    c->p2p_res = NULL;
    c->p2p_cap = 0;
    for (int j = 0; j < INCCL_MAX_LOCAL_INPUTS; ++j) {
        c->p2p_peer_part[j] = NULL;
        c->p2p_peer_res[j] = NULL;
    }
    size_t cap = (elems + (1u << 19) - 1) & ~(size_t)((1u << 19) - 1);   /* 2 MiB granules */
    p2p_handles mine, *all = (p2p_handles *)calloc((size_t)W, sizeof(p2p_handles));
    if (!all) {
        inccl_p2p_release(&old);
        return inccl_set_error(INCCL_ERR_NOMEM, "p2p: out of memory");
    }
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
    int rc_x = inccl_boot_allgather(g, &mine, all, sizeof(p2p_handles));
    if (rc_x) {
        free(all);
        inccl_p2p_release(&old);
        return rc_x;
    }
    for (int j = 0; rc == 0 && j < W; ++j) {
        if (j == me) {
            c->p2p_peer_part[j] = c->p2p_part;
            c->p2p_peer_res[j] = c->p2p_res;
            continue;
        }
        void *pp = NULL, *pr = NULL;
        e = hipIpcOpenMemHandle(&pp, all[j].part, hipIpcMemLazyEnablePeerAccess);
        if (e == hipSuccess) e = hipIpcOpenMemHandle(&pr, all[j].res, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) rc = inccl_hip_check(e, "hipIpcOpenMemHandle");
        c->p2p_peer_part[j] = (int32_t *)pp;
        c->p2p_peer_res[j] = (float *)pr;
    }
    p2p_trace(c, "mapped", all, W);
    free(all);
    /* every peer has mapped the new buffers: the old ones can go */
    int rc_b = inccl_boot_barrier(g);
    inccl_p2p_release(&old);
    if (rc_b) return rc_b;
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
    return 0;
}

static int sync_and_barrier(struct inccl_communicator *c, hipStream_t st)
{
    INCCL_HIP(hipStreamSynchronize(st));
    return inccl_group_barrier(c->group);
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
    /* the previous call's gather may still be reading the peers' result shards,
     * which the peers rewrite once this call's first barrier has passed: order
     * it before that barrier's host sync when the caller switches streams */
    if (c->p2p_last_stream && c->p2p_last_stream != st) INCCL_HIP(hipStreamWaitEvent(st, c->ev[8], 0));
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
    rc = inccl_k_peer_reduce(peer, W, c->p2p_res + (size_t)me * shard, shard, k, amax, scale_R, c->out_shift, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p reduce-scatter launch failed (%d)", rc);
    rc = sync_and_barrier(c, st);
    if (rc) return rc;
    /* 5. gather every shard into dst (ragged last shard clamped to n) */
    const void *src[INCCL_MAX_LOCAL_INPUTS];
    int64_t off[INCCL_MAX_LOCAL_INPUTS], cnt[INCCL_MAX_LOCAL_INPUTS];
    for (int j = 0; j < W; ++j) {
        const size_t lo = (size_t)j * shard;
        src[j] = c->p2p_peer_res[j] + lo;
        off[j] = (int64_t)lo;
        cnt[j] = lo >= n ? 0 : (int64_t)((n - lo) < shard ? (n - lo) : shard);
    }
    rc = inccl_k_peer_gather(src, off, cnt, W, dst, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p gather launch failed (%d)", rc);
    INCCL_HIP(hipEventRecord(c->ev[8], st));
    c->p2p_last_stream = st;
    return 0;
}

/* bfloat16 / float16 buckets (kind) over the same buffers and barriers: quant +
 * local sum of the 2-byte buckets -> part; barrier; shard `me` pulled from every
 * peer, summed, dequantised and narrowed in one kernel into res (2-byte elements
 * at me * shard); barrier; every rank's 2-byte result shard gathered -- 2 bytes
 * per element over xGMI instead of the int32 allreduce's 4.  dst must be 4-byte
 * aligned. */
int inccl_p2p_piece16(struct inccl_communicator *c, int kind, const uint16_t *const *srcs, int R, uint16_t *dst,
                      size_t n, int k, const uint32_t *amax, int scale_R, hipStream_t st)
{
    const int W = c->group->world_size, me = c->group->rank;
    if (W > INCCL_MAX_LOCAL_INPUTS) return inccl_set_error(INCCL_ERR_ARG, "p2p engine supports up to %d GPUs",
                                                          INCCL_MAX_LOCAL_INPUTS);
    const size_t shard = inccl_shard_elems(n, W), total = shard * (size_t)W;
    int rc = p2p_ensure(c, total);
    if (rc) return rc;
    if (c->p2p_last_stream && c->p2p_last_stream != st) INCCL_HIP(hipStreamWaitEvent(st, c->ev[8], 0));
    rc = inccl_k_stream(kind, INCCL_KIND_Q32, (const void *const *)srcs, R, c->p2p_part, n, k, amax, scale_R, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p 16-bit quant+sum launch failed (%d)", rc);
    if (total > n) INCCL_HIP(hipMemsetAsync(c->p2p_part + n, 0, (total - n) * sizeof(int32_t), st));
    rc = sync_and_barrier(c, st);
    if (rc) return rc;
    const void *peer[INCCL_MAX_LOCAL_INPUTS];
    for (int j = 0; j < W; ++j) peer[j] = c->p2p_peer_part[j] + (size_t)me * shard;
    rc = inccl_k_peer_reduce16(kind, peer, W, (uint16_t *)c->p2p_res + (size_t)me * shard, shard, k, amax, scale_R,
                               c->out_shift, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p 16-bit reduce-scatter launch failed (%d)", rc);
    rc = sync_and_barrier(c, st);
    if (rc) return rc;
    const void *src[INCCL_MAX_LOCAL_INPUTS];
    int64_t off[INCCL_MAX_LOCAL_INPUTS], cnt[INCCL_MAX_LOCAL_INPUTS];
    for (int j = 0; j < W; ++j) {
        const size_t lo = (size_t)j * shard;
        src[j] = (const uint16_t *)c->p2p_peer_res[j] + lo;
        off[j] = (int64_t)lo;
        cnt[j] = lo >= n ? 0 : (int64_t)((n - lo) < shard ? (n - lo) : shard);
    }
    rc = inccl_k_peer_gather16(src, off, cnt, W, dst, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p 16-bit gather launch failed (%d)", rc);
    INCCL_HIP(hipEventRecord(c->ev[8], st));
    c->p2p_last_stream = st;
    return 0;
}

/* Reduce-scatter over the same buffers: quant + local sum -> part; barrier;
 * shard `me` pulled from every peer, summed and dequantised (narrowed for the
 * 2-byte kinds) straight into dst; barrier, so that no rank rewrites its part
 * (the next call's quantise) while a peer still reads it.  n = W * shard,
 * shard % 4 == 0. */
int inccl_p2p_reduce_scatter(struct inccl_communicator *c, int kind, const void *const *srcs, int R, void *dst,
                             size_t n, int k, const uint32_t *amax, int scale_R, hipStream_t st)
{
    const int W = c->group->world_size, me = c->group->rank;
    if (W > INCCL_MAX_LOCAL_INPUTS) return inccl_set_error(INCCL_ERR_ARG, "p2p engine supports up to %d GPUs",
                                                          INCCL_MAX_LOCAL_INPUTS);
    const size_t shard = n / (size_t)W;
    if (shard * (size_t)W != n || (shard & 3)) return inccl_set_error(INCCL_ERR_ARG, "p2p reduce-scatter: bad shard");
    int rc = p2p_ensure(c, n);
    if (rc) return rc;
    if (c->p2p_last_stream && c->p2p_last_stream != st) INCCL_HIP(hipStreamWaitEvent(st, c->ev[8], 0));
    rc = inccl_k_stream(kind, INCCL_KIND_Q32, srcs, R, c->p2p_part, n, k, amax, scale_R, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p reduce-scatter quant+sum launch failed (%d)", rc);
    rc = sync_and_barrier(c, st);
    if (rc) return rc;
    const void *peer[INCCL_MAX_LOCAL_INPUTS];
    for (int j = 0; j < W; ++j) peer[j] = c->p2p_peer_part[j] + (size_t)me * shard;
    rc = kind == INCCL_KIND_F32
             ? inccl_k_peer_reduce(peer, W, (float *)dst, shard, k, amax, scale_R, c->out_shift, st)
             : inccl_k_peer_reduce16(kind, peer, W, (uint16_t *)dst, shard, k, amax, scale_R, c->out_shift, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p reduce-scatter launch failed (%d)", rc);
    rc = sync_and_barrier(c, st);
    if (rc) return rc;
    INCCL_HIP(hipEventRecord(c->ev[8], st));
    c->p2p_last_stream = st;
    return 0;
}

/* The int32 allreduce over the same buffers and barriers as inccl_p2p_piece,
 * with the sum left in int32 (the reference's switch add, nts.c:361-363, and
 * nothing else): copy in -> barrier -> pull + sum shard `me` from every peer ->
 * barrier -> gather every shard.  send may alias recv. */
int inccl_p2p_allreduce_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t n,
                            hipStream_t st)
{
    const int W = c->group->world_size, me = c->group->rank;
    if (W > INCCL_MAX_LOCAL_INPUTS) return inccl_set_error(INCCL_ERR_ARG, "p2p engine supports up to %d GPUs",
                                                          INCCL_MAX_LOCAL_INPUTS);
    if (n == 0) return 0;
    const size_t shard = inccl_shard_elems(n, W), total = shard * (size_t)W;
    int rc = p2p_ensure(c, total);
    if (rc) return rc;
    if (c->p2p_last_stream && c->p2p_last_stream != st) INCCL_HIP(hipStreamWaitEvent(st, c->ev[8], 0));
    INCCL_HIP(hipMemcpyAsync(c->p2p_part, send, n * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    if (total > n) INCCL_HIP(hipMemsetAsync(c->p2p_part + n, 0, (total - n) * sizeof(int32_t), st));
    rc = sync_and_barrier(c, st);
    if (rc) return rc;
    const void *peer[INCCL_MAX_LOCAL_INPUTS];
    for (int j = 0; j < W; ++j) peer[j] = c->p2p_peer_part[j] + (size_t)me * shard;
    rc = inccl_k_peer_sum_q32(peer, W, (int32_t *)(c->p2p_res + (size_t)me * shard), shard, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p int32 reduce-scatter launch failed (%d)", rc);
    rc = sync_and_barrier(c, st);
    if (rc) return rc;
    const void *src[INCCL_MAX_LOCAL_INPUTS];
    int64_t off[INCCL_MAX_LOCAL_INPUTS], cnt[INCCL_MAX_LOCAL_INPUTS];
    for (int j = 0; j < W; ++j) {
        const size_t lo = (size_t)j * shard;
        src[j] = c->p2p_peer_res[j] + lo;
        off[j] = (int64_t)lo;
        cnt[j] = lo >= n ? 0 : (int64_t)((n - lo) < shard ? (n - lo) : shard);
    }
    rc = inccl_k_peer_gather(src, off, cnt, W, recv, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "p2p int32 gather launch failed (%d)", rc);
    INCCL_HIP(hipEventRecord(c->ev[8], st));
    c->p2p_last_stream = st;
    return 0;
}
