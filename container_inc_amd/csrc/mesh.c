/* mesh.c -- host side of the "mesh" engine: a large-bucket allreduce as one
 * persistent kernel per rank (work items, schedule and protocol in
 * inccl_mesh.hip).
 *
 * The p2p engine (p2p.c) runs quantise -> barrier -> pull reduce-scatter ->
 * barrier -> pull all-gather, with two host stream synchronisations per call
 * and no overlap between the phases.  Here one kernel does the whole call: its
 * push / reduce / gather items of different chunks meet through flags in HBM,
 * so quantisation, the local sums and the xGMI traffic in both directions
 * overlap, and the host never waits.
 *
 * Per rank, four device allocations shared over HIP IPC (separate, so that no
 * single export needs to exceed the group's IPC bound; see runtime.c):
 *   sig    [0, 64 KiB) signal array: arrive[8][1024] and ready[8][1024] words;
 *          [64 KiB, +256) call counter, retired workgroups, ticket, abort word,
 *          started workgroups, pushes finished per destination, clock
 *          readings (inccl_mesh.hip MeshArgs::ctr)
 *   inbox  W * cap int32: slot j holds rank j's partial of my shard
 *   res    cap fp32: my dequantised result shard
 *   resin  W * cap fp32 ("meshw"): slot j holds rank j's result shard
 * Created collectively on the first call, regrown collectively when a larger
 * bucket arrives (all ranks make the same calls, as with RCCL). */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "inccl_internal.h"
#include "inccl_kernels.h"

#define MESH_SIG_BYTES ((size_t)2 * INCCL_MAX_LOCAL_INPUTS * INCCL_MESH_MAX_CHUNKS * sizeof(uint32_t))
#define MESH_CTR_OFFSET MESH_SIG_BYTES
#define MESH_DATA_OFFSET (MESH_SIG_BYTES + (size_t)65536)

/* $INCCL_TRACE: one timestamped line per setup step (debugging aid) */
#define MTRACE(...)                                                                      \
    do {                                                                                 \
        if (getenv("INCCL_TRACE")) {                                                     \
            struct timespec ts_;                                                         \
            clock_gettime(CLOCK_MONOTONIC, &ts_);                                        \
            fprintf(stderr, "[inccl %d %ld.%06ld] ", c->group->rank, (long)ts_.tv_sec,   \
                    ts_.tv_nsec / 1000);                                                 \
            fprintf(stderr, __VA_ARGS__);                                                \
            fputc('\n', stderr);                                                         \
        }                                                                                \
    } while (0)

typedef struct {
    hipIpcMemHandle_t h[INCCL_MESH_REGIONS];
    int pci_domain, pci_bus, pci_dev;   /* ranks sharing a GPU split its workgroup slots */
} mesh_peer_info;

void inccl_mesh_release(struct inccl_communicator *c)
{
    const int W = c->group->world_size, me = c->group->rank;
    if (!c->mesh_buf && !c->mesh_reg[1] && !c->mesh_reg[2] && !c->mesh_reg[3]) return;
    hipDeviceSynchronize();
    for (int r = 0; r < INCCL_MESH_REGIONS; ++r) {
        for (int j = 0; j < W && j < INCCL_MAX_LOCAL_INPUTS; ++j) {
            if (j != me && c->mesh_peer[r][j]) hipIpcCloseMemHandle(c->mesh_peer[r][j]);
            c->mesh_peer[r][j] = NULL;
        }
        if (c->mesh_reg[r]) hipFree(c->mesh_reg[r]);
        c->mesh_reg[r] = NULL;
    }
    c->mesh_buf = NULL;
    if (c->mesh_err_host) hipHostFree(c->mesh_err_host);
    c->mesh_err_host = NULL;
    c->mesh_err_dev = NULL;
    c->mesh_cap = 0;
}

/* bytes of region r for W ranks and `cap` elements per slot */
static size_t mesh_region_bytes(int r, int W, size_t cap)
{
    switch (r) {
        case 0: return MESH_DATA_OFFSET;                          /* signals + counters */
        case 2: return cap * sizeof(uint32_t);                    /* my result shard */
        default: return (size_t)W * cap * sizeof(uint32_t);       /* inbox / result inbox */
    }
}

/* collective: every rank calls it with the same shard size */
static int mesh_ensure(struct inccl_communicator *c, size_t shard)
{
    struct inccl_group *g = c->group;
    const int W = g->world_size, me = g->rank;
    if (c->mesh_buf && c->mesh_cap >= shard) return 0;
    if (W > INCCL_MAX_LOCAL_INPUTS)
        return inccl_set_error(INCCL_ERR_ARG, "mesh engine supports up to %d GPUs", INCCL_MAX_LOCAL_INPUTS);
    const size_t cap = (shard + ((size_t)1 << 19) - 1) & ~(((size_t)1 << 19) - 1);   /* 2 MiB granules */
    /* every rank computes the same sizes, so every rank refuses alike */
    if (mesh_region_bytes(1, W, cap) > g->ipc_max_bytes)
        return inccl_set_error(INCCL_ERR_ARG, "mesh: a %zu-element shard needs a %zu-byte inbox; this group's IPC "
                               "buffers stay below %zu bytes (under PyTorch's bundled HSA runtime, importing a larger "
                               "one hangs; runtime.c)", shard, mesh_region_bytes(1, W, cap), g->ipc_max_bytes);
    /* make before break (as p2p_ensure): the old buffers stay alive, and mapped
     * by the peers, until every rank has mapped the new ones */
    struct inccl_communicator old = *c;
    if (c->mesh_buf) {   /* everyone's queued accesses to the old buffers drain first */
        MTRACE("mesh regrow %zu -> %zu: device sync", c->mesh_cap, shard);
        INCCL_HIP(hipDeviceSynchronize());
        int rc = inccl_boot_barrier(g);
        if (rc) return rc;
        c->mesh_buf = NULL;
        c->mesh_err_host = NULL;
        c->mesh_err_dev = NULL;
        c->mesh_cap = 0;
        memset(c->mesh_reg, 0, sizeof(c->mesh_reg));
        memset(c->mesh_peer, 0, sizeof(c->mesh_peer));
    }
    const int dev = g->device >= 0 ? g->device : 0;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    mesh_peer_info mine, *all = (mesh_peer_info *)calloc((size_t)W, sizeof(mesh_peer_info));
    if (!all) {
        inccl_mesh_release(&old);
        return inccl_set_error(INCCL_ERR_NOMEM, "mesh: out of memory");
    }
    memset(&mine, 0, sizeof(mine));
    int rc = 0;
    /* local failures are carried to the collective outcome check below.  Four
     * separate allocations, so that no single IPC export reaches 2 GiB for
     * buckets up to ~2 GiB at any W */
    hipError_t e = hipSuccess;
    for (int r = 0; r < INCCL_MESH_REGIONS && e == hipSuccess; ++r) {
        e = inccl_ipc_malloc((void **)&c->mesh_reg[r], mesh_region_bytes(r, W, cap));
        if (e == hipSuccess) e = hipIpcGetMemHandle(&mine.h[r], c->mesh_reg[r]);
    }
    c->mesh_buf = c->mesh_reg[0];
    if (e == hipSuccess) e = hipMemset(c->mesh_buf, 0, MESH_DATA_OFFSET);   /* flags + counters */
    if (e == hipSuccess) e = hipDeviceSynchronize();   /* zeroed before any peer maps it */
    if (e == hipSuccess) e = hipHostMalloc((void **)&c->mesh_err_host, 32 * sizeof(uint32_t), hipHostMallocMapped);
    if (e == hipSuccess) {
        for (int i = 0; i < 32; ++i) ((volatile uint32_t *)c->mesh_err_host)[i] = 0;
        e = hipHostGetDevicePointer((void **)&c->mesh_err_dev, c->mesh_err_host, 0);
    }
    if (e == hipSuccess) e = hipDeviceGetAttribute(&mine.pci_domain, hipDeviceAttributePciDomainID, dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&mine.pci_bus, hipDeviceAttributePciBusId, dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&mine.pci_dev, hipDeviceAttributePciDeviceId, dev);
    if (e != hipSuccess) rc = inccl_hip_check(e, "mesh: buffer setup");
    MTRACE("mesh alloc 4 regions, inbox %zu B (%s): allgather", mesh_region_bytes(1, W, cap),
           e == hipSuccess ? "ok" : hipGetErrorString(e));
    /* where everyone is: ranks sharing a GPU size their grids together */
    int rc_x = inccl_boot_allgather(g, &mine, all, sizeof(mesh_peer_info));
    if (rc_x) {
        free(all);
        inccl_mesh_release(c);   /* back to a clean state: the next call starts over */
        inccl_mesh_release(&old);
        return rc_x;
    }
    int sharing = 0;
    for (int j = 0; j < W; ++j)
        sharing += all[j].pci_domain == mine.pci_domain && all[j].pci_bus == mine.pci_bus &&
                   all[j].pci_dev == mine.pci_dev;
    /* two workgroups per CU; ranks sharing one GPU split those slots, so that
     * their grids co-reside (every k_mesh<R> fits two 256-lane workgroups per CU;
     * the schedule's progress argument needs each rank to keep one running) */
    const char *ge = getenv("INCCL_MESH_GRID");
    int grid = ge ? atoi(ge) : 0;
    if (grid <= 0) grid = 2 * cus / (sharing > 0 ? sharing : 1);
    if (grid < 4) grid = 4;
    for (int j = 0; j < W; ++j)
        for (int r = 0; r < INCCL_MESH_REGIONS; ++r) {
            if (j == me) {
                c->mesh_peer[r][j] = c->mesh_reg[r];
                continue;
            }
            if (rc) continue;
            void *p = NULL;
            e = hipIpcOpenMemHandle(&p, all[j].h[r], hipIpcMemLazyEnablePeerAccess);
            if (e != hipSuccess) rc = inccl_hip_check(e, "mesh: hipIpcOpenMemHandle");
            c->mesh_peer[r][j] = (char *)p;
        }
    free(all);
    /* agree on the outcome, so that every rank falls back alike */
    int32_t mine_rc = rc ? 1 : 0, all_rc[INCCL_MAX_LOCAL_INPUTS];
    MTRACE("mesh peers mapped (rc %d): agree", rc);
    int rc2 = inccl_boot_allgather(g, &mine_rc, all_rc, sizeof(int32_t));
    if (rc2) {
        inccl_mesh_release(c);
        inccl_mesh_release(&old);
        return rc2;
    }
    for (int j = 0; j < W; ++j)
        if (all_rc[j]) {
            if (!rc) rc = inccl_set_error(INCCL_ERR_HIP, "mesh: rank %d could not map the peer buffers", j);
            inccl_mesh_release(c);
            inccl_mesh_release(&old);
            return rc;
        }
    /* every peer has mapped the new buffers: the old ones can go */
    if (old.mesh_buf) {
        int rc_b = inccl_boot_barrier(g);
        inccl_mesh_release(&old);
        MTRACE("mesh: old buffers released");
        if (rc_b) return rc_b;
    }
    c->mesh_cap = cap;
    c->mesh_grid = grid;
    c->mesh_last_stream = NULL;
    if (c->mesh_timeout_ticks == 0) c->mesh_timeout_ticks = inccl_wait_ticks(g);
    return 0;
}

/* Chunk size: about 256 chunks per shard for overlap, 16-256 KiB each
 * ($INCCL_MESH_CHUNK elements overrides; agreed over the group, api.c). */
static size_t mesh_chunk(const struct inccl_communicator *c, size_t shard)
{
    size_t ch = c->mesh_chunk_env;
    if (ch == 0) {
        ch = (shard + 255) / 256;
        ch = (ch + 4095) & ~(size_t)4095;
        if (ch > 65536) ch = 65536;
    }
    ch = (ch + 63) & ~(size_t)63;
    if ((shard + ch - 1) / ch > INCCL_MESH_MAX_CHUNKS)
        ch = ((shard + INCCL_MESH_MAX_CHUNKS - 1) / INCCL_MESH_MAX_CHUNKS + 63) & ~(size_t)63;
    if (ch > shard) ch = shard;
    return ch;
}

/* After a timed-out call (epoch e, nchunks chunks): how many of its flags are
 * raised, counted by the host through both mappings of each signal array --
 * this rank's own allocation, and its IPC mapping of every peer's.  "arrived
 * from" j = my arrive[j][*] >= e; "mine at" j = arrive[me][*] in rank j's array
 * as read through my mapping of it (what my pushes wrote there); "ready" the
 * same for ready flags.  A push counted as finished whose flag is missing from
 * the receiver's own view but present through the sender's mapping would mean
 * the two mappings do not reach the same memory. */
static void mesh_flag_census(struct inccl_communicator *c, uint32_t e, uint32_t nchunks, char *out, size_t len)
{
    const int W = c->group->world_size, me = c->group->rank;
    if (nchunks == 0 || nchunks > INCCL_MESH_MAX_CHUNKS) {
        snprintf(out, len, "no flag census");
        return;
    }
    static uint32_t buf[INCCL_MESH_MAX_CHUNKS];
    int cnt[4][INCCL_MAX_LOCAL_INPUTS];
    memset(cnt, 0xff, sizeof(cnt));   /* -1: not read */
    for (int j = 0; j < W && j < INCCL_MAX_LOCAL_INPUTS; ++j) {
        const uint32_t *own = (const uint32_t *)c->mesh_buf, *peer = (const uint32_t *)c->mesh_peer[0][j];
        const uint32_t *src[4] = {own + (size_t)j * INCCL_MESH_MAX_CHUNKS,
                                  own + (size_t)(INCCL_MAX_LOCAL_INPUTS + j) * INCCL_MESH_MAX_CHUNKS,
                                  peer ? peer + (size_t)me * INCCL_MESH_MAX_CHUNKS : NULL,
                                  peer ? peer + (size_t)(INCCL_MAX_LOCAL_INPUTS + me) * INCCL_MESH_MAX_CHUNKS : NULL};
        for (int k = 0; k < 4; ++k) {
            if (!src[k] || hipMemcpy(buf, src[k], nchunks * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
                continue;
            cnt[k][j] = 0;
            for (uint32_t i = 0; i < nchunks; ++i) cnt[k][j] += (int32_t)(buf[i] - e) >= 0;
        }
    }
    static const char *const names[4] = {"arrived from", "ready from", "mine at", "my ready at"};
    size_t o = 0;
    for (int k = 0; k < 4 && o < len; ++k) {
        o += (size_t)snprintf(out + o, len - o, "%s%s [", k ? "; " : "", names[k]);
        for (int j = 0; j < W && j < INCCL_MAX_LOCAL_INPUTS && o < len; ++j)
            o += (size_t)snprintf(out + o, len - o, "%s%d", j ? "," : "", cnt[k][j]);
        if (o < len) o += (size_t)snprintf(out + o, len - o, "] of %u", nchunks);
    }
}

static int mesh_piece(struct inccl_communicator *c, int kind16, const void *const *srcs, int R, void *dst, size_t n,
                      int k, const uint32_t *amax, int scale_R, int rs, hipStream_t st)
{
    const int W = c->group->world_size, me = c->group->rank;
    const size_t shard = inccl_shard_elems(n, W);
    if (rs && shard * (size_t)W != n)
        return inccl_set_error(INCCL_ERR_ARG, "mesh reduce-scatter: %zu elements are not %d shards of 64k", n, W);
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    INCCL_HIP(hipStreamIsCapturing(st, &cap));
    const int capturing = cap != hipStreamCaptureStatusNone;
    if (capturing && (!c->mesh_buf || c->mesh_cap < shard))   /* collective setup cannot run in a capture */
        return inccl_set_error(INCCL_ERR_STATE, "mesh: make one call of this size outside graph capture first");
    /* an earlier call's failure is reported before anything else, a regrow
     * included (it would replace the error words) */
    const uint32_t err = c->mesh_err_host ? *(volatile uint32_t *)c->mesh_err_host : 0;
    if (err & INCCL_MESH_ERR_BOUNDS)   /* the kernel's per-item bounds check (inccl_mesh.hip inside()) */
        return inccl_set_error(INCCL_ERR_STATE, "mesh: an earlier call stopped at its bounds check (item %u, peer %u; "
                               "results invalid)", (err >> 8) & 0xffu, (err >> 4) & 0xfu);
    if (err) {   /* which wait expired, and this rank's progress (inccl_mesh.hip wait_flag) */
        const volatile uint32_t *e4 = (const volatile uint32_t *)c->mesh_err_host;
        char pushes[96], flags[320], clock[160];
        int o = 0;
        for (int j = 0; j < W && j < INCCL_MAX_LOCAL_INPUTS; ++j)
            o += snprintf(pushes + o, sizeof(pushes) - (size_t)o, "%s%u", j ? "," : "", e4[6 + j]);
        /* GPU clock (100 MHz / 16) in ms: timeout, call start, last push per destination */
        o = snprintf(clock, sizeof(clock), "clock ms: timeout %.3f, start %.3f, last push to", e4[15] * 1.6e-4,
                     e4[16] * 1.6e-4);
        for (int j = 0; j < W && j < INCCL_MAX_LOCAL_INPUTS && o < (int)sizeof(clock); ++j)
            o += snprintf(clock + o, sizeof(clock) - (size_t)o, "%s%.3f", j ? "," : " ", e4[17 + j] * 1.6e-4);
        mesh_flag_census(c, e4[2], e4[13], flags, sizeof(flags));
        return inccl_set_error(INCCL_ERR_STATE, "mesh: an earlier call timed out waiting for a peer (results invalid; "
                               "rank %d, %s of chunk %u, peer %u: flag %u, waited for epoch %u, re-read %u; "
                               "%u tickets taken, %u workgroups started, %u retired of %d; pushes finished per "
                               "destination [%s]; %s; %s)",
                               me, ((err >> 8) & 0xffu) == 3 ? "reduce's arrival flag" : "gather's ready flag",
                               err >> 16, (err >> 4) & 0xfu, e4[1], e4[2], e4[14], e4[3], e4[4], e4[5], c->mesh_grid,
                               pushes, flags, clock);
    }
    int rc = mesh_ensure(c, shard);
    if (rc) return rc;
    const size_t chunk = mesh_chunk(c, shard);
    const int nchunks = (int)((shard + chunk - 1) / chunk);
    /* a reduce / gather starts `lag` slots after what it waits for.  Default: the
     * whole shard, i.e. every push is taken before the first reduce and every
     * reduce before the first gather -- a workgroup waiting on a flag holds its
     * CU slot idle, and on one GPU (256 MiB, R = 2) lag = 1 / 171 / 400 / all
     * chunks ran 823 / 668 / 474 / 402 us.  Phases still overlap at their
     * seams, and both xGMI directions are busy in the push and gather phases.
     * ($INCCL_MESH_LAG slots overrides; agreed over the group, api.c.) */
    int lag = c->mesh_lag_env ? c->mesh_lag_env : nchunks;
    if (lag < 1) lag = 1;
    if (lag > nchunks) lag = nchunks;
    struct inccl_mesh_launch l;
    memset(&l, 0, sizeof(l));
    for (int r = 0; r < R; ++r) l.src[r] = (const float *)srcs[r];
    l.R = R;
    l.dst = (float *)dst;
    l.kind16 = kind16;
    l.n = n;
    l.shard = shard;
    l.chunk = chunk;
    l.inbox_stride = c->mesh_cap;
    l.nchunks = nchunks;
    l.lag = lag;
    l.grid = c->mesh_grid;
    for (int j = 0; j < W; ++j) {
        l.peer_sig[j] = (uint32_t *)c->mesh_peer[0][j];
        l.peer_inbox[j] = (uint32_t *)c->mesh_peer[1][j];
        l.peer_res[j] = (const uint32_t *)c->mesh_peer[2][j];
        l.peer_resin[j] = (uint32_t *)c->mesh_peer[3][j];
    }
    l.own_resin = l.peer_resin[me];
    l.push_res = c->mesh_push;
    l.rs = rs;
    l.own_inbox = l.peer_inbox[me];
    l.own_res = (uint32_t *)l.peer_res[me];
    l.own_sig = (const uint32_t *)c->mesh_buf;
    l.ctr = (uint32_t *)(c->mesh_buf + MESH_CTR_OFFSET);
    l.err = c->mesh_err_dev;
    l.W = W;
    l.me = me;
    l.timeout_ticks = c->mesh_timeout_ticks;
    l.scale_exp = k;
    l.amax_bits = amax;
    l.scale_R = scale_R;
    l.out_shift = c->out_shift;
    const size_t es = kind16 ? sizeof(uint16_t) : sizeof(float);   /* source and result element bytes */
    l.src_bytes = n * es;
    l.dst_bytes = (rs ? shard : n) * es;
    l.inbox_bytes = mesh_region_bytes(1, W, c->mesh_cap);
    l.res_bytes = mesh_region_bytes(2, W, c->mesh_cap);
    l.resin_bytes = mesh_region_bytes(3, W, c->mesh_cap);
    /* the buffer-reuse argument needs this rank's calls in order: chain across
     * streams (inside a capture the caller's capture stream orders them) */
    if (!capturing && c->mesh_last_stream && c->mesh_last_stream != st) INCCL_HIP(hipStreamWaitEvent(st, c->ev[6], 0));
    MTRACE("mesh launch n %zu shard %zu chunk %zu nchunks %d lag %d grid %d", n, shard, chunk, nchunks, lag, l.grid);
    rc = inccl_k_mesh(&l, st);
    if (rc) return inccl_set_error(rc == INCCL_ERR_ARG ? INCCL_ERR_ARG : INCCL_ERR_HIP, "mesh kernel launch failed (%d)", rc);
    if (!capturing) {
        INCCL_HIP(hipEventRecord(c->ev[6], st));
        c->mesh_last_stream = st;
    }
    return 0;
}

int inccl_mesh_piece(struct inccl_communicator *c, const float *const *srcs, int R, float *dst, size_t n, int k,
                     const uint32_t *amax, int scale_R, hipStream_t st)
{
    return mesh_piece(c, 0, (const void *const *)srcs, R, dst, n, k, amax, scale_R, 0, st);
}

/* reduce-scatter (inccl_reduce_scatter_*): the same kernel and the same
 * instructions as the allreduce, with the gathers of other ranks' chunks reduced
 * to their flag waits and gather(c, me) copying this rank's own result chunk
 * into dst (its n / W elements, n % (64 W) == 0); kind INCCL_KIND_F32, BF16 or
 * F16 */
int inccl_mesh_reduce_scatter(struct inccl_communicator *c, int kind, const void *const *srcs, int R, void *dst,
                              size_t n, int k, const uint32_t *amax, int scale_R, hipStream_t st)
{
    return mesh_piece(c, kind == INCCL_KIND_F32 ? 0 : kind, srcs, R, dst, n, k, amax, scale_R, 1, st);
}

/* bf16 / fp16 buckets: the same kernel with 2-byte sources, int32 partials and a
 * 2-byte result, so the xGMI bytes are 4 + 2 per element instead of 4 + 4 */
int inccl_mesh_piece16(struct inccl_communicator *c, int kind, const uint16_t *const *srcs, int R, uint16_t *dst,
                       size_t n, int k, const uint32_t *amax, int scale_R, hipStream_t st)
{
    if (kind != INCCL_KIND_BF16 && kind != INCCL_KIND_F16) return inccl_set_error(INCCL_ERR_ARG, "mesh: bad kind %d", kind);
    return mesh_piece(c, kind, (const void *const *)srcs, R, dst, n, k, amax, scale_R, 0, st);
}
