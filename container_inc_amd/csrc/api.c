/* api.c -- libinccl_amd host API (C11).
 *
 * Drop-in implementation of repository/include/api.h:93-101 plus the additive
 * MI355X entry points of include/inccl_amd.h.  Host code only: every byte of
 * arithmetic runs in the HIP kernels behind inccl_kernels.h or in RCCL.
 * There is no CPU fallback: without a usable GPU the calls fail. */
#define _GNU_SOURCE
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "inccl_internal.h"
#include "inccl_kernels.h"

/* ------------------------------------------------------------------ */
/* errors                                                               */
/* ------------------------------------------------------------------ */
static __thread char g_err[1536];

int inccl_set_error(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    if (getenv("INCCL_DEBUG")) fprintf(stderr, "[inccl] %s\n", g_err);
    return code;
}

int inccl_hip_check(hipError_t e, const char *what)
{
    return inccl_set_error(INCCL_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

const char *inccl_last_error(void) { return g_err; }

const char *inccl_version(void) { return "inccl-amd 0.1.0 gfx950"; }

int inccl_ensure_dev(void **p, size_t *cur, size_t need)
{
    if (*p && *cur >= need) return 0;
    if (*p) {
        INCCL_HIP(hipDeviceSynchronize());
        INCCL_HIP(hipFree(*p));
        *p = NULL;
        *cur = 0;
    }
    if (need == 0) return 0;
    INCCL_HIP(hipMalloc(p, need));
    *cur = need;
    return 0;
}

/* Device memory that peers map over HIP IPC and that a running kernel polls or
 * reads after a flag (the ll and mesh engines).  Default "uncached"
 * (hipDeviceMallocUncached): every access bypasses the L2, so a remote GPU's
 * xGMI store into this HBM cannot hide behind a line this GPU's L2 cached
 * before it.  Coarse-grained hipMalloc memory is only guaranteed coherent with
 * other agents at kernel boundaries.  $INCCL_IPC_MEM = uncached | finegrained |
 * coarse selects the kind (same on every rank). */
unsigned inccl_ipc_mem_flags(void)
{
    const char *e = getenv("INCCL_IPC_MEM");
    if (e && strcmp(e, "coarse") == 0) return hipDeviceMallocDefault;
    if (e && strcmp(e, "finegrained") == 0) return hipDeviceMallocFinegrained;
    return hipDeviceMallocUncached;
}

hipError_t inccl_ipc_malloc(void **p, size_t bytes)
{
    const unsigned f = inccl_ipc_mem_flags();
    if (f == hipDeviceMallocDefault) return hipMalloc(p, bytes);
    return hipExtMallocWithFlags(p, bytes, f);
}

int inccl_mem_kind(const void *p)
{
    if (!p) return inccl_set_error(INCCL_ERR_ARG, "mem_kind: NULL pointer");
    hipPointerAttribute_t a;
    memset(&a, 0, sizeof(a));
    INCCL_HIP(hipPointerGetAttributes(&a, p));
    if (a.type != hipMemoryTypeDevice) return inccl_set_error(INCCL_ERR_ARG, "mem_kind: not device memory");
    return (int)a.allocationFlags;
}

/* ------------------------------------------------------------------ */
/* stateless device API                                                 */
/* ------------------------------------------------------------------ */
static int kerr(int rc)
{
    if (rc == 0) return 0;
    if (rc == INCCL_ERR_ARG) return inccl_set_error(rc, "invalid argument");
    return inccl_set_error(INCCL_ERR_HIP, "kernel launch failed: %s", hipGetErrorString((hipError_t)rc));
}

int inccl_stream_op(int in_kind, int out_kind, const void *const *srcs_dev, int R, void *dst_dev, size_t n,
                    int scale_exp, const uint32_t *amax_bits_dev, int scale_R, void *stream)
{
    if (!srcs_dev) return inccl_set_error(INCCL_ERR_ARG, "srcs is NULL");
    return kerr(inccl_k_stream(in_kind, out_kind, srcs_dev, R, dst_dev, n, scale_exp, amax_bits_dev, scale_R, stream));
}

/* ---- ordering across caller streams ----
 * A communicator's calls share its workspaces (the int32 partials, the auto
 * scale's max word, the gather buffer).  A call that uses one (inccl_ws_claim,
 * before its first use) on another stream than the last such call's first
 * waits for that call's end: ev[9], recorded at the end of every call that
 * claimed the workspaces (an event outlives its stream, so the caller may have
 * dropped the previous stream since).  Calls that touch no shared workspace --
 * the single-GPU fused kernel at a fixed scale, the IPC engines on their own
 * buffers -- record nothing: an event between back-to-back kernels costs the
 * GPU about 3 us.  Captured calls are left to the capture's own order. */
int inccl_ws_claim(struct inccl_communicator *c, hipStream_t st)
{
    if (c->ws_claimed) return 0;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    INCCL_HIP(hipStreamIsCapturing(st, &cs));
    c->ws_capturing = cs != hipStreamCaptureStatusNone;
    if (!c->ws_capturing && c->ws_last_stream && c->ws_last_stream != st)
        INCCL_HIP(hipStreamWaitEvent(st, c->ev[9], 0));
    c->ws_claimed = 1;
    c->ws_stream = st;
    return 0;
}

static int ws_leave(struct inccl_communicator *c, int rc)
{
    /* recorded on failure too: work the failed call already queued on its
     * stream (absmax into d_words, quantise into d_q32, ...) may still run, and
     * the next call on another stream must not write those workspaces under it.
     * A failure keeps its own rc. */
    if (c->ws_claimed && !c->ws_capturing) {
        const hipError_t e = hipEventRecord(c->ev[9], c->ws_stream);
        if (e == hipSuccess) c->ws_last_stream = c->ws_stream;
        else if (rc == 0) rc = inccl_hip_check(e, "hipEventRecord(workspace order)");
    }
    c->ws_claimed = 0;
    return rc;
}

#define INCCL_ORDERED(c, stream, call)                              \
    do {                                                            \
        if (!(c)) return (call);                                    \
        (c)->ws_claimed = 0;                                        \
        (c)->stage_cnt = 0;                                         \
        return ws_leave((c), (call));                               \
    } while (0)

/* ---- per-stage timing (inccl_comm_set_stage_timing) ----
 * stage_open records a begin event on the stage's stream and returns its slot
 * (-1: timing off, the stream is being captured, or the slots are full);
 * stage_close records the matching end event.  Failures to record only drop
 * the sample: timing never changes a call's outcome. */
static int stage_open(struct inccl_communicator *c, hipStream_t st)
{
    if (!c->stage_on || c->stage_cnt >= INCCL_STAGE_SLOTS) return -1;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return -1;
    const int i = c->stage_cnt;
    for (int e = 2 * i; e < 2 * i + 2; ++e)
        if (!c->stage_ev[e] && hipEventCreate(&c->stage_ev[e]) != hipSuccess) return -1;
    if (hipEventRecord(c->stage_ev[2 * i], st) != hipSuccess) return -1;
    c->stage_kind[i] = -1;   /* closed by stage_close */
    c->stage_cnt = i + 1;
    return i;
}

static void stage_close(struct inccl_communicator *c, int i, hipStream_t st, int kind)
{
    if (i < 0) return;
    if (hipEventRecord(c->stage_ev[2 * i + 1], st) == hipSuccess) c->stage_kind[i] = kind;
}

int inccl_comm_set_stage_timing(struct inccl_communicator *comm, int on)
{
    if (!comm) return inccl_set_error(INCCL_ERR_ARG, "communicator is NULL");
    comm->stage_on = on != 0;
    comm->stage_cnt = 0;
    return 0;
}

int inccl_comm_stage_times(struct inccl_communicator *comm, double *us, int kinds, double *wall_us)
{
    if (!comm || (!us && kinds > 0) || kinds < 0) return inccl_set_error(INCCL_ERR_ARG, "bad stage_times args");
    for (int k = 0; k < kinds; ++k) us[k] = 0.0;
    if (wall_us) *wall_us = 0.0;
    int n = 0;
    double t0 = 0.0, t1 = 0.0;
    /* every event against the first begin event: stage 0 opens on the call's
     * stream before any other stage starts (the side stream waits for it) */
    for (int i = 0; i < comm->stage_cnt; ++i) {
        if (comm->stage_kind[i] < 0) continue;
        INCCL_HIP(hipEventSynchronize(comm->stage_ev[2 * i + 1]));
        float b = 0.f, e = 0.f;
        INCCL_HIP(hipEventElapsedTime(&b, comm->stage_ev[0], comm->stage_ev[2 * i]));
        INCCL_HIP(hipEventElapsedTime(&e, comm->stage_ev[0], comm->stage_ev[2 * i + 1]));
        if (comm->stage_kind[i] < kinds) us[comm->stage_kind[i]] += ((double)e - (double)b) * 1e3;
        if (n == 0 || b < t0) t0 = b;
        if (n == 0 || e > t1) t1 = e;
        ++n;
    }
    if (wall_us) *wall_us = (t1 - t0) * 1e3;
    return n;
}

/* ---- prepared stream ops ---- */
struct inccl_op {
    struct inccl_communicator *comm;   /* NULL: a stream op; else an allreduce of comm (in_kind: its format) */
    int in_kind, out_kind, R, scale_exp, scale_R, chunks;
    const void *srcs[INCCL_MAX_LOCAL_INPUTS];
    void *dst;
    size_t n;
    void *stream;
};

static int kind_pair_ok(int in_kind, int out_kind)
{
    const int plain = (in_kind == INCCL_KIND_F32 || in_kind == INCCL_KIND_Q32 || in_kind == INCCL_KIND_Q32BE) &&
                      (out_kind == INCCL_KIND_F32 || out_kind == INCCL_KIND_Q32 || out_kind == INCCL_KIND_Q32BE);
    int half = 0;
    for (int h = INCCL_KIND_BF16; h <= INCCL_KIND_F16; ++h)
        half = half || (in_kind == h && (out_kind == h || out_kind == INCCL_KIND_Q32)) ||
               (in_kind == INCCL_KIND_Q32 && out_kind == h);
    return plain || half;
}

struct inccl_op *inccl_op_create(int in_kind, int out_kind, const void *const *srcs_dev, int R, void *dst_dev,
                                 size_t n, int scale_exp, int scale_R, void *stream)
{
    if (!kind_pair_ok(in_kind, out_kind) || !srcs_dev || R < 1 || R > INCCL_MAX_LOCAL_INPUTS ||
        (n > 0 && !dst_dev) || scale_exp < INCCL_SCALE_MIN || scale_exp > INCCL_SCALE_MAX || scale_R < 0) {
        inccl_set_error(INCCL_ERR_ARG, "inccl_op_create: invalid argument");
        return NULL;
    }
    for (int r = 0; r < R; ++r)
        if (!srcs_dev[r] && n > 0) {
            inccl_set_error(INCCL_ERR_ARG, "inccl_op_create: srcs[%d] is NULL", r);
            return NULL;
        }
    struct inccl_op *op = (struct inccl_op *)calloc(1, sizeof(*op));
    if (!op) {
        inccl_set_error(INCCL_ERR_NOMEM, "inccl_op_create: out of memory");
        return NULL;
    }
    op->in_kind = in_kind;
    op->out_kind = out_kind;
    op->R = R;
    op->scale_exp = scale_exp;
    op->scale_R = scale_R;
    for (int r = 0; r < R; ++r) op->srcs[r] = srcs_dev[r];
    op->dst = dst_dev;
    op->n = n;
    op->stream = stream;
    return op;
}

struct inccl_op *inccl_op_create_allreduce_f32(struct inccl_communicator *comm, const float *const *srcs_dev, int R,
                                               float *dst_dev, size_t n, int scale_exp, int chunks, void *stream)
{
    if (!comm) {
        inccl_set_error(INCCL_ERR_ARG, "inccl_op_create_allreduce_f32: comm is NULL");
        return NULL;
    }
    if (scale_exp == INCCL_SCALE_AUTO) {   /* the auto scale is a per-call absmax: nothing to bind */
        inccl_set_error(INCCL_ERR_ARG, "inccl_op_create_allreduce_f32: a prepared op takes a fixed scale exponent");
        return NULL;
    }
    struct inccl_op *op = inccl_op_create(INCCL_KIND_F32, INCCL_KIND_F32, (const void *const *)srcs_dev, R, dst_dev, n,
                                          scale_exp, R, stream);
    if (!op) return NULL;
    op->comm = comm;
    op->chunks = chunks;
    return op;
}

static int allreduce_16(struct inccl_communicator *c, int kind, const uint16_t *const *srcs_dev, int R,
                        uint16_t *dst_dev, size_t n, int scale_exp, void *stream);

struct inccl_op *inccl_op_create_allreduce16(struct inccl_communicator *comm, int kind,
                                             const uint16_t *const *srcs_dev, int R, uint16_t *dst_dev, size_t n,
                                             int scale_exp, void *stream)
{
    if (!comm || (kind != INCCL_KIND_BF16 && kind != INCCL_KIND_F16)) {
        inccl_set_error(INCCL_ERR_ARG, "inccl_op_create_allreduce16: comm is NULL or kind is not BF16 / F16");
        return NULL;
    }
    if (scale_exp == INCCL_SCALE_AUTO) {
        inccl_set_error(INCCL_ERR_ARG, "inccl_op_create_allreduce16: a prepared op takes a fixed scale exponent");
        return NULL;
    }
    struct inccl_op *op = inccl_op_create(kind, kind, (const void *const *)srcs_dev, R, dst_dev, n, scale_exp, R, stream);
    if (!op) return NULL;
    op->comm = comm;
    return op;
}

int inccl_op_run(struct inccl_op *op)
{
    if (!op) return inccl_set_error(INCCL_ERR_ARG, "inccl_op_run: op is NULL");
    if (op->comm && op->in_kind != INCCL_KIND_F32)
        return allreduce_16(op->comm, op->in_kind, (const uint16_t *const *)op->srcs, op->R, (uint16_t *)op->dst, op->n,
                            op->scale_exp, op->stream);
    if (op->comm)
        return inccl_allreduce_f32_pipelined(op->comm, (const float *const *)op->srcs, op->R, (float *)op->dst, op->n,
                                             op->scale_exp, op->chunks, op->stream);
    return kerr(inccl_k_stream(op->in_kind, op->out_kind, op->srcs, op->R, op->dst, op->n, op->scale_exp, NULL,
                               op->scale_R, op->stream));
}

int inccl_op_destroy(struct inccl_op *op)
{
    free(op);
    return 0;
}

int inccl_quantise_f32(const float *x_dev, int32_t *q_dev, size_t n, int scale_exp, int wire_be, void *stream)
{
    const void *s[1] = {x_dev};
    return inccl_stream_op(INCCL_KIND_F32, wire_be ? INCCL_KIND_Q32BE : INCCL_KIND_Q32, s, 1, q_dev, n, scale_exp,
                           NULL, 1, stream);
}

int inccl_dequantise_q32(const int32_t *q_dev, float *y_dev, size_t n, int scale_exp, int wire_be, void *stream)
{
    const void *s[1] = {q_dev};
    return inccl_stream_op(wire_be ? INCCL_KIND_Q32BE : INCCL_KIND_Q32, INCCL_KIND_F32, s, 1, y_dev, n, scale_exp,
                           NULL, 1, stream);
}

int inccl_reduce_f32(const float *const *srcs_dev, int R, float *dst_dev, size_t n, int scale_exp, void *stream)
{
    return inccl_stream_op(INCCL_KIND_F32, INCCL_KIND_F32, (const void *const *)srcs_dev, R, dst_dev, n, scale_exp,
                           NULL, R, stream);
}

int inccl_absmax_f32(const float *const *srcs_dev, int R, size_t n, uint32_t *amax_bits_dev, int zero_first,
                     void *stream)
{
    if (!srcs_dev) return inccl_set_error(INCCL_ERR_ARG, "srcs is NULL");
    return kerr(inccl_k_absmax(srcs_dev, R, n, amax_bits_dev, zero_first, stream));
}

int inccl_absmax_f16(const uint16_t *const *srcs_dev, int R, size_t n, uint32_t *amax_bits_dev, int zero_first,
                     void *stream)
{
    if (!srcs_dev) return inccl_set_error(INCCL_ERR_ARG, "srcs is NULL");
    return kerr(inccl_k_absmax_f16(srcs_dev, R, n, amax_bits_dev, zero_first, stream));
}

int inccl_absmax_bf16(const uint16_t *const *srcs_dev, int R, size_t n, uint32_t *amax_bits_dev, int zero_first,
                      void *stream)
{
    if (!srcs_dev) return inccl_set_error(INCCL_ERR_ARG, "srcs is NULL");
    return kerr(inccl_k_absmax_bf16(srcs_dev, R, n, amax_bits_dev, zero_first, stream));
}

int inccl_reduce_f32_auto(const float *const *srcs_dev, int R, float *dst_dev, size_t n, uint32_t *amax_word_dev,
                          void *stream)
{
    int rc = inccl_absmax_f32(srcs_dev, R, n, amax_word_dev, 1, stream);
    if (rc) return rc;
    return inccl_stream_op(INCCL_KIND_F32, INCCL_KIND_F32, (const void *const *)srcs_dev, R, dst_dev, n, 0,
                           amax_word_dev, R, stream);
}

int inccl_quant_sum_f32(const float *const *srcs_dev, int R, int32_t *dst_dev, size_t n, int scale_exp, int wire_be,
                        void *stream)
{
    return inccl_stream_op(INCCL_KIND_F32, wire_be ? INCCL_KIND_Q32BE : INCCL_KIND_Q32,
                           (const void *const *)srcs_dev, R, dst_dev, n, scale_exp, NULL, R, stream);
}

int inccl_sum_q32(const int32_t *const *srcs_dev, int R, int32_t *dst_dev, size_t n, int in_be, int out_be,
                  void *stream)
{
    return inccl_stream_op(in_be ? INCCL_KIND_Q32BE : INCCL_KIND_Q32, out_be ? INCCL_KIND_Q32BE : INCCL_KIND_Q32,
                           (const void *const *)srcs_dev, R, dst_dev, n, 0, NULL, R, stream);
}

int inccl_sum_dequant_q32(const int32_t *const *srcs_dev, int R, float *dst_dev, size_t n, int scale_exp, int in_be,
                          void *stream)
{
    return inccl_stream_op(in_be ? INCCL_KIND_Q32BE : INCCL_KIND_Q32, INCCL_KIND_F32, (const void *const *)srcs_dev,
                           R, dst_dev, n, scale_exp, NULL, R, stream);
}

int inccl_checksum_q32(const int32_t *q_dev, size_t n, uint64_t index_base, uint32_t *out_dev, int zero_first,
                       void *stream)
{
    return kerr(inccl_k_checksum(q_dev, n, index_base, out_dev, zero_first, stream));
}

int inccl_choose_scale(float absmax, int R_total)
{
    /* host twin of choose_scale() in inccl_kernels.hip */
    if (!(absmax > 0.0f)) return INCCL_SCALE_MAX;
    if (isinf(absmax)) return INCCL_SCALE_MIN;
    double t = (double)absmax * (double)(R_total > 0 ? R_total : 1);
    int e = 0;
    double m = frexp(t, &e);
    int k = (m == 0.5) ? (31 - e) : (30 - e);
    if (k < INCCL_SCALE_MIN) k = INCCL_SCALE_MIN;
    if (k > INCCL_SCALE_MAX) k = INCCL_SCALE_MAX;
    return k;
}

void inccl_set_tuning(int grid_cap, int nt_loads) { inccl_k_set_tuning(grid_cap, nt_loads); }

/* ------------------------------------------------------------------ */
/* groups                                                               */
/* ------------------------------------------------------------------ */
static int pick_device(int rank, int device)
{
    if (device >= 0) return device;
    const char *e = getenv("INCCL_DEVICE");
    if (e && *e) return atoi(e);
    e = getenv("LOCAL_RANK");
    if (e && *e) return atoi(e);
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return -1;
    return rank % n;
}

static struct inccl_group *group_alloc(int world_size, int rank, int device)
{
    if (world_size < 1 || rank < 0 || rank >= world_size) {
        inccl_set_error(INCCL_ERR_ARG, "bad world_size %d / rank %d", world_size, rank);
        return NULL;
    }
    /* INCCL_BOOTSTRAP_ONLY=1: a GPU-less group for rendezvous/barrier tests of
     * the host logic; every communicator call on it fails. */
    const char *bo = getenv("INCCL_BOOTSTRAP_ONLY");
    const int bootstrap_only = bo && atoi(bo) != 0;
    int dev = bootstrap_only ? -1 : pick_device(rank, device);
    if (dev < 0 && !bootstrap_only) {
        inccl_set_error(INCCL_ERR_HIP, "no HIP device available");
        return NULL;
    }
    if (dev >= 0) {
        hipError_t e = hipSetDevice(dev);
        if (e != hipSuccess) {
            inccl_hip_check(e, "hipSetDevice");
            return NULL;
        }
    }
    struct inccl_group *g = (struct inccl_group *)calloc(1, sizeof(*g));
    if (!g) return NULL;
    g->rank = rank;
    g->world_size = world_size;
    g->device = dev;
    g->master_fd = -1;
    g->ipc_max_bytes = inccl_ipc_local_max_bytes();   /* agreed over the ranks after the bootstrap */
    return g;
}

struct inccl_group *inccl_group_create_local(int world_size, int rank, const char *hub_name, int device)
{
    struct inccl_group *g = group_alloc(world_size, rank, device);
    if (!g) return NULL;
    g->transport = INCCL_TRANSPORT_LOCAL;
    snprintf(g->master_ip, sizeof(g->master_ip), "local");
    g->hub = inccl_hub_attach(hub_name ? hub_name : "default", world_size);
    if (!g->hub) {
        free(g);
        return NULL;
    }
    return g;
}

struct inccl_group *inccl_group_create_ex(int world_size, int rank, const char *master_ip, int port, int device)
{
    if (master_ip && strcmp(master_ip, "local") == 0) return inccl_group_create_local(world_size, rank, "default", device);
    struct inccl_group *g = group_alloc(world_size, rank, device);
    if (!g) return NULL;
    g->transport = INCCL_TRANSPORT_RCCL;
    snprintf(g->master_ip, sizeof(g->master_ip), "%s", master_ip ? master_ip : "127.0.0.1");
    if (port <= 0) {
        const char *e = getenv("INCCL_MASTER_PORT");
        port = (e && *e) ? atoi(e) : MASTER_PORT;
    }
    g->port = port;
    int rc = (world_size == 1) ? 0 : (rank == 0 ? inccl_boot_master(g) : inccl_boot_worker(g));
    if (rc == 0 && rank == 0 && g->peer_fds == NULL) {
        g->peer_fds = (int *)calloc((size_t)world_size, sizeof(int));
        for (int i = 0; g->peer_fds && i < world_size; ++i) g->peer_fds[i] = -1;
    }
    if (rc == 0 && world_size > 1) {
        /* the smallest IPC bound over the ranks (MiB), so that every rank
         * refuses an oversized IPC buffer alike: max of the complements */
        const size_t mib = g->ipc_max_bytes >> 20;
        uint32_t w = 0xFFFFFFFFu - (uint32_t)(mib < 0xFFFFFFFEu ? mib : 0xFFFFFFFEu);
        rc = inccl_group_allreduce_max_u32(g, &w);
        if (rc == 0) {
            const size_t agreed = (size_t)(0xFFFFFFFFu - w) << 20;
            if (agreed < g->ipc_max_bytes) g->ipc_max_bytes = agreed;
        }
    }
    if (rc != 0) {
        fprintf(stderr, "inccl_group_create: %s\n", inccl_last_error());
        inccl_boot_close(g);
        free(g);
        return NULL;
    }
    return g;
}

struct inccl_group *inccl_group_create(int world_size, int rank, const char *master_ip)
{
    return inccl_group_create_ex(world_size, rank, master_ip, 0, -1);
}

int inccl_group_destroy(struct inccl_group *group)
{
    if (group) {
        inccl_boot_close(group);
        inccl_hub_detach(group->hub);
        free(group);
    }
    return 1;   /* api.c:151-154 returns 1 */
}

int inccl_group_rank(const struct inccl_group *g) { return g ? g->rank : -1; }
int inccl_group_size(const struct inccl_group *g) { return g ? g->world_size : -1; }
int inccl_group_device(const struct inccl_group *g) { return g ? g->device : -1; }
const char *inccl_group_transport(const struct inccl_group *g)
{
    return (g && g->transport == INCCL_TRANSPORT_LOCAL) ? "local" : "rccl";
}

/* ------------------------------------------------------------------ */
/* communicators                                                        */
/* ------------------------------------------------------------------ */

/* The knobs that pick a call's route or schedule come from each process's
 * environment.  Ranks that read different values would take different routes
 * for the same call (one rank the mesh kernel, another the p2p pull-reduce; one
 * ncclAllReduce, another ncclReduceScatter + ncclAllGather): mismatched
 * barriers or collectives, a hang or wrong shards.  So the group agrees on them
 * once, here, as inccl_group_create_ex does for the IPC bound: thresholds and
 * switches take the group minimum (a route is used only where every rank
 * allows it), and INCCL_ENGINE must name the same engine on every rank. */
typedef struct {
    uint64_t ll_max_bytes, rccl_ar_bytes, mesh_chunk;
    int32_t mesh_rs, force_sharded, mesh_lag, host_chunk_mib;
    char engine[16];
} comm_knobs;

static int agree_knobs(struct inccl_communicator *c, const char *eng)
{
    struct inccl_group *g = c->group;
    comm_knobs mine, *all = (comm_knobs *)calloc((size_t)g->world_size, sizeof(comm_knobs));
    if (!all) return inccl_set_error(INCCL_ERR_NOMEM, "communicator: out of memory");
    memset(&mine, 0, sizeof(mine));
    mine.ll_max_bytes = c->ll_max_bytes;
    mine.rccl_ar_bytes = c->rccl_ar_bytes;
    mine.mesh_chunk = c->mesh_chunk_env;
    mine.mesh_rs = c->mesh_rs;
    mine.force_sharded = c->force_sharded;
    mine.mesh_lag = c->mesh_lag_env;
    mine.host_chunk_mib = c->host_chunk_mib;
    snprintf(mine.engine, sizeof(mine.engine), "%s", eng ? eng : "");
    int rc = inccl_boot_allgather(g, &mine, all, sizeof(comm_knobs));
    for (int j = 0; !rc && j < g->world_size; ++j) {
        const comm_knobs *k = &all[j];
        if (strncmp(k->engine, mine.engine, sizeof(mine.engine)) != 0) {
            rc = inccl_set_error(INCCL_ERR_ARG, "INCCL_ENGINE differs across ranks (rank %d: \"%.15s\", rank %d: \"%.15s\")",
                                 g->rank, mine.engine, j, k->engine);
            break;
        }
        if (k->ll_max_bytes < c->ll_max_bytes) c->ll_max_bytes = (size_t)k->ll_max_bytes;
        if (k->rccl_ar_bytes < c->rccl_ar_bytes) c->rccl_ar_bytes = (size_t)k->rccl_ar_bytes;
        if (k->mesh_chunk < c->mesh_chunk_env) c->mesh_chunk_env = (size_t)k->mesh_chunk;
        if (k->mesh_rs < c->mesh_rs) c->mesh_rs = k->mesh_rs;
        if (k->force_sharded < c->force_sharded) c->force_sharded = k->force_sharded;
        if (k->mesh_lag < c->mesh_lag_env) c->mesh_lag_env = k->mesh_lag;
        if (k->host_chunk_mib < c->host_chunk_mib) c->host_chunk_mib = k->host_chunk_mib;
    }
    free(all);
    return rc;
}

static int copy_streams_ensure(struct inccl_communicator *c);

static int comm_init(struct inccl_communicator *c, uint32_t size)
{
    struct inccl_group *g = c->group;
    if (g->device < 0) return inccl_set_error(INCCL_ERR_STATE, "group has no device (bootstrap-only)");
    INCCL_HIP(hipSetDevice(g->device));
    /* api.c:164 registers 2*size bytes per direction.  Here those pinned
     * buffers only serve the staged host pipeline ($INCCL_HOST_STAGING=pool),
     * which allocates them on first use (ensure_staging); the default path DMAs
     * the caller's memory directly.  The size still sets that pipeline's chunk,
     * capped at 16 MiB per ping-pong half (this also keeps 2*size from
     * overflowing the 32-bit field for size >= 2 GiB). */
    const uint64_t want = 2ull * (uint64_t)size;
    c->payload_buf_size = (uint32_t)(want < (32ull << 20) ? want : (32ull << 20));
    c->window_size = WINDOW_SIZE;                /* api.c:226 */
    INCCL_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    INCCL_HIP(hipStreamCreateWithFlags(&c->side_stream, hipStreamNonBlocking));
    /* the host paths' copy streams (copy_streams_ensure): made here for a
     * one-rank communicator, on first use otherwise */
    if (g->world_size == 1) {
        int rc_cs = copy_streams_ensure(c);
        if (rc_cs) return rc_cs;
    }
    for (int i = 0; i < 10; ++i) INCCL_HIP(hipEventCreateWithFlags(&c->ev[i], hipEventDisableTiming));
    INCCL_HIP(hipMalloc((void **)&c->d_words, 256));
    INCCL_HIP(hipMemset(c->d_words, 0, 256));
    c->comm_id = g->comm_seq++;
    const char *llb = getenv("INCCL_LL_MAX_BYTES");   /* small-bucket one-kernel path; 0 disables */
    c->ll_max_bytes = llb ? (size_t)strtoull(llb, NULL, 0) : ((size_t)1 << 20);
    if (c->ll_max_bytes > ((size_t)1 << 30)) c->ll_max_bytes = (size_t)1 << 30;   /* 32-bit buffer offsets */
    const char *mrs = getenv("INCCL_MESH_RS");        /* the mesh engines' own reduce-scatter route (0: off) */
    c->mesh_rs = mrs ? atoi(mrs) != 0 : 1;
    const char *arb = getenv("INCCL_RCCL_AR_BYTES");  /* rccl engine: one all-reduce up to this; 0 disables */
    c->rccl_ar_bytes = arb ? (size_t)strtoull(arb, NULL, 0) : ((size_t)1 << 20);
    const char *fs = getenv("INCCL_FORCE_SHARDED");   /* test hook: the sharded paths even at world 1 */
    c->force_sharded = fs && atoi(fs) != 0;
    const char *mce = getenv("INCCL_MESH_CHUNK");
    c->mesh_chunk_env = mce ? (size_t)strtoull(mce, NULL, 0) : 0;
    const char *mle = getenv("INCCL_MESH_LAG");
    c->mesh_lag_env = mle ? atoi(mle) : 0;
    if (c->mesh_lag_env < 0) c->mesh_lag_env = 0;
    const char *hce = getenv("INCCL_HOST_CHUNK_MIB");
    c->host_chunk_mib = hce ? atoi(hce) : 0;
    if (c->host_chunk_mib < 1 || c->host_chunk_mib > 1024) c->host_chunk_mib = 16;
    const char *eng = getenv("INCCL_ENGINE");
    if (g->transport == INCCL_TRANSPORT_RCCL && g->world_size > 1) {
        int rc = agree_knobs(c, eng);
        if (rc) return rc;
    }
    if (eng && *eng && g->transport == INCCL_TRANSPORT_RCCL) {
        int rc = inccl_comm_set_engine(c, eng);
        if (rc) return rc;
    }
    /* RCCL communicator up front (errors surface at creation), unless the p2p
     * engine was chosen: then RCCL is created on first use, if ever */
    if (g->transport == INCCL_TRANSPORT_RCCL && c->engine == INCCL_ENGINE_RCCL) {
        const char *force = getenv("INCCL_FORCE_RCCL");
        if (g->world_size > 1 || (force && atoi(force) != 0)) {
            int rc = inccl_rccl_comm_init(c);
            if (g->world_size > 1) {
                /* agree on the outcome: if RCCL cannot come up on every rank (e.g.
                 * ranks sharing one GPU), every rank switches to the IPC p2p
                 * engine alike; the rccl engine can still be selected later and
                 * then reports its own error */
                int32_t mine = rc ? 1 : 0;
                int32_t *all = (int32_t *)calloc((size_t)g->world_size, sizeof(int32_t));
                if (!all) return inccl_set_error(INCCL_ERR_NOMEM, "communicator: out of memory");
                int rc2 = inccl_boot_allgather(g, &mine, all, sizeof(int32_t));
                int failed = -1;
                for (int j = 0; !rc2 && j < g->world_size; ++j)
                    if (all[j] && failed < 0) failed = j;
                free(all);
                if (rc2) return rc2;
                if (failed >= 0) {
                    fprintf(stderr, "inccl: RCCL communicator unavailable on rank %d%s%s; using the p2p engine\n",
                            failed, rc ? ": " : "", rc ? inccl_last_error() : "");
                    inccl_rccl_comm_destroy(c);
                    c->engine = INCCL_ENGINE_P2P;
                }
            } else if (rc) {
                return rc;
            }
        }
    }
    /* int32 workspace of one bucket of `size` bytes up front */
    if (size) {
        int rc = inccl_ensure_dev(&c->d_q32, &c->d_q32_bytes, (size_t)size);
        if (rc) return rc;
    }
    return 0;
}

int inccl_communicator_destroy(struct inccl_communicator *comm)
{
    if (!comm) return 0;
    if (comm->group->device >= 0) hipSetDevice(comm->group->device);
    if (comm->stream) hipStreamSynchronize(comm->stream);
    if (comm->p2p_part || comm->ll_buf || comm->mesh_buf) {   /* peers may still be reading our IPC buffers */
        hipDeviceSynchronize();   /* our queued reads of theirs have drained ... */
        inccl_boot_barrier(comm->group);   /* ... and so have everyone else's */
        inccl_p2p_release(comm);
        inccl_ll_release(comm);
        inccl_mesh_release(comm);
    }
    inccl_rccl_comm_destroy(comm);
    if (comm->copy_streams[0]) hipStreamSynchronize(comm->copy_streams[0]);
    if (comm->copy_streams[1]) hipStreamSynchronize(comm->copy_streams[1]);
    for (int i = 0; i < comm->nreg; ++i) hipHostUnregister(comm->reg[i].p);
    comm->nreg = 0;
    if (comm->d_q32) hipFree(comm->d_q32);
    if (comm->d_f32) hipFree(comm->d_f32);
    if (comm->d_stage) hipFree(comm->d_stage);
    if (comm->d_words) hipFree(comm->d_words);
    inccl_copy_pool_destroy(comm->pool);
    inccl_d2h_worker_destroy(comm->d2h);
    if (comm->send_payload) hipHostFree(comm->send_payload);
    if (comm->receive_payload) hipHostFree(comm->receive_payload);
    for (int i = 0; i < 10; ++i)
        if (comm->ev[i]) hipEventDestroy(comm->ev[i]);
    for (int i = 0; i < 2 * INCCL_STAGE_SLOTS; ++i)
        if (comm->stage_ev[i]) hipEventDestroy(comm->stage_ev[i]);
    if (comm->copy_streams[0]) hipStreamDestroy(comm->copy_streams[0]);
    if (comm->copy_streams[1]) hipStreamDestroy(comm->copy_streams[1]);
    if (comm->side_stream) hipStreamDestroy(comm->side_stream);
    if (comm->stream) hipStreamDestroy(comm->stream);
    free(comm);
    return 0;
}

struct inccl_communicator *inccl_communicator_create(struct inccl_group *group, uint32_t size)
{
    if (!group) {
        inccl_set_error(INCCL_ERR_ARG, "group is NULL");
        return NULL;
    }
    struct inccl_communicator *c = (struct inccl_communicator *)calloc(1, sizeof(*c));
    if (!c) return NULL;
    c->group = group;
    int rc = comm_init(c, size);
    if (rc) {
        fprintf(stderr, "inccl_communicator_create: %s\n", inccl_last_error());
        inccl_communicator_destroy(c);
        return NULL;
    }
    return c;
}

void *inccl_comm_stream(struct inccl_communicator *comm) { return comm ? (void *)comm->stream : NULL; }

int inccl_comm_set_engine(struct inccl_communicator *comm, const char *name)
{
    if (!comm || !name) return inccl_set_error(INCCL_ERR_ARG, "bad set_engine args");
    if (strcmp(name, "rccl") == 0) {
        comm->engine = INCCL_ENGINE_RCCL;
        return 0;
    }
    if (strcmp(name, "a2a") == 0) {
        if (comm->group->transport != INCCL_TRANSPORT_RCCL)
            return inccl_set_error(INCCL_ERR_ARG, "a2a engine needs a multi-process (rccl) group");
        comm->engine = INCCL_ENGINE_A2A;
        return 0;
    }
    if (strcmp(name, "p2p") == 0) {
        if (comm->group->transport != INCCL_TRANSPORT_RCCL)
            return inccl_set_error(INCCL_ERR_ARG, "p2p engine needs a multi-process (rccl) group");
        comm->engine = INCCL_ENGINE_P2P;
        return 0;
    }
    if (strcmp(name, "mesh") == 0 || strcmp(name, "meshw") == 0) {
        if (comm->group->transport != INCCL_TRANSPORT_RCCL)
            return inccl_set_error(INCCL_ERR_ARG, "mesh engine needs a multi-process (rccl) group");
        comm->engine = INCCL_ENGINE_MESH;
        comm->mesh_push = name[4] == 'w';
        return 0;
    }
    if (strcmp(name, "ar") == 0) {
        comm->engine = INCCL_ENGINE_AR;
        return 0;
    }
    if (strcmp(name, "ll") == 0) {
        if (comm->group->transport != INCCL_TRANSPORT_RCCL)
            return inccl_set_error(INCCL_ERR_ARG, "ll engine needs a multi-process (rccl) group");
        if (comm->ll_max_bytes == 0) return inccl_set_error(INCCL_ERR_ARG, "ll engine disabled (INCCL_LL_MAX_BYTES=0)");
        comm->engine = INCCL_ENGINE_LL;
        return 0;
    }
    return inccl_set_error(INCCL_ERR_ARG, "unknown engine '%s' (rccl | ar | a2a | p2p | ll | mesh | meshw)", name);
}

const char *inccl_comm_engine(const struct inccl_communicator *comm)
{
    if (!comm) return "";
    if (comm->group->transport == INCCL_TRANSPORT_LOCAL) return "local";
    switch (comm->engine) {
        case INCCL_ENGINE_P2P: return "p2p";
        case INCCL_ENGINE_A2A: return "a2a";
        case INCCL_ENGINE_LL: return "ll";
        case INCCL_ENGINE_MESH: return comm->mesh_push ? "meshw" : "mesh";
        case INCCL_ENGINE_AR: return "ar";
        default: return "rccl";
    }
}

int inccl_comm_barrier(struct inccl_communicator *comm)
{
    if (!comm) return inccl_set_error(INCCL_ERR_ARG, "comm is NULL");
    return inccl_tp_barrier(comm);
}

int inccl_comm_ipc_mem_kind(struct inccl_communicator *comm, const char *engine)
{
    if (!comm || !engine) return inccl_set_error(INCCL_ERR_ARG, "bad ipc_mem_kind args");
    const void *p = NULL;
    if (strcmp(engine, "ll") == 0) p = comm->ll_buf;
    else if (strcmp(engine, "mesh") == 0 || strcmp(engine, "meshw") == 0) p = comm->mesh_reg[1];   /* the inbox */
    else if (strcmp(engine, "p2p") == 0) p = comm->p2p_part;
    else return inccl_set_error(INCCL_ERR_ARG, "ipc_mem_kind: unknown engine '%s' (ll | mesh | p2p)", engine);
    if (!p) return inccl_set_error(INCCL_ERR_STATE, "ipc_mem_kind: engine '%s' has no IPC buffer yet", engine);
    if (comm->group->device >= 0) INCCL_HIP(hipSetDevice(comm->group->device));
    return inccl_mem_kind(p);
}

int inccl_comm_set_average(struct inccl_communicator *comm, int on)
{
    if (!comm) return inccl_set_error(INCCL_ERR_ARG, "NULL communicator");
    const int W = comm->group->world_size;
    if (!on) {
        comm->out_shift = 0;
        return 0;
    }
    if (W & (W - 1))
        return inccl_set_error(INCCL_ERR_ARG, "set_average: world %d is not a power of two (the mean would round)", W);
    int s = 0;
    while ((1 << s) < W) ++s;
    comm->out_shift = s;
    return 0;
}

int inccl_comm_set_nonfinite(struct inccl_communicator *comm, int mode)
{
    if (!comm) return inccl_set_error(INCCL_ERR_ARG, "NULL communicator");
    if (mode != INCCL_NONFINITE_SATURATE && mode != INCCL_NONFINITE_NAN)
        return inccl_set_error(INCCL_ERR_ARG, "set_nonfinite: unknown mode %d", mode);
    comm->nonfinite = mode;
    return 0;
}

int inccl_comm_clear_error(struct inccl_communicator *comm)
{
    if (!comm) return inccl_set_error(INCCL_ERR_ARG, "comm is NULL");
    if (comm->group->transport != INCCL_TRANSPORT_RCCL || comm->group->world_size == 1) return 0;
    INCCL_HIP(hipSetDevice(comm->group->device));
    const int had = (comm->ll_err_host && *(volatile uint32_t *)comm->ll_err_host) ||
                    (comm->mesh_err_host && *(volatile uint32_t *)comm->mesh_err_host);
    /* every rank's kernels have finished (a timed-out kernel finishes by itself)
     * and nobody reads a peer's buffer any more: drop them; the next ll / mesh
     * call allocates, zeroes and exchanges fresh ones */
    INCCL_HIP(hipDeviceSynchronize());
    int rc = inccl_boot_barrier(comm->group);
    if (rc) return rc;
    inccl_ll_release(comm);
    inccl_mesh_release(comm);
    rc = inccl_boot_barrier(comm->group);
    if (rc) return rc;
    return had;
}

/* ------------------------------------------------------------------ */
/* device-resident collectives                                          */
/* ------------------------------------------------------------------ */
static int allreduce_q32_body(struct inccl_communicator *c, const int32_t *src_dev, int32_t *dst_dev, size_t n,
                              void *stream)
{
    if (!c || (!src_dev && n) || (!dst_dev && n)) return inccl_set_error(INCCL_ERR_ARG, "bad allreduce_q32 args");
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    if (n == 0) return 0;
    return inccl_tp_allreduce_q32(c, src_dev, dst_dev, n, st);
}

int inccl_allreduce_q32(struct inccl_communicator *c, const int32_t *src_dev, int32_t *dst_dev, size_t n,
                        void *stream)
{
    INCCL_ORDERED(c, stream, allreduce_q32_body(c, src_dev, dst_dev, n, stream));
}

/* Variant B: quant + local sum -> grouped ncclSend/Recv of
 * int32 shards -> this library's fused sum over the W received shards +
 * dequantise (the switch aggregate, non_termination_switch.c:361-363, fused with
 * the back stage) -> ncclAllGather.  `ws` holds W*shard (send) + W*shard (recv). */
static int allreduce_piece_a2a(struct inccl_communicator *c, const float *const *srcs, int R, float *dst, size_t n,
                               int k, const uint32_t *amax, int scale_R, int32_t *ws, float *fws, hipStream_t st)
{
    const int W = c->group->world_size, me = c->group->rank;
    const size_t shard = inccl_shard_elems(n, W), total = shard * (size_t)W;
    int32_t *qsend = ws, *qrecv = ws + total;
    int rc = kerr(inccl_k_stream(INCCL_KIND_F32, INCCL_KIND_Q32, (const void *const *)srcs, R, qsend, n, k, amax,
                                 scale_R, st));
    if (rc) return rc;
    if (total > n) INCCL_HIP(hipMemsetAsync(qsend + n, 0, (total - n) * sizeof(int32_t), st));
    rc = inccl_rccl_alltoall_q32(c, qsend, qrecv, shard, st);
    if (rc) return rc;
    const void *parts[INCCL_MAX_LOCAL_INPUTS];
    for (int j = 0; j < W; ++j) parts[j] = (j == me) ? (const void *)(qsend + (size_t)me * shard)
                                                      : (const void *)(qrecv + (size_t)j * shard);
    const size_t lo = (size_t)me * shard;
    const int in_place = (total == n);
    float *gather = in_place ? dst : fws;
    rc = kerr(inccl_k_stream_s(INCCL_KIND_Q32, INCCL_KIND_F32, parts, W, gather + lo, shard, k, amax, scale_R,
                               c->out_shift, st));
    if (rc) return rc;
    rc = inccl_tp_all_gather_f32(c, gather + lo, gather, shard, st);
    if (rc) return rc;
    if (!in_place) INCCL_HIP(hipMemcpyAsync(dst, fws, n * sizeof(float), hipMemcpyDeviceToDevice, st));
    return 0;
}

/* One bucket piece: quant + local sum -> reduce-scatter -> dequant shard ->
 * all-gather.  `ws` holds W*shard + shard int32; `fws` (if the gather cannot
 * land in dst in place) W*shard fp32. */
static int allreduce_piece(struct inccl_communicator *c, const float *const *srcs, int R, float *dst, size_t n,
                           int k, const uint32_t *amax, int scale_R, int32_t *ws, float *fws, hipStream_t st)
{
    const int W = c->group->world_size, me = c->group->rank;
    const size_t shard = inccl_shard_elems(n, W), total = shard * (size_t)W;
    int32_t *qsend = ws, *qrecv = ws + total;
    int si = stage_open(c, st);
    int rc = kerr(inccl_k_stream(INCCL_KIND_F32, INCCL_KIND_Q32, (const void *const *)srcs, R, qsend, n, k, amax,
                                 scale_R, st));
    if (rc) return rc;
    if (total > n) INCCL_HIP(hipMemsetAsync(qsend + n, 0, (total - n) * sizeof(int32_t), st));
    stage_close(c, si, st, INCCL_STAGE_QUANT);
    si = stage_open(c, st);
    rc = inccl_tp_reduce_scatter_q32(c, qsend, qrecv, shard, st);
    if (rc) return rc;
    stage_close(c, si, st, INCCL_STAGE_RS);
    const size_t lo = (size_t)me * shard;
    const int in_place = (total == n);
    float *gather = in_place ? dst : fws;
    const void *s1[1] = {qrecv};
    si = stage_open(c, st);
    rc = kerr(inccl_k_stream_s(INCCL_KIND_Q32, INCCL_KIND_F32, s1, 1, gather + lo, shard, k, amax, scale_R,
                               c->out_shift, st));
    if (rc) return rc;
    stage_close(c, si, st, INCCL_STAGE_DEQUANT);
    si = stage_open(c, st);
    rc = inccl_tp_all_gather_f32(c, gather + lo, gather, shard, st);
    if (rc) return rc;
    stage_close(c, si, st, INCCL_STAGE_AG);
    if (!in_place) {
        si = stage_open(c, st);
        INCCL_HIP(hipMemcpyAsync(dst, fws, n * sizeof(float), hipMemcpyDeviceToDevice, st));
        stage_close(c, si, st, INCCL_STAGE_COPY);
    }
    return 0;
}

/* The scale of one allreduce.  A fixed exponent passes through.  INCCL_SCALE_AUTO
 * takes the absmax of the local buckets (kind F32, BF16 or F16) and its max over
 * the group (with bit 31 set when a rank saw a NaN or +-Inf and the
 * communicator propagates them, inccl_comm_set_nonfinite).  On the IPC engines that max is agreed on the host anyway (the node's
 * shared memory), so the host also picks the exponent (inccl_choose_scale, the
 * host twin of the kernels' choose_scale): *k_out, no device word, no copy
 * back.  Otherwise the max stays on the device (*amax_out) for the kernels to
 * resolve. */
static int resolve_scale(struct inccl_communicator *c, int kind, const void *const *srcs, int R, size_t n,
                         int scale_exp, hipStream_t st, const uint32_t **amax_out, int *k_out)
{
    *amax_out = NULL;
    *k_out = scale_exp;
    if (scale_exp != INCCL_SCALE_AUTO) {
        if (scale_exp < INCCL_SCALE_MIN || scale_exp > INCCL_SCALE_MAX)
            return inccl_set_error(INCCL_ERR_ARG, "scale_exp %d out of range", scale_exp);
        return 0;
    }
    const int zf = 1 | (c->nonfinite == INCCL_NONFINITE_NAN ? INCCL_ABSMAX_FLAG_NONFINITE : 0);
    int rc = inccl_ws_claim(c, st);   /* the max word is shared by every call */
    if (rc) return rc;
    rc = kind == INCCL_KIND_BF16  ? inccl_absmax_bf16((const uint16_t *const *)srcs, R, n, c->d_words, zf, st)
             : kind == INCCL_KIND_F16 ? inccl_absmax_f16((const uint16_t *const *)srcs, R, n, c->d_words, zf, st)
                                      : inccl_absmax_f32((const float *const *)srcs, R, n, c->d_words, zf, st);
    if (rc) return rc;
    const int W = c->group->world_size;
    if (W > 1 && c->group->transport == INCCL_TRANSPORT_RCCL &&
        (c->engine == INCCL_ENGINE_P2P || c->engine == INCCL_ENGINE_LL || c->engine == INCCL_ENGINE_MESH)) {
        uint32_t v = 0;
        INCCL_HIP(hipMemcpyAsync(&v, c->d_words, sizeof(v), hipMemcpyDeviceToHost, st));
        INCCL_HIP(hipStreamSynchronize(st));
        rc = inccl_group_allreduce_max_u32(c->group, &v);
        if (rc) return rc;
        if (v >> 31) {   /* a non-finite input somewhere (INCCL_NONFINITE_NAN): the kernels see the flag */
            INCCL_HIP(hipMemcpyAsync(c->d_words, &v, sizeof(v), hipMemcpyHostToDevice, st));
            INCCL_HIP(hipStreamSynchronize(st));
            *amax_out = c->d_words;
            *k_out = 0;
            return 0;
        }
        float amax;
        memcpy(&amax, &v, sizeof(amax));
        *k_out = inccl_choose_scale(amax, R * W);
        return 0;
    }
    if (W > 1) {
        rc = inccl_tp_allreduce_max_u32(c, c->d_words, 1, st);
        if (rc) return rc;
    }
    *amax_out = c->d_words;
    *k_out = 0;
    return 0;
}

int inccl_allreduce_f32(struct inccl_communicator *c, const float *const *srcs_dev, int R, float *dst_dev, size_t n,
                        int scale_exp, void *stream)
{
    return inccl_allreduce_f32_pipelined(c, srcs_dev, R, dst_dev, n, scale_exp, 1, stream);
}

/* the rccl engine's small-bucket route: n int32 partials within rccl_ar_bytes
 * (INCCL_RCCL_AR_BYTES, default 1 MiB) go through one ncclAllReduce */
static int rccl_small(const struct inccl_communicator *c, size_t n)
{
    return c->engine == INCCL_ENGINE_RCCL && c->group->transport == INCCL_TRANSPORT_RCCL &&
           n <= c->rccl_ar_bytes / sizeof(int32_t);
}

static int allreduce_f32_body(struct inccl_communicator *c, const float *const *srcs_dev, int R, float *dst_dev,
                              size_t n, int scale_exp, int chunks, void *stream)
{
    if (!c || !srcs_dev || R < 1 || R > INCCL_MAX_LOCAL_INPUTS || (!dst_dev && n))
        return inccl_set_error(INCCL_ERR_ARG, "bad allreduce_f32 args");
    for (int r = 0; r < R; ++r)
        if (!srcs_dev[r] && n) return inccl_set_error(INCCL_ERR_ARG, "srcs[%d] is NULL", r);
    if (n == 0) return 0;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    const int W = c->group->world_size;
    const uint32_t *amax = NULL;
    int k = 0;
    int rc = resolve_scale(c, INCCL_KIND_F32, (const void *const *)srcs_dev, R, n, scale_exp, st, &amax, &k);
    if (rc) return rc;
    const int scale_R = R * W;

    if (W == 1 && !c->force_sharded)   /* one fused HBM pass: quant + sum + dequant */
        return kerr(inccl_k_stream_s(INCCL_KIND_F32, INCCL_KIND_F32, (const void *const *)srcs_dev, R, dst_dev, n, k,
                                     amax, scale_R, c->out_shift, st));

    /* the IPC engines: the ll kernel for small buckets when the ll engine was
     * chosen explicitly (ll.c), else the one-kernel mesh exchange (mesh.c) or the
     * host-synchronised p2p exchange (p2p.c).  The p2p engine (and the automatic
     * fallback to it when RCCL is unavailable) never routes to ll by itself. */
    if ((c->engine == INCCL_ENGINE_P2P || c->engine == INCCL_ENGINE_LL || c->engine == INCCL_ENGINE_MESH) &&
        c->group->transport == INCCL_TRANSPORT_RCCL) {
        const int si = stage_open(c, st);
        if (c->engine == INCCL_ENGINE_LL && n <= c->ll_max_bytes / sizeof(float) && W > 1)
            rc = inccl_ll_piece(c, srcs_dev, R, dst_dev, n, k, amax, scale_R, 0, 0, st);
        else if (c->engine == INCCL_ENGINE_MESH)
            rc = inccl_mesh_piece(c, srcs_dev, R, dst_dev, n, k, amax, scale_R, st);
        else
            rc = inccl_p2p_piece(c, srcs_dev, R, dst_dev, n, k, amax, scale_R, st);
        if (!rc) stage_close(c, si, st, INCCL_STAGE_IPC);
        return rc;
    }
    /* RCCL's own allreduce on the int32 partials: quant + local sum -> in-place
     * ncclAllReduce(int32, sum) -> dequantise (the switch aggregate inside RCCL).
     * The rccl engine takes it too for small buckets: one collective launch in
     * place of two where latency, not bytes, sets the time. */
    if (c->engine == INCCL_ENGINE_AR || rccl_small(c, n)) {
        rc = inccl_ws_claim(c, st);
        if (rc) return rc;
        rc = inccl_ensure_dev(&c->d_q32, &c->d_q32_bytes, n * sizeof(int32_t));
        if (rc) return rc;
        int32_t *q = (int32_t *)c->d_q32;
        int si = stage_open(c, st);
        rc = kerr(inccl_k_stream(INCCL_KIND_F32, INCCL_KIND_Q32, (const void *const *)srcs_dev, R, q, n, k, amax,
                                 scale_R, st));
        if (rc) return rc;
        stage_close(c, si, st, INCCL_STAGE_QUANT);
        si = stage_open(c, st);
        rc = inccl_tp_allreduce_q32(c, q, q, n, st);
        if (rc) return rc;
        stage_close(c, si, st, INCCL_STAGE_AR);
        si = stage_open(c, st);
        const void *s1[1] = {q};
        rc = kerr(inccl_k_stream_s(INCCL_KIND_Q32, INCCL_KIND_F32, s1, 1, dst_dev, n, k, amax, scale_R,
                                   c->out_shift, st));
        stage_close(c, si, st, INCCL_STAGE_DEQUANT);
        return rc;
    }
    if (c->engine == INCCL_ENGINE_A2A && c->group->transport == INCCL_TRANSPORT_RCCL) {
        if (W > INCCL_MAX_LOCAL_INPUTS)
            return inccl_set_error(INCCL_ERR_ARG, "a2a engine sums at most %d shards", INCCL_MAX_LOCAL_INPUTS);
        const size_t shard = inccl_shard_elems(n, W), total = shard * (size_t)W;
        rc = inccl_ws_claim(c, st);
        if (rc) return rc;
        rc = inccl_ensure_dev(&c->d_q32, &c->d_q32_bytes, 2 * total * sizeof(int32_t));
        if (rc) return rc;
        if (total != n) {
            rc = inccl_ws_claim(c, st);
            if (rc) return rc;
            rc = inccl_ensure_dev(&c->d_f32, &c->d_f32_bytes, total * sizeof(float));
            if (rc) return rc;
        }
        return allreduce_piece_a2a(c, srcs_dev, R, dst_dev, n, k, amax, scale_R, (int32_t *)c->d_q32,
                                   (float *)c->d_f32, st);
    }
    /* chunk boundaries: multiples of W*64 elements so every chunk's shards are
     * 256-B aligned inside dst; each chunk has its own workspace region */
    if (chunks < 1) chunks = 1;
    const size_t unit = (size_t)W * 64;
    size_t per = ((n + (size_t)chunks - 1) / (size_t)chunks + unit - 1) / unit * unit;
    if (per == 0) per = unit;
    size_t ws_elems = 0, fws_elems = 0;
    for (size_t off = 0; off < n; off += per) {
        const size_t cnt = (n - off) < per ? (n - off) : per;
        const size_t shard = inccl_shard_elems(cnt, W);
        ws_elems += shard * (size_t)W + shard;
        if (shard * (size_t)W != cnt) fws_elems = shard * (size_t)W;
    }
    rc = inccl_ws_claim(c, st);
    if (rc) return rc;
    rc = inccl_ensure_dev(&c->d_q32, &c->d_q32_bytes, ws_elems * sizeof(int32_t));
    if (rc) return rc;
    if (fws_elems) {
        rc = inccl_ws_claim(c, st);
        if (rc) return rc;
        rc = inccl_ensure_dev(&c->d_f32, &c->d_f32_bytes, fws_elems * sizeof(float));
        if (rc) return rc;
    }
    int32_t *ws = (int32_t *)c->d_q32;
    const float *sub[INCCL_MAX_LOCAL_INPUTS];
    if (per >= n) return allreduce_piece(c, srcs_dev, R, dst_dev, n, k, amax, scale_R, ws, (float *)c->d_f32, st);

    /* pipelined: quantise chunk i+1 on the side stream while chunk i's
     * collectives run on `st` (RCCL kernels and the HBM-bound quantiser share
     * the chip).  ev[0]: side stream caught up with st's prior work. */
    /* (stage timing: a first, empty stage on st anchors the clock before the
     * side stream starts) */
    stage_close(c, stage_open(c, st), st, INCCL_STAGE_KINDS);
    INCCL_HIP(hipEventRecord(c->ev[0], st));
    INCCL_HIP(hipStreamWaitEvent(c->side_stream, c->ev[0], 0));
    for (size_t off = 0; off < n; off += per) {
        const size_t cnt = (n - off) < per ? (n - off) : per;
        const size_t shard = inccl_shard_elems(cnt, W), total = shard * (size_t)W;
        for (int r = 0; r < R; ++r) sub[r] = srcs_dev[r] + off;
        int32_t *qsend = ws, *qrecv = ws + total;
        int si = stage_open(c, c->side_stream);
        rc = kerr(inccl_k_stream(INCCL_KIND_F32, INCCL_KIND_Q32, (const void *const *)sub, R, qsend, cnt, k, amax,
                                 scale_R, c->side_stream));
        if (rc) return rc;
        if (total > cnt) INCCL_HIP(hipMemsetAsync(qsend + cnt, 0, (total - cnt) * sizeof(int32_t), c->side_stream));
        stage_close(c, si, c->side_stream, INCCL_STAGE_QUANT);
        INCCL_HIP(hipEventRecord(c->ev[1], c->side_stream));
        INCCL_HIP(hipStreamWaitEvent(st, c->ev[1], 0));
        si = stage_open(c, st);
        rc = inccl_tp_reduce_scatter_q32(c, qsend, qrecv, shard, st);
        if (rc) return rc;
        stage_close(c, si, st, INCCL_STAGE_RS);
        const int in_place = (total == cnt);
        float *gather = in_place ? dst_dev + off : (float *)c->d_f32;
        const size_t lo = (size_t)c->group->rank * shard;
        const void *s1[1] = {qrecv};
        si = stage_open(c, st);
        rc = kerr(inccl_k_stream_s(INCCL_KIND_Q32, INCCL_KIND_F32, s1, 1, gather + lo, shard, k, amax, scale_R,
                                   c->out_shift, st));
        if (rc) return rc;
        stage_close(c, si, st, INCCL_STAGE_DEQUANT);
        si = stage_open(c, st);
        rc = inccl_tp_all_gather_f32(c, gather + lo, gather, shard, st);
        if (rc) return rc;
        stage_close(c, si, st, INCCL_STAGE_AG);
        if (!in_place) {
            si = stage_open(c, st);
            INCCL_HIP(hipMemcpyAsync(dst_dev + off, c->d_f32, cnt * sizeof(float), hipMemcpyDeviceToDevice, st));
            stage_close(c, si, st, INCCL_STAGE_COPY);
        }
        ws += total + shard;
    }
    /* `st` already waited on every side-stream chunk */
    return 0;
}

int inccl_allreduce_f32_pipelined(struct inccl_communicator *c, const float *const *srcs_dev, int R, float *dst_dev,
                                  size_t n, int scale_exp, int chunks, void *stream)
{
    INCCL_ORDERED(c, stream, allreduce_f32_body(c, srcs_dev, R, dst_dev, n, scale_exp, chunks, stream));
}

/* 2-byte buckets (kind INCCL_KIND_BF16 or INCCL_KIND_F16): the fp32 path's
 * arithmetic on the widened values.  The int32 partial sums travel as in the
 * fp32 path (the switch's aggregate, nts.c:361-363); only the result's format
 * differs, so the "rccl" engine's all-gather moves 2 bytes per element instead
 * of 4 (an all-gather copies bytes: the same one serves both formats), and the
 * mesh and p2p engines' reduce kernels narrow to the bucket's format before
 * their result exchange. */
static int allreduce_16_body(struct inccl_communicator *c, int kind, const uint16_t *const *srcs_dev, int R,
                             uint16_t *dst_dev, size_t n, int scale_exp, void *stream)
{
    if (!c || !srcs_dev || R < 1 || R > INCCL_MAX_LOCAL_INPUTS || (!dst_dev && n))
        return inccl_set_error(INCCL_ERR_ARG, "bad allreduce_%s args", kind == INCCL_KIND_F16 ? "f16" : "bf16");
    for (int r = 0; r < R; ++r)
        if (!srcs_dev[r] && n) return inccl_set_error(INCCL_ERR_ARG, "srcs[%d] is NULL", r);
    if (n == 0) return 0;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    const int W = c->group->world_size, me = c->group->rank;
    const void *const *srcs = (const void *const *)srcs_dev;
    const uint32_t *amax = NULL;
    int k = 0;
    {
        const int rc = resolve_scale(c, kind, srcs, R, n, scale_exp, st, &amax, &k);
        if (rc) return rc;
    }
    const int scale_R = R * W;
    if (W == 1 && !c->force_sharded)   /* one fused HBM pass */
        return kerr(inccl_k_stream_s(kind, kind, srcs, R, dst_dev, n, k, amax, scale_R,
                                     c->out_shift, st));

    if ((c->engine == INCCL_ENGINE_RCCL && !rccl_small(c, n)) || c->group->transport == INCCL_TRANSPORT_LOCAL) {
        /* quant + local sum -> reduce-scatter (int32) -> dequantise own shard to
         * bf16 -> all-gather (bf16), as allreduce_piece with a 2-byte result;
         * small buckets fall through to the one-all-reduce route at the end */
        const size_t shard = inccl_shard_elems(n, W), total = shard * (size_t)W;
        int rc = inccl_ws_claim(c, st);
        if (rc) return rc;
        rc = inccl_ensure_dev(&c->d_q32, &c->d_q32_bytes, (total + shard) * sizeof(int32_t));
        if (rc) return rc;
        const int in_place = (total == n);
        if (!in_place) {
            rc = inccl_ws_claim(c, st);
            if (rc) return rc;
            rc = inccl_ensure_dev(&c->d_f32, &c->d_f32_bytes, total * sizeof(uint16_t));
            if (rc) return rc;
        }
        int32_t *qsend = (int32_t *)c->d_q32, *qrecv = qsend + total;
        rc = kerr(inccl_k_stream(kind, INCCL_KIND_Q32, srcs, R, qsend, n, k, amax, scale_R, st));
        if (rc) return rc;
        if (total > n) INCCL_HIP(hipMemsetAsync(qsend + n, 0, (total - n) * sizeof(int32_t), st));
        rc = inccl_tp_reduce_scatter_q32(c, qsend, qrecv, shard, st);
        if (rc) return rc;
        uint16_t *gather = in_place ? dst_dev : (uint16_t *)c->d_f32;
        const size_t lo = (size_t)me * shard;
        const void *s1[1] = {qrecv};
        rc = kerr(inccl_k_stream_s(INCCL_KIND_Q32, kind, s1, 1, gather + lo, shard, k, amax, scale_R,
                                   c->out_shift, st));
        if (rc) return rc;
        rc = inccl_tp_all_gather_bf16(c, gather + lo, gather, shard, st);
        if (rc) return rc;
        if (!in_place) INCCL_HIP(hipMemcpyAsync(dst_dev, gather, n * sizeof(uint16_t), hipMemcpyDeviceToDevice, st));
        return 0;
    }
    /* the mesh engines: the persistent kernel with 2-byte sources and results (mesh.c) */
    if (c->engine == INCCL_ENGINE_MESH && c->group->transport == INCCL_TRANSPORT_RCCL)
        return inccl_mesh_piece16(c, kind, srcs_dev, R, dst_dev, n, k, amax, scale_R, st);
    /* the p2p engine: 2-byte result shards gathered over xGMI (p2p.c).  The
     * route never depends on this rank's dst alignment (every rank must take
     * it): a dst that is not 4-B aligned gets it into the aligned workspace and
     * one copy out */
    if (c->engine == INCCL_ENGINE_P2P && c->group->transport == INCCL_TRANSPORT_RCCL) {
        if (((uintptr_t)dst_dev & 3u) == 0) return inccl_p2p_piece16(c, kind, srcs_dev, R, dst_dev, n, k, amax, scale_R, st);
        int rc = inccl_ws_claim(c, st);
        if (rc) return rc;
        rc = inccl_ensure_dev(&c->d_f32, &c->d_f32_bytes, n * sizeof(uint16_t));
        if (rc) return rc;
        rc = inccl_p2p_piece16(c, kind, srcs_dev, R, (uint16_t *)c->d_f32, n, k, amax, scale_R, st);
        if (rc) return rc;
        INCCL_HIP(hipMemcpyAsync(dst_dev, c->d_f32, n * sizeof(uint16_t), hipMemcpyDeviceToDevice, st));
        return 0;
    }
    /* every other engine: its int32 allreduce of the quantised partials (RCCL
     * all-reduce for "ar" / "a2a", the p2p exchange for the IPC engines) */
    int rc = inccl_ws_claim(c, st);
    if (rc) return rc;
    rc = inccl_ensure_dev(&c->d_q32, &c->d_q32_bytes, n * sizeof(int32_t));
    if (rc) return rc;
    int32_t *q = (int32_t *)c->d_q32;
    rc = kerr(inccl_k_stream(kind, INCCL_KIND_Q32, srcs, R, q, n, k, amax, scale_R, st));
    if (rc) return rc;
    rc = inccl_tp_allreduce_q32(c, q, q, n, st);
    if (rc) return rc;
    const void *s1[1] = {q};
    return kerr(inccl_k_stream_s(INCCL_KIND_Q32, kind, s1, 1, dst_dev, n, k, amax, scale_R,
                                 c->out_shift, st));
}

static int allreduce_16(struct inccl_communicator *c, int kind, const uint16_t *const *srcs_dev, int R,
                        uint16_t *dst_dev, size_t n, int scale_exp, void *stream)
{
    INCCL_ORDERED(c, stream, allreduce_16_body(c, kind, srcs_dev, R, dst_dev, n, scale_exp, stream));
}

int inccl_allreduce_bf16(struct inccl_communicator *c, const uint16_t *const *srcs_dev, int R, uint16_t *dst_dev,
                         size_t n, int scale_exp, void *stream)
{
    return allreduce_16(c, INCCL_KIND_BF16, srcs_dev, R, dst_dev, n, scale_exp, stream);
}

int inccl_allreduce_f16(struct inccl_communicator *c, const uint16_t *const *srcs_dev, int R, uint16_t *dst_dev,
                        size_t n, int scale_exp, void *stream)
{
    return allreduce_16(c, INCCL_KIND_F16, srcs_dev, R, dst_dev, n, scale_exp, stream);
}

/* Reduce-scatter (include/inccl_amd.h): the allreduce's arithmetic, rank `me`
 * keeping shard me of the result.  kind F32, BF16 or F16. */
static int reduce_scatter_body(struct inccl_communicator *c, int kind, const void *const *srcs, int R, void *dst,
                               size_t n, int scale_exp, void *stream)
{
    static const char *const names[] = {"f32", "", "", "bf16", "f16"};
    if (!c || !srcs || R < 1 || R > INCCL_MAX_LOCAL_INPUTS || (!dst && n))
        return inccl_set_error(INCCL_ERR_ARG, "bad reduce_scatter_%s args", names[kind]);
    for (int r = 0; r < R; ++r)
        if (!srcs[r] && n) return inccl_set_error(INCCL_ERR_ARG, "srcs[%d] is NULL", r);
    const int W = c->group->world_size, me = c->group->rank;
    if (n % (size_t)W)
        return inccl_set_error(INCCL_ERR_ARG, "reduce_scatter_%s: %zu elements do not split into %d shards",
                               names[kind], n, W);
    if (n == 0) return 0;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    const size_t shard = n / (size_t)W, es = kind == INCCL_KIND_F32 ? 4 : 2;
    for (int r = 0; r < R; ++r) {   /* the one-kernel routes read sources while writing dst */
        const uintptr_t s0 = (uintptr_t)srcs[r], d0 = (uintptr_t)dst;
        if (d0 < s0 + n * es && s0 < d0 + shard * es)
            return inccl_set_error(INCCL_ERR_ARG, "reduce_scatter_%s: dst overlaps srcs[%d]", names[kind], r);
    }
    const uint32_t *amax = NULL;
    int k = 0;
    int rc = resolve_scale(c, kind, srcs, R, n, scale_exp, st, &amax, &k);
    if (rc) return rc;
    const int scale_R = R * W;
    if (W == 1 && !c->force_sharded)   /* one fused HBM pass */
        return kerr(inccl_k_stream_s(kind, kind, srcs, R, dst, n, k, amax, scale_R, c->out_shift, st));
    if (c->engine == INCCL_ENGINE_RCCL || c->group->transport == INCCL_TRANSPORT_LOCAL) {
        /* quant + local sum -> int32 reduce-scatter -> dequantise the shard */
        rc = inccl_ws_claim(c, st);
        if (rc) return rc;
        rc = inccl_ensure_dev(&c->d_q32, &c->d_q32_bytes, (n + shard) * sizeof(int32_t));
        if (rc) return rc;
        int32_t *qsend = (int32_t *)c->d_q32, *qrecv = qsend + n;
        int si = stage_open(c, st);
        rc = kerr(inccl_k_stream(kind, INCCL_KIND_Q32, srcs, R, qsend, n, k, amax, scale_R, st));
        if (rc) return rc;
        stage_close(c, si, st, INCCL_STAGE_QUANT);
        si = stage_open(c, st);
        rc = inccl_tp_reduce_scatter_q32(c, qsend, qrecv, shard, st);
        if (rc) return rc;
        stage_close(c, si, st, INCCL_STAGE_RS);
        si = stage_open(c, st);
        const void *s1[1] = {qrecv};
        rc = kerr(inccl_k_stream_s(INCCL_KIND_Q32, kind, s1, 1, dst, shard, k, amax, scale_R, c->out_shift, st));
        stage_close(c, si, st, INCCL_STAGE_DEQUANT);
        return rc;
    }
    const int ipc = c->engine == INCCL_ENGINE_P2P || c->engine == INCCL_ENGINE_LL || c->engine == INCCL_ENGINE_MESH;
    /* Every route below is chosen from what all ranks share (engine, n, W and
     * the knobs agreed in agree_knobs), never from this rank's dst alignment:
     * a dst the vector kernels cannot store to (fp32 not 16-B, 16-bit not 8-B
     * aligned) gets the same route into an aligned workspace and one copy out. */
    const int rcclt = c->group->transport == INCCL_TRANSPORT_RCCL;
    const int mesh_route = c->mesh_rs && c->engine == INCCL_ENGINE_MESH && rcclt && !(shard % 64);
    const int p2p_route = ipc && rcclt && !(shard & 3);
    if (mesh_route || p2p_route) {
        void *out = dst;
        if (((uintptr_t)dst & (kind == INCCL_KIND_F32 ? 15u : 7u)) != 0) {
            rc = inccl_ws_claim(c, st);
            if (rc) return rc;
            rc = inccl_ensure_dev(&c->d_f32, &c->d_f32_bytes, shard * es);
            if (rc) return rc;
            out = c->d_f32;
        }
        /* the mesh engines' own route (INCCL_MESH_RS, default on): their one
         * persistent kernel, the allreduce's instructions with the other ranks'
         * gathers reduced to their waits (mesh.c; DESIGN.md, "Mesh
         * reduce-scatter route").  The ll engine's one kernel for a small fp32
         * bucket: every rank's quads published with a flag, this rank's shard
         * summed and dequantised.  Otherwise the p2p pull-reduce. */
        const int si = stage_open(c, st);
        if (mesh_route)
            rc = inccl_mesh_reduce_scatter(c, kind, srcs, R, out, n, k, amax, scale_R, st);
        else if (kind == INCCL_KIND_F32 && c->engine == INCCL_ENGINE_LL && n <= c->ll_max_bytes / sizeof(float))
            rc = inccl_ll_piece(c, (const float *const *)srcs, R, (float *)out, n, k, amax, scale_R,
                                (size_t)me * shard, shard, st);
        else
            rc = inccl_p2p_reduce_scatter(c, kind, srcs, R, out, n, k, amax, scale_R, st);
        if (rc) return rc;
        stage_close(c, si, st, INCCL_STAGE_IPC);
        if (out == dst) return 0;
        INCCL_HIP(hipMemcpyAsync(dst, out, shard * es, hipMemcpyDeviceToDevice, st));
        return 0;
    }
    /* every other engine, or a shard the pull-reduce cannot take: the engine's
     * int32 allreduce, then the shard dequantised */
    rc = inccl_ws_claim(c, st);
    if (rc) return rc;
    rc = inccl_ensure_dev(&c->d_q32, &c->d_q32_bytes, n * sizeof(int32_t));
    if (rc) return rc;
    int32_t *q = (int32_t *)c->d_q32;
    rc = kerr(inccl_k_stream(kind, INCCL_KIND_Q32, srcs, R, q, n, k, amax, scale_R, st));
    if (rc) return rc;
    rc = inccl_tp_allreduce_q32(c, q, q, n, st);
    if (rc) return rc;
    const void *s1[1] = {q + (size_t)me * shard};
    return kerr(inccl_k_stream_s(INCCL_KIND_Q32, kind, s1, 1, dst, shard, k, amax, scale_R, c->out_shift, st));
}

static int reduce_scatter_any(struct inccl_communicator *c, int kind, const void *const *srcs, int R, void *dst,
                              size_t n, int scale_exp, void *stream)
{
    INCCL_ORDERED(c, stream, reduce_scatter_body(c, kind, srcs, R, dst, n, scale_exp, stream));
}

int inccl_reduce_scatter_f32(struct inccl_communicator *c, const float *const *srcs_dev, int R, float *dst_dev,
                             size_t n, int scale_exp, void *stream)
{
    return reduce_scatter_any(c, INCCL_KIND_F32, (const void *const *)srcs_dev, R, dst_dev, n, scale_exp, stream);
}

int inccl_reduce_scatter_bf16(struct inccl_communicator *c, const uint16_t *const *srcs_dev, int R, uint16_t *dst_dev,
                              size_t n, int scale_exp, void *stream)
{
    return reduce_scatter_any(c, INCCL_KIND_BF16, (const void *const *)srcs_dev, R, dst_dev, n, scale_exp, stream);
}

int inccl_reduce_scatter_f16(struct inccl_communicator *c, const uint16_t *const *srcs_dev, int R, uint16_t *dst_dev,
                             size_t n, int scale_exp, void *stream)
{
    return reduce_scatter_any(c, INCCL_KIND_F16, (const void *const *)srcs_dev, R, dst_dev, n, scale_exp, stream);
}

/* ------------------------------------------------------------------ */
/* host-memory collectives                                              */
/* ------------------------------------------------------------------ */
/* Replaces api.c:403-452 / :330-401.  The reference encodes 1024-element
 * messages into the registered buffer (api.c:300-302), lets the switch add
 * them and decodes completions into dst (api.c:428-430).  Here the messages
 * become large chunks staged through the pinned send/receive buffers, the
 * sum runs on the GPU (RCCL or the local hub's sum kernel), and the same
 * "whole messages only" rule applies. */
/* The host paths' H2D and D2H streams.  They are high-priority streams: those
 * come from their own hardware-queue pool.  Created as normal streams after the
 * process had already launched work (e.g. torch tensors made first), the H2D
 * and D2H copies of config 3 ran one after the other (28 GB/s instead of
 * 44-46 GB/s both ways at once; tools/host_pipe_probe.py).
 * When: a one-rank communicator makes them at creation (made after the
 * process's big allocations they ran the pipeline at 44 instead of 45.7 GB/s);
 * a multi-rank one on its first host-path call, because high-priority queues
 * held by the processes sharing a GPU stalled their mesh engines' persistent
 * kernels for seconds at a time (DESIGN.md "Mesh reduce-scatter route",
 * liveness).  $INCCL_COPY_STREAMS=default keeps normal priority. */
static int copy_streams_ensure(struct inccl_communicator *c)
{
    if (c->copy_streams[0] && c->copy_streams[1]) return 0;
    const char *cse = getenv("INCCL_COPY_STREAMS");
    int prio_lo = 0, prio_hi = 0;
    INCCL_HIP(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    for (int i = 0; i < 2; ++i) {
        if (c->copy_streams[i]) continue;
        if (cse && strcmp(cse, "default") == 0)
            INCCL_HIP(hipStreamCreateWithFlags(&c->copy_streams[i], hipStreamNonBlocking));
        else
            INCCL_HIP(hipStreamCreateWithPriority(&c->copy_streams[i], hipStreamNonBlocking, prio_hi));
    }
    return 0;
}

/* Grow the pinned staging (the reference's 2*size registered buffers) so each
 * ping-pong half holds `half_bytes`. */
static int ensure_staging(struct inccl_communicator *c, size_t half_bytes)
{
    if ((size_t)c->payload_buf_size >= 2 * half_bytes && c->send_payload) return 0;
    if (c->copy_streams[0]) INCCL_HIP(hipStreamSynchronize(c->copy_streams[0]));
    if (c->copy_streams[1]) INCCL_HIP(hipStreamSynchronize(c->copy_streams[1]));
    if (c->send_payload) hipHostFree(c->send_payload);
    if (c->receive_payload) hipHostFree(c->receive_payload);
    c->send_payload = c->receive_payload = NULL;
    c->payload_buf_size = 0;
    INCCL_HIP(hipHostMalloc((void **)&c->send_payload, 2 * half_bytes, hipHostMallocDefault));
    INCCL_HIP(hipHostMalloc((void **)&c->receive_payload, 2 * half_bytes, hipHostMallocDefault));
    c->payload_buf_size = (uint32_t)(2 * half_bytes);
    return 0;
}

int inccl_host_register(struct inccl_communicator *c, void *ptr, size_t bytes)
{
    if (!c || !ptr || !bytes) return inccl_set_error(INCCL_ERR_ARG, "bad host_register args");
    if (c->nreg >= INCCL_MAX_HOST_REGIONS)
        return inccl_set_error(INCCL_ERR_ARG, "host_register: at most %d ranges", INCCL_MAX_HOST_REGIONS);
    for (int i = 0; i < c->nreg; ++i)
        if ((char *)ptr < c->reg[i].p + c->reg[i].len && c->reg[i].p < (char *)ptr + bytes)
            return inccl_set_error(INCCL_ERR_ARG, "host_register: range overlaps a registered one");
    INCCL_HIP(hipSetDevice(c->group->device));
    INCCL_HIP(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
    c->reg[c->nreg].p = (char *)ptr;
    c->reg[c->nreg].len = bytes;
    c->nreg++;
    return 0;
}

int inccl_host_deregister(struct inccl_communicator *c, void *ptr)
{
    if (!c || !ptr) return inccl_set_error(INCCL_ERR_ARG, "bad host_deregister args");
    for (int i = 0; i < c->nreg; ++i)
        if (c->reg[i].p == (char *)ptr) {
            if (c->copy_streams[0]) INCCL_HIP(hipStreamSynchronize(c->copy_streams[0]));
            if (c->copy_streams[1]) INCCL_HIP(hipStreamSynchronize(c->copy_streams[1]));
            INCCL_HIP(hipHostUnregister(ptr));
            c->reg[i] = c->reg[--c->nreg];
            return 0;
        }
    return inccl_set_error(INCCL_ERR_ARG, "host_deregister: %p is not a registered range", ptr);
}

/* page-locked host memory (hipHostMalloc'ed or hipHostRegister'ed by anyone) */
static int host_pinned(const void *p)
{
    hipPointerAttribute_t a;
    memset(&a, 0, sizeof(a));
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();   /* pageable memory: not an error for the caller */
        return 0;
    }
    return a.type == hipMemoryTypeHost;
}

static int host_registered(const struct inccl_communicator *c, const void *p, size_t bytes)
{
    for (int i = 0; i < c->nreg; ++i)
        if ((const char *)p >= c->reg[i].p && (const char *)p + bytes <= c->reg[i].p + c->reg[i].len) return 1;
    return 0;
}

/* Direct DMA between the caller's memory and two ping-ponging device chunks:
 * chunk i's H2D overlaps chunk i-1's D2H (PCIe is full duplex).  Used when src
 * and dst are registered, and -- unless $INCCL_HOST_STAGING=pool -- for
 * unregistered (pageable) memory too: HIP's own pageable copies run at the
 * pinned rate on MI355X boxes (tools/api_write_probe.py HOSTREF=1: 56 GB/s each
 * way), far above the staged pipeline below.  A pageable copy returns only when
 * done, so with pageable memory a helper thread issues the D2Hs (hostdma.c) and
 * the two directions stay in flight together.  $INCCL_HOST_CHUNK_MIB sets the
 * chunk (default 16 MiB). */
/* inside the host pipelines' chunk loops: a failed HIP call ends the loop (not
 * the function), so that the D2H helper's posted jobs are drained before return */
#define LOOP_HIP(call)                                 \
    {                                                  \
        const hipError_t e_ = (call);                  \
        if (e_ != hipSuccess) {                        \
            rc = inccl_hip_check(e_, #call);           \
            break;                                     \
        }                                              \
    }

/* INCCL_HOST_CHUNK_MIB, agreed over the group (agree_knobs): chunks are collective */
static size_t host_chunk_elems(const struct inccl_communicator *c)
{
    return ((size_t)c->host_chunk_mib << 20) / sizeof(int32_t);
}

static int allreduce_host_q32_direct(struct inccl_communicator *c, const int32_t *src, size_t n, int32_t *dst,
                                     int pageable)
{
    const size_t CH = host_chunk_elems(c);
    int rc = inccl_ensure_dev(&c->d_stage, &c->d_stage_bytes, 2 * CH * sizeof(int32_t));
    if (rc) return rc;
    if (pageable && !c->d2h) c->d2h = inccl_d2h_worker_create(c->group->device);
    struct inccl_d2h_worker *w = pageable ? c->d2h : NULL;   /* NULL: D2Hs issued here */
    int32_t *d[2] = {(int32_t *)c->d_stage, (int32_t *)c->d_stage + CH};
    rc = copy_streams_ensure(c);
    if (rc) return rc;
    hipStream_t h2d = c->copy_streams[0], d2h = c->copy_streams[1], ks = c->stream;
    hipEvent_t e_h2d[2] = {c->ev[0], c->ev[1]}, e_ar[2] = {c->ev[2], c->ev[3]}, e_d2h[2] = {c->ev[4], c->ev[5]};
    INCCL_HIP(hipStreamSynchronize(ks));
    const unsigned long long base = w ? inccl_d2h_posted(w) : 0;
    const size_t nch = (n + CH - 1) / CH;
    for (size_t i = 0; i < nch && rc == 0; ++i) {
        const int s = (int)(i & 1);
        const size_t off = i * CH, cnt = (n - off) < CH ? (n - off) : CH;
        if (i >= 2) {   /* d[s] drained by chunk i-2 */
            if (w) {
                const hipError_t e = inccl_d2h_wait_issued(w, base + i - 1);
                if (e != hipSuccess) {
                    rc = inccl_hip_check(e, "D2H of a host chunk");
                    break;
                }
            }
            LOOP_HIP(hipStreamWaitEvent(h2d, e_d2h[s], 0));
        }
        LOOP_HIP(hipMemcpyAsync(d[s], src + off, cnt * sizeof(int32_t), hipMemcpyHostToDevice, h2d));
        LOOP_HIP(hipEventRecord(e_h2d[s], h2d));
        LOOP_HIP(hipStreamWaitEvent(ks, e_h2d[s], 0));
        rc = inccl_tp_allreduce_q32(c, d[s], d[s], cnt, ks);            /* the switch's sum, nts.c:361-363 */
        if (rc) break;
        LOOP_HIP(hipEventRecord(e_ar[s], ks));
        if (w) {
            inccl_d2h_post(w, dst + off, d[s], cnt * sizeof(int32_t), e_ar[s], e_d2h[s], d2h);
        } else {
            LOOP_HIP(hipStreamWaitEvent(d2h, e_ar[s], 0));
            LOOP_HIP(hipMemcpyAsync(dst + off, d[s], cnt * sizeof(int32_t), hipMemcpyDeviceToHost, d2h));
            LOOP_HIP(hipEventRecord(e_d2h[s], d2h));
        }
    }
    if (w) {   /* every posted job issued before the stream is drained, also after a failure */
        const hipError_t e = inccl_d2h_wait_issued(w, inccl_d2h_posted(w));
        if (e != hipSuccess && !rc) rc = inccl_hip_check(e, "D2H of a host chunk");
    }
    INCCL_HIP(hipStreamSynchronize(d2h));
    return rc;
}

/* Replaces api.c:403-452 / :330-401.  The reference encodes 1024-element
 * messages into the registered buffer (api.c:300-302), lets the switch add
 * them and decodes completions into dst (api.c:428-430), two messages in
 * flight (api.c:408).  Here messages become chunks of up to 16 MiB that stream
 * through a 5-stage pipeline, chunk i+1's copy-in overlapping chunk i's DMA,
 * reduction and copy-out:
 *   host copy-in (pool) -> H2D (copy stream 0) -> device allreduce (RCCL, or the
 *   local hub's sum kernel) -> D2H (copy stream 1) -> host copy-out (pool)
 * The pinned staging halves ping-pong as the reference's two-message window
 * does.  The "whole messages only" rule (api.c:406) is kept. */
static int allreduce_host_q32(struct inccl_communicator *c, const int32_t *src, uint32_t len, int32_t *dst)
{
    const size_t message_num = len / PAYLOAD_COUNT;          /* api.c:406 */
    const size_t n = message_num * PAYLOAD_COUNT;
    if (n == 0) return 0;
    if (!src || !dst) return inccl_set_error(INCCL_ERR_ARG, "NULL src/dst");
    INCCL_HIP(hipSetDevice(c->group->device));
    if (host_registered(c, src, n * sizeof(int32_t)) && host_registered(c, dst, n * sizeof(int32_t)))
        return allreduce_host_q32_direct(c, src, n, dst, 0);
    const char *staging = getenv("INCCL_HOST_STAGING");   /* "pool": the staged pipeline below */
    if (!staging || strcmp(staging, "pool") != 0) return allreduce_host_q32_direct(c, src, n, dst, 1);
    /* chunk: what the reference buffers hold, at least 1 MiB, at most 16 MiB */
    size_t chunk_bytes = c->payload_buf_size / 2;
    if (chunk_bytes < ((size_t)1 << 20)) chunk_bytes = (size_t)1 << 20;
    if (chunk_bytes > ((size_t)16 << 20)) chunk_bytes = (size_t)16 << 20;
    if (chunk_bytes > n * sizeof(int32_t)) chunk_bytes = n * sizeof(int32_t);
    chunk_bytes = chunk_bytes / MESSAGE_SIZE * MESSAGE_SIZE;
    int rc = ensure_staging(c, chunk_bytes);
    if (rc) return rc;
    const size_t CH = chunk_bytes / sizeof(int32_t);
    rc = inccl_ensure_dev(&c->d_stage, &c->d_stage_bytes, 2 * chunk_bytes);
    if (rc) return rc;
    if (!c->pool) {
        const char *e = getenv("INCCL_COPY_THREADS");
        c->pool = inccl_copy_pool_create(e && *e ? atoi(e) : 4);   /* NULL -> plain memcpy */
    }
    int32_t *d[2] = {(int32_t *)c->d_stage, (int32_t *)c->d_stage + CH};
    char *in[2] = {c->send_payload, c->send_payload + chunk_bytes};
    char *out[2] = {c->receive_payload, c->receive_payload + chunk_bytes};
    rc = copy_streams_ensure(c);
    if (rc) return rc;
    hipStream_t h2d = c->copy_streams[0], d2h = c->copy_streams[1], ks = c->stream;
    hipEvent_t e_h2d[2] = {c->ev[0], c->ev[1]}, e_ar[2] = {c->ev[2], c->ev[3]}, e_d2h[2] = {c->ev[4], c->ev[5]};
    INCCL_HIP(hipStreamSynchronize(ks));
    const size_t nch = (n + CH - 1) / CH;
    for (size_t i = 0; i < nch; ++i) {
        const int s = (int)(i & 1);
        const size_t off = i * CH, cnt = (n - off) < CH ? (n - off) : CH;
        if (i >= 2) INCCL_HIP(hipEventSynchronize(e_h2d[s]));           /* in[s] read by chunk i-2's DMA */
        inccl_copy(c->pool, in[s], src + off, cnt * sizeof(int32_t));   /* api.c:300-302 (no byte swap) */
        if (i >= 2) INCCL_HIP(hipStreamWaitEvent(h2d, e_d2h[s], 0));    /* d[s] drained by chunk i-2 */
        INCCL_HIP(hipMemcpyAsync(d[s], in[s], cnt * sizeof(int32_t), hipMemcpyHostToDevice, h2d));
        INCCL_HIP(hipEventRecord(e_h2d[s], h2d));
        INCCL_HIP(hipStreamWaitEvent(ks, e_h2d[s], 0));
        rc = inccl_tp_allreduce_q32(c, d[s], d[s], cnt, ks);            /* the switch's sum, nts.c:361-363 */
        if (rc) return rc;
        INCCL_HIP(hipEventRecord(e_ar[s], ks));
        INCCL_HIP(hipStreamWaitEvent(d2h, e_ar[s], 0));
        INCCL_HIP(hipMemcpyAsync(out[s], d[s], cnt * sizeof(int32_t), hipMemcpyDeviceToHost, d2h));
        INCCL_HIP(hipEventRecord(e_d2h[s], d2h));
        if (i >= 1) {   /* decode the previous completion while this chunk is in flight (api.c:428-430) */
            const int ps = (int)((i - 1) & 1);
            const size_t poff = (i - 1) * CH, pcnt = (n - poff) < CH ? (n - poff) : CH;
            INCCL_HIP(hipEventSynchronize(e_d2h[ps]));
            inccl_copy(c->pool, dst + poff, out[ps], pcnt * sizeof(int32_t));
        }
    }
    const int ls = (int)((nch - 1) & 1);
    const size_t loff = (nch - 1) * CH, lcnt = n - loff;
    INCCL_HIP(hipEventSynchronize(e_d2h[ls]));
    inccl_copy(c->pool, dst + loff, out[ls], lcnt * sizeof(int32_t));
    return 0;
}

void inccl_allreduce_write(struct inccl_communicator *comm, int32_t *src_data, uint32_t len, int32_t *dst_data)
{
    if (!comm) {
        fprintf(stderr, "inccl_allreduce_write: NULL communicator\n");
        return;
    }
    if (allreduce_host_q32(comm, src_data, len, dst_data) != 0)
        fprintf(stderr, "inccl_allreduce_write: %s\n", inccl_last_error());
}

void inccl_allreduce_sendrecv(struct inccl_communicator *comm, int32_t *src_data, uint32_t len, int32_t *dst_data)
{
    if (!comm) {
        fprintf(stderr, "inccl_allreduce_sendrecv: NULL communicator\n");
        return;
    }
    if (allreduce_host_q32(comm, src_data, len, dst_data) != 0)
        fprintf(stderr, "inccl_allreduce_sendrecv: %s\n", inccl_last_error());
}

/* BASELINE config 3: fp32 gradient in host memory, buckets pipelined over
 * three streams -- H2D (copy_streams[0]), reduce (stream), D2H (copy_streams[1]). */
int inccl_allreduce_f32_host(struct inccl_communicator *c, const float *src_host, float *dst_host, size_t n,
                             int scale_exp, size_t bucket_bytes)
{
    if (!c || (!src_host && n) || (!dst_host && n)) return inccl_set_error(INCCL_ERR_ARG, "bad allreduce_f32_host args");
    if (n == 0) return 0;
    INCCL_HIP(hipSetDevice(c->group->device));
    size_t B = bucket_bytes / sizeof(float);
    B = B / 64 * 64;
    if (B == 0 || B > n) B = n;
    int rc = inccl_ensure_dev(&c->d_stage, &c->d_stage_bytes, 4 * B * sizeof(float));
    if (rc) return rc;
    float *in[2] = {(float *)c->d_stage, (float *)c->d_stage + B};
    float *out[2] = {(float *)c->d_stage + 2 * B, (float *)c->d_stage + 3 * B};
    rc = copy_streams_ensure(c);
    if (rc) return rc;
    hipStream_t h2d = c->copy_streams[0], d2h = c->copy_streams[1], ks = c->stream;
    hipEvent_t ev_h2d[2] = {c->ev[0], c->ev[1]}, ev_k[2] = {c->ev[2], c->ev[3]}, ev_d2h[2] = {c->ev[4], c->ev[5]};
    /* pageable dst: its D2Hs come from the helper thread (hostdma.c), or each one
     * would hold this thread until done and serialise the two directions */
    if (!host_pinned(dst_host) && !c->d2h) c->d2h = inccl_d2h_worker_create(c->group->device);
    struct inccl_d2h_worker *w = host_pinned(dst_host) ? NULL : c->d2h;
    const unsigned long long base = w ? inccl_d2h_posted(w) : 0;
    /* start clean: streams idle w.r.t. earlier work on the compute stream */
    INCCL_HIP(hipStreamSynchronize(ks));
    size_t i = 0;
    for (size_t off = 0; off < n && rc == 0; off += B, ++i) {
        const size_t cnt = (n - off) < B ? (n - off) : B;
        const int s = (int)(i & 1);
        if (i >= 2) LOOP_HIP(hipStreamWaitEvent(h2d, ev_k[s], 0));      /* in[s] consumed */
        LOOP_HIP(hipMemcpyAsync(in[s], src_host + off, cnt * sizeof(float), hipMemcpyHostToDevice, h2d));
        LOOP_HIP(hipEventRecord(ev_h2d[s], h2d));
        LOOP_HIP(hipStreamWaitEvent(ks, ev_h2d[s], 0));
        if (i >= 2) {   /* out[s] drained */
            if (w) {   /* ev_d2h[s] holds chunk i-2's record only once the helper issued it */
                const hipError_t e = inccl_d2h_wait_issued(w, base + i - 1);
                if (e != hipSuccess) {
                    rc = inccl_hip_check(e, "D2H of a host bucket");
                    break;
                }
            }
            LOOP_HIP(hipStreamWaitEvent(ks, ev_d2h[s], 0));
        }
        const float *srcs[1] = {in[s]};
        rc = inccl_allreduce_f32(c, srcs, 1, out[s], cnt, scale_exp, ks);
        if (rc) break;
        LOOP_HIP(hipEventRecord(ev_k[s], ks));
        if (w) {
            inccl_d2h_post(w, dst_host + off, out[s], cnt * sizeof(float), ev_k[s], ev_d2h[s], d2h);
        } else {
            LOOP_HIP(hipStreamWaitEvent(d2h, ev_k[s], 0));
            LOOP_HIP(hipMemcpyAsync(dst_host + off, out[s], cnt * sizeof(float), hipMemcpyDeviceToHost, d2h));
            LOOP_HIP(hipEventRecord(ev_d2h[s], d2h));
        }
    }
    if (w) {
        const hipError_t e = inccl_d2h_wait_issued(w, inccl_d2h_posted(w));
        if (e != hipSuccess && !rc) rc = inccl_hip_check(e, "D2H of a host bucket");
    }
    INCCL_HIP(hipStreamSynchronize(d2h));
    INCCL_HIP(hipStreamSynchronize(ks));
    INCCL_HIP(hipStreamSynchronize(h2d));
    return rc;
}
