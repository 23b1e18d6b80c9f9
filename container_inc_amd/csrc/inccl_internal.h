/* inccl_internal.h -- private definitions of libinccl_amd.so (C11 host code).
 *
 * The reference's structs (repository/include/api.h:42-91) hold libibverbs
 * handles; here the same roles are played by a transport (RCCL over xGMI, or
 * the in-process "local" hub where the GPU acts as the aggregation switch),
 * pinned host staging buffers (the registered MRs) and device workspaces. */
#ifndef INCCL_INTERNAL_H
#define INCCL_INTERNAL_H
#define INCCL_STAGE_SLOTS 64   /* stages recorded per call (16 chunks x 4 stages) */

#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime_api.h>

#include "inccl_amd.h"

#define INCCL_TRANSPORT_RCCL 0
#define INCCL_TRANSPORT_LOCAL 1
/* communicator-level exchange engine (group transport RCCL only) */
#define INCCL_ENGINE_RCCL 0
#define INCCL_ENGINE_P2P 1
#define INCCL_ENGINE_A2A 2
#define INCCL_ENGINE_LL 3
#define INCCL_ENGINE_MESH 4
#define INCCL_ENGINE_AR 5
#define INCCL_MAX_HOST_REGIONS 16
#define INCCL_MESH_REGIONS 4
/* Largest single allocation exported over HIP IPC (runtime.c).  Importing a
 * peer's allocation above 2 GiB hangs under PyTorch's bundled HSA runtime
 * (ROCr 7.0.2) and works under /opt/rocm's 7.2 (DESIGN.md "2 GiB per IPC
 * export"); the bound follows the HSA runtime the process mapped, and a group
 * agrees on the smallest over its ranks ($INCCL_IPC_MAX_BYTES overrides). */
#define INCCL_IPC_MAX_BYTES_DEFAULT (((size_t)2 << 30) - ((size_t)2 << 20))
#define INCCL_IPC_MAX_BYTES_UNBOUNDED ((size_t)1 << 40)
unsigned inccl_hsa_release_of(const char *build);   /* "..-rocm-rel-7.2-.." -> 702, 0 without the tag */
size_t inccl_ipc_local_max_bytes(void);

struct inccl_local_hub;
struct inccl_shm_bar;
struct inccl_copy_pool;
struct inccl_d2h_worker;

struct inccl_group {
    int rank;
    int world_size;
    int device;
    int transport;
    char master_ip[64];
    int port;
    /* rccl transport: control sockets.  rank 0 holds one fd per peer (the
     * reference's group_fd_list, api.h:58); other ranks hold master_fd. */
    int master_fd;
    int *peer_fds;
    struct inccl_shm_bar *shm_bar;   /* same-node fast barrier (NULL: TCP barrier) */
    size_t ipc_max_bytes;            /* largest IPC export, agreed over the ranks (runtime.c) */
    uint32_t max_seq;                /* host max-allreduces through shm so far (picks the word bank) */
    /* local transport */
    struct inccl_local_hub *hub;
    int comm_seq;   /* communicators created so far (names the hub slot) */
};

struct inccl_communicator {
    struct inccl_group *group;
    uint32_t payload_buf_size;   /* 2*size bytes, api.c:164 */
    uint32_t window_size;        /* WINDOW_SIZE, api.c:226 */
    char *send_payload;          /* pinned host staging (api.c:168) */
    char *receive_payload;       /* pinned host staging (api.c:169) */
    hipStream_t stream;          /* the communicator's compute/comm stream */
    hipStream_t side_stream;     /* second stream for pipelined variants */
    hipStream_t copy_streams[2]; /* H2D / D2H for the host-memory pipeline */
    void *nccl;                  /* ncclComm_t (rccl transport) */
    int comm_id;                 /* index within the group */
    /* device workspaces, grown on demand (never inside a capture) */
    void *d_q32;                 /* int32 partials, padded to world * shard */
    size_t d_q32_bytes;
    void *d_f32;                 /* fp32 gather target when dst cannot be used in place */
    size_t d_f32_bytes;
    void *d_stage;               /* host-path device staging (2 x in + 2 x out buckets) */
    size_t d_stage_bytes;
    uint32_t *d_words;           /* small scratch words: [0] absmax, [1] checksum */
    /* p2p engine: library-owned buffers shared with every peer through HIP IPC
     * handles; each GPU pulls its shard from all peers over xGMI */
    int engine;                  /* INCCL_ENGINE_* */
    int out_shift;               /* log2(world) when results are averaged (inccl_comm_set_average), else 0 */
    int nonfinite;               /* INCCL_NONFINITE_* (inccl_comm_set_nonfinite) */
    size_t p2p_cap;              /* elements per buffer */
    int32_t *p2p_part;           /* this rank's quantised partial sums (W * shard) */
    float *p2p_res;              /* this rank's dequantised shard lives at rank * shard */
    int32_t *p2p_peer_part[INCCL_MAX_LOCAL_INPUTS];
    float *p2p_peer_res[INCCL_MAX_LOCAL_INPUTS];
    /* ll engine (small buckets, one kernel per call): one IPC buffer per rank =
     * signal array + call counter + two parity data slots */
    char *ll_buf;
    char *ll_peer[INCCL_MAX_LOCAL_INPUTS];
    size_t ll_cap;               /* elements per data slot */
    uint32_t *ll_err_host;       /* host-mapped: set by a kernel whose peers timed out */
    uint32_t *ll_err_dev;
    uint64_t ll_timeout_ticks;
    hipStream_t ll_last_stream;  /* ordering across caller streams (ev[7]) */
    size_t ll_max_bytes;         /* buckets up to this size take the ll kernel */
    int mesh_rs;                 /* INCCL_MESH_RS (default 1): reduce-scatter through the mesh kernel */
    int force_sharded;           /* INCCL_FORCE_SHARDED: test hook, the sharded paths even at world 1 */
    size_t mesh_chunk_env;       /* INCCL_MESH_CHUNK elements (0: mesh.c's default) */
    int mesh_lag_env;            /* INCCL_MESH_LAG slots (0: the whole shard) */
    int host_chunk_mib;          /* INCCL_HOST_CHUNK_MIB: host pipeline chunk (default 16) */
    /* every knob above that picks a route or a schedule is agreed over the
     * group when the communicator is created (api.c agree_knobs): ranks whose
     * environments differ still take the same route on every call */
    size_t rccl_ar_bytes;        /* rccl engine: int32 partials up to this size take one
                                    ncclAllReduce instead of reduce-scatter + all-gather */
    /* mesh engine (large buckets, one persistent kernel per call): one IPC buffer
     * per rank = signal array + counters + inbox (W partial shards) + result shard */
    char *mesh_buf;                                        /* = mesh_reg[0]: signals + counters */
    char *mesh_reg[INCCL_MESH_REGIONS];                    /* sig, inbox, result shard, result inbox */
    char *mesh_peer[INCCL_MESH_REGIONS][INCCL_MAX_LOCAL_INPUTS];   /* rank j's regions ([r][me] = own) */
    size_t mesh_cap;             /* elements per inbox slot / result shard */
    int mesh_grid;               /* this rank's workgroups per call */
    uint32_t *mesh_err_host;     /* host-mapped: set by a kernel whose peers timed out */
    uint32_t *mesh_err_dev;
    uint64_t mesh_timeout_ticks;
    hipStream_t mesh_last_stream;  /* ordering across caller streams (ev[6]) */
    int mesh_push;               /* "meshw": result chunks pushed into every rank's result inbox */
    /* host memory registered by the caller (inccl_host_register, the ibv_reg_mr of
     * api.c:170-176): the host collectives DMA such ranges directly */
    struct { char *p; size_t len; } reg[INCCL_MAX_HOST_REGIONS];
    int nreg;
    struct inccl_copy_pool *pool;  /* host staging copies (copypool.c) */
    struct inccl_d2h_worker *d2h;  /* issues pageable D2H copies beside the H2Ds (hostdma.c) */
    hipEvent_t ev[10];           /* [8]: p2p ordering across caller streams; [9]: workspace ordering
                                  * across caller streams (ws_last_stream) */
    /* per-stage timing (inccl_comm_set_stage_timing): begin/end timing events
     * per recorded stage of the last call, ev[2*i] / ev[2*i+1] */
    int stage_on, stage_cnt, stage_kind[INCCL_STAGE_SLOTS];
    hipEvent_t stage_ev[2 * INCCL_STAGE_SLOTS];
    hipStream_t ws_last_stream;  /* the stream of the last call that used the shared workspaces */
    hipStream_t ws_stream;       /* this call's stream, once it claimed them (inccl_ws_claim) */
    int ws_claimed, ws_capturing;
    hipStream_t p2p_last_stream;
};

/* transport operations; all stream-ordered on `st` */
int inccl_tp_reduce_scatter_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t shard,
                                hipStream_t st);
int inccl_tp_all_gather_f32(struct inccl_communicator *c, const float *send, float *recv, size_t shard,
                            hipStream_t st);
int inccl_tp_all_gather_bf16(struct inccl_communicator *c, const uint16_t *send, uint16_t *recv, size_t shard,
                             hipStream_t st);
int inccl_tp_allreduce_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t n,
                           hipStream_t st);
int inccl_tp_allreduce_max_u32(struct inccl_communicator *c, uint32_t *buf, size_t n, hipStream_t st);
int inccl_tp_barrier(struct inccl_communicator *c);

/* rccl transport */
int inccl_rccl_comm_init(struct inccl_communicator *c);
void inccl_rccl_comm_destroy(struct inccl_communicator *c);
int inccl_rccl_reduce_scatter_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t shard,
                                  hipStream_t st);
int inccl_rccl_all_gather_f32(struct inccl_communicator *c, const float *send, float *recv, size_t shard,
                              hipStream_t st);
int inccl_rccl_all_gather_bf16(struct inccl_communicator *c, const uint16_t *send, uint16_t *recv, size_t shard,
                               hipStream_t st);
int inccl_rccl_allreduce_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t n,
                             hipStream_t st);
int inccl_rccl_allreduce_max_u32(struct inccl_communicator *c, uint32_t *buf, size_t n, hipStream_t st);
/* grouped send/recv: shard j of `send` to rank j, rank j's shard `me` into recv + j*shard */
int inccl_rccl_alltoall_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t shard,
                            hipStream_t st);

/* p2p engine */
int inccl_p2p_piece(struct inccl_communicator *c, const float *const *srcs, int R, float *dst, size_t n, int k,
                    const uint32_t *amax, int scale_R, hipStream_t st);
/* 2-byte buckets, kind INCCL_KIND_BF16 or INCCL_KIND_F16 */
int inccl_p2p_piece16(struct inccl_communicator *c, int kind, const uint16_t *const *srcs, int R, uint16_t *dst,
                      size_t n, int k, const uint32_t *amax, int scale_R, hipStream_t st);
void inccl_p2p_release(struct inccl_communicator *c);
/* reduce-scatter of kind F32 / BF16 / F16 buckets over the p2p buffers: n = W *
 * shard, shard % 4 == 0; dst = the dequantised shard `me` (inccl_reduce_scatter_*) */
int inccl_p2p_reduce_scatter(struct inccl_communicator *c, int kind, const void *const *srcs, int R, void *dst,
                             size_t n, int k, const uint32_t *amax, int scale_R, hipStream_t st);
/* int32 allreduce (wrapping sum) over the p2p engine's IPC buffers: the
 * reference API's inccl_allreduce_write on a multi-process group without RCCL */
int inccl_p2p_allreduce_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t n,
                            hipStream_t st);

/* ll engine (ll.c): n <= c->ll_max_bytes / 4.  rs_n > 0: reduce-scatter, dst =
 * elements [rs_lo, rs_lo + rs_n) of the result (both multiples of 4) */
int inccl_ll_piece(struct inccl_communicator *c, const float *const *srcs, int R, float *dst, size_t n, int k,
                   const uint32_t *amax, int scale_R, size_t rs_lo, size_t rs_n, hipStream_t st);
void inccl_ll_release(struct inccl_communicator *c);
uint64_t inccl_wait_ticks(struct inccl_group *g);   /* bound of an in-kernel wait */

/* mesh engine (mesh.c) */
int inccl_mesh_piece(struct inccl_communicator *c, const float *const *srcs, int R, float *dst, size_t n, int k,
                     const uint32_t *amax, int scale_R, hipStream_t st);
int inccl_mesh_piece16(struct inccl_communicator *c, int kind, const uint16_t *const *srcs, int R, uint16_t *dst,
                       size_t n, int k, const uint32_t *amax, int scale_R, hipStream_t st);
int inccl_mesh_reduce_scatter(struct inccl_communicator *c, int kind, const void *const *srcs, int R, void *dst,
                              size_t n, int k, const uint32_t *amax, int scale_R, hipStream_t st);
void inccl_mesh_release(struct inccl_communicator *c);

/* local transport */
struct inccl_local_hub *inccl_hub_attach(const char *name, int world_size);
void inccl_hub_detach(struct inccl_local_hub *hub);
int inccl_local_reduce_scatter_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t shard,
                                   hipStream_t st);
int inccl_local_all_gather_f32(struct inccl_communicator *c, const float *send, float *recv, size_t shard,
                               hipStream_t st);
int inccl_local_allreduce_q32(struct inccl_communicator *c, const int32_t *send, int32_t *recv, size_t n,
                              hipStream_t st);
int inccl_local_allreduce_max_u32(struct inccl_communicator *c, uint32_t *buf, size_t n, hipStream_t st);
int inccl_local_barrier(struct inccl_communicator *c);

/* TCP bootstrap (bootstrap.c) */
int inccl_boot_master(struct inccl_group *g);
int inccl_boot_worker(struct inccl_group *g);
int inccl_boot_bcast(struct inccl_group *g, void *buf, size_t bytes);   /* from rank 0 */
int inccl_boot_barrier(struct inccl_group *g);
int inccl_boot_allgather(struct inccl_group *g, const void *mine, void *all, size_t bytes);
int inccl_boot_shm_init(struct inccl_group *g);   /* collective; falls back silently */
int inccl_group_barrier(struct inccl_group *g);   /* shm barrier if set up, else TCP */
int inccl_group_allreduce_max_u32(struct inccl_group *g, uint32_t *v);   /* through shm if set up, else TCP */
void inccl_boot_close(struct inccl_group *g);

/* errors */
int inccl_set_error(int code, const char *fmt, ...);
int inccl_hip_check(hipError_t e, const char *what);
#define INCCL_HIP(call)                                         \
    do {                                                        \
        hipError_t e_ = (call);                                 \
        if (e_ != hipSuccess) return inccl_hip_check(e_, #call); \
    } while (0)

/* shard size for world ranks: multiple of 64 elements (256 B) so every shard
 * starts 16-B aligned for the dwordx4 kernels */
static inline size_t inccl_shard_elems(size_t n, int world)
{
    size_t per = (n + (size_t)world - 1) / (size_t)world;
    return (per + 63) & ~(size_t)63;
}

int inccl_ensure_dev(void **p, size_t *cur, size_t need);
/* before a call first uses the communicator's shared workspaces (d_q32, d_f32,
 * d_words): orders it after the last call that used them on another stream */
int inccl_ws_claim(struct inccl_communicator *c, hipStream_t st);
/* IPC-shared device memory polled by running kernels (ll, mesh): $INCCL_IPC_MEM */
unsigned inccl_ipc_mem_flags(void);
hipError_t inccl_ipc_malloc(void **p, size_t bytes);
int inccl_mem_kind(const void *p);   /* hipPointerAttribute_t.allocationFlags */

/* copypool.c */
struct inccl_copy_pool *inccl_copy_pool_create(int n);
void inccl_copy_pool_destroy(struct inccl_copy_pool *p);
void inccl_copy(struct inccl_copy_pool *p, void *dst, const void *src, size_t bytes);

/* hostdma.c */
struct inccl_d2h_worker *inccl_d2h_worker_create(int device);
void inccl_d2h_worker_destroy(struct inccl_d2h_worker *w);
unsigned long long inccl_d2h_posted(struct inccl_d2h_worker *w);
void inccl_d2h_post(struct inccl_d2h_worker *w, void *dst, const void *src, size_t bytes, hipEvent_t after,
                    hipEvent_t done, hipStream_t st);
hipError_t inccl_d2h_wait_issued(struct inccl_d2h_worker *w, unsigned long long count);

#endif
