/*
 * inccl_amd.h -- additive MI355X API of libinccl_amd.so (fp32 gradient buckets,
 * device pointers, explicit streams).  None of this exists in the reference;
 * each entry point names the reference code whose arithmetic it carries.
 *
 * Conventions
 *   - Pointers named *_dev are device (HBM) pointers; `srcs` arguments are HOST
 *     arrays holding R device pointers.
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream).
 *     Calls are stream-ordered and do not synchronise unless stated.
 *   - Return 0 on success; a negative INCCL_ERR_* code, or a positive
 *     hipError_t / ncclResult_t value, on failure.  inccl_last_error() has text.
 *   - 16-byte-aligned buffers take the dwordx4 streaming path; anything else
 *     falls back to an element-granular kernel (still on the GPU).
 *
 * Numerics (the spec the CPU oracle restates, oracle/inccl_oracle.c)
 *   quantise    q = sat_int32(round_half_even(x * 2^k)); NaN -> 0; +-Inf saturate
 *   reduce      s = sum_r q_r  mod 2^32                  (non_termination_switch.c:361-363)
 *   dequantise  y = (float)s * 2^-k                       ((float) rounds to nearest even)
 *   k in [INCCL_SCALE_MIN, INCCL_SCALE_MAX]; INCCL_SCALE_AUTO picks the largest k
 *   with R_total * max|x| * 2^k <= 2^30 from a device-side absmax reduction.
 */
#ifndef INCCL_AMD_H
#define INCCL_AMD_H

#include <stddef.h>
#include <stdint.h>

#include "api.h"

#ifdef __cplusplus
extern "C" {
#endif

#define INCCL_MAX_LOCAL_INPUTS 8        /* R per kernel launch */
#define INCCL_SCALE_MIN (-64)
#define INCCL_SCALE_MAX 64
#define INCCL_SCALE_AUTO 0x7fffffff

#define INCCL_OK 0
#define INCCL_ERR_ARG (-1)
#define INCCL_ERR_HIP (-2)
#define INCCL_ERR_NCCL (-3)
#define INCCL_ERR_SYS (-4)
#define INCCL_ERR_STATE (-5)
#define INCCL_ERR_NOMEM (-6)

/* element kinds of the generic streaming kernel */
#define INCCL_KIND_F32 0     /* fp32 gradient                                  */
#define INCCL_KIND_Q32 1     /* int32, host byte order                         */
#define INCCL_KIND_Q32BE 2   /* int32, big-endian wire word (api.c:301, util.c:404) */
#define INCCL_KIND_BF16 3    /* bfloat16 gradient (2-byte elements): quantised as the fp32 it
                                widens to exactly; dequantised as bf16_rne((float)s * 2^-k).
                                Pairs: BF16->BF16, BF16->Q32, Q32->BF16 */
#define INCCL_KIND_F16 4     /* IEEE binary16 gradient: quantised as the fp32 it widens to exactly;
                                dequantised as f16_rne((float)s * 2^-k) (+-Inf past 65504).
                                Pairs: F16->F16, F16->Q32, Q32->F16 */

const char *inccl_last_error(void);
const char *inccl_version(void);

/* ---------- stateless device kernels (one GPU, stream-ordered) ---------- */

/* fp32 -> int32 fixed point (new front stage).  wire_be != 0 also applies the
 * reference's htonl encode (api.c:300-302) in the same pass. */
int inccl_quantise_f32(const float *x_dev, int32_t *q_dev, size_t n, int scale_exp, int wire_be, void *stream);
/* int32 -> fp32 (new back stage).  wire_be != 0 first applies ntohl (api.c:428-430). */
int inccl_dequantise_q32(const int32_t *q_dev, float *y_dev, size_t n, int scale_exp, int wire_be, void *stream);
/* Fused single-GPU bucket reduce: dst = dequant(sum_r quant(srcs[r])), R <= 8.
 * One HBM pass: (R + 1) * 4 * n bytes.  dst may alias srcs[0]. */
int inccl_reduce_f32(const float *const *srcs_dev, int R, float *dst_dev, size_t n, int scale_exp, void *stream);
/* As above with INCCL_SCALE_AUTO semantics; amax_word_dev is a 4-byte device
 * scratch word (zeroed and written by the call). */
int inccl_reduce_f32_auto(const float *const *srcs_dev, int R, float *dst_dev, size_t n, uint32_t *amax_word_dev,
                          void *stream);
/* Local quantise + sum to int32 (first stage of the multi-GPU path). */
int inccl_quant_sum_f32(const float *const *srcs_dev, int R, int32_t *dst_dev, size_t n, int scale_exp, int wire_be,
                        void *stream);
/* Switch aggregate (non_termination_switch.c:361-363, util.c:403-405):
 * dst = sum_r srcs[r] mod 2^32, optional big-endian decode of the inputs
 * (in_be) and encode of the output (out_be). */
int inccl_sum_q32(const int32_t *const *srcs_dev, int R, int32_t *dst_dev, size_t n, int in_be, int out_be,
                  void *stream);
/* Sum + dequantise: dst = dequant(sum_r srcs[r]) (reduce-scatter variant B epilogue). */
int inccl_sum_dequant_q32(const int32_t *const *srcs_dev, int R, float *dst_dev, size_t n, int scale_exp, int in_be,
                          void *stream);
/* Generic form of all of the above (kinds INCCL_KIND_*).  amax_bits_dev != NULL
 * derives k from that device word and scale_R contributors instead of scale_exp. */
int inccl_stream_op(int in_kind, int out_kind, const void *const *srcs_dev, int R, void *dst_dev, size_t n,
                    int scale_exp, const uint32_t *amax_bits_dev, int scale_R, void *stream);
/* A prepared stream op: inccl_stream_op's arguments (a fixed scale exponent)
 * checked and bound once, so that each run is one kernel launch with no
 * argument marshalling -- for small buckets, whose launch costs more than their
 * kernel (4 MiB fused, R = 2: ~2.2 us of device time), called through a
 * binding such as Python's ctypes, where building the arguments of every call
 * costs several us more.  The bound buffers and stream must outlive the op.
 * inccl_op_run launches on the bound stream, stream-ordered like the call it
 * prepares; NULL from create = invalid arguments (inccl_last_error). */
struct inccl_op;
struct inccl_op *inccl_op_create(int in_kind, int out_kind, const void *const *srcs_dev, int R, void *dst_dev,
                                 size_t n, int scale_exp, int scale_R, void *stream);
int inccl_op_run(struct inccl_op *op);
int inccl_op_destroy(struct inccl_op *op);
/* max |x| over R buckets into *amax_bits_dev (float bits; NaN ignored).  The word
 * is zeroed first when bit 0 of zero_first is set, else max-accumulated.  With
 * INCCL_ABSMAX_FLAG_NONFINITE also set in zero_first, a NaN or +-Inf element sets
 * bit 31 of the word instead (which no |x| has, so a max over words and ranks
 * keeps it); a kernel handed such a word as its auto scale dequantises every
 * element to NaN (inccl_comm_set_nonfinite). */
#define INCCL_ABSMAX_FLAG_NONFINITE 2
int inccl_absmax_f32(const float *const *srcs_dev, int R, size_t n, uint32_t *amax_bits_dev, int zero_first,
                     void *stream);
/* Position-weighted linear checksum sum_i (2(base+i)+1)*q[i] mod 2^32 into *out_dev. */
int inccl_checksum_q32(const int32_t *q_dev, size_t n, uint64_t index_base, uint32_t *out_dev, int zero_first,
                       void *stream);
/* Host helper: the scale rule of INCCL_SCALE_AUTO. */
int inccl_choose_scale(float absmax, int R_total);
/* Tuning knobs of the streaming kernel (grid cap in workgroups, 0 = default;
 * nontemporal loads on/off).  For benchmarks and sweeps only. */
void inccl_set_tuning(int grid_cap, int nt_loads);

/* ---------- groups and communicators ---------- */

/* Like inccl_group_create with an explicit rendezvous port (0 = MASTER_PORT or
 * $INCCL_MASTER_PORT) and HIP device (-1 = $INCCL_DEVICE, $LOCAL_RANK, or rank
 * modulo the device count). */
struct inccl_group *inccl_group_create_ex(int world_size, int rank, const char *master_ip, int port, int device);
/* In-process transport: `world_size` ranks are threads of this process sharing
 * one GPU.  Every rank thread calls this with the same `hub_name`; the GPU plays
 * the aggregation switch (its sum kernel reduces the ranks' buffers). */
struct inccl_group *inccl_group_create_local(int world_size, int rank, const char *hub_name, int device);
int inccl_group_rank(const struct inccl_group *group);
int inccl_group_size(const struct inccl_group *group);
int inccl_group_device(const struct inccl_group *group);
/* "rccl" or "local" */
const char *inccl_group_transport(const struct inccl_group *group);
/* Largest single buffer the IPC engines (p2p, mesh) may share with peers, in
 * bytes.  It follows the HSA runtime the process runs on: PyTorch's bundled
 * ROCr (ROCm 7.0.2) hangs importing a peer allocation above 2 GiB, so 2 GiB -
 * 2 MiB there; no bound under a ROCr that reports ROCm 7.2 or later
 * (/opt/rocm; inccl_hsa_runtime_release); $INCCL_IPC_MAX_BYTES overrides
 * (whole MiB, at least 1 MiB).  inccl_ipc_max_bytes: this process;
 * inccl_group_ipc_max_bytes: the smallest over the group's ranks, agreed at
 * creation -- a bucket whose IPC buffer would exceed it is refused on every
 * rank alike.  The first call of inccl_ipc_max_bytes, inccl_hsa_runtime_release
 * or inccl_hsa_runtime_build in a process INITIALISES HIP (hipInit) and briefly
 * HSA (hsa_init / hsa_shut_down) to ask the runtime: do not call them in a
 * process that must stay free of a GPU context (one that will fork or exec
 * GPU work). */
size_t inccl_ipc_max_bytes(void);
size_t inccl_group_ipc_max_bytes(const struct inccl_group *group);
/* The ROCm release of the HSA runtime this process mapped, as that runtime
 * reports it (HSA_AMD_SYSTEM_INFO_BUILD_VERSION "..-rocm-rel-7.2-.." -> 702),
 * and the build string itself; 0 / "" when it cannot be asked (no GPU). */
unsigned inccl_hsa_runtime_release(void);
const char *inccl_hsa_runtime_build(void);
/* RCCL: *compiled = the NCCL_VERSION_CODE of the headers this library was
 * built against (/opt/rocm), *loaded = ncclGetVersion() of the librccl the
 * process bound to (torch's in a Python process).  0 or an error code. */
int inccl_rccl_version(int *compiled, int *loaded);
/* The communicator's own HIP stream (void* hipStream_t). */
void *inccl_comm_stream(struct inccl_communicator *comm);
int inccl_comm_barrier(struct inccl_communicator *comm);
/* Exchange engine of a multi-process communicator for inccl_allreduce_f32:
 *   "rccl"  quant+sum -> ncclReduceScatter(int32) -> dequant -> ncclAllGather (default);
 *           buckets whose int32 partials fit $INCCL_RCCL_AR_BYTES (default 1 MiB) take
 *           quant+sum -> ncclAllReduce(int32) -> dequant, as "ar"
 *   "a2a"   quant+sum -> grouped ncclSend/Recv of int32 shards -> this library's fused
 *           sum + dequantise kernel over the W shards -> ncclAllGather
 *   "p2p"   library buffers shared via HIP IPC; each GPU pulls its shard from every
 *           peer over xGMI with the fused sum+dequantise kernel, then pulls every
 *           peer's result shard (two group barriers per call).  Also the automatic
 *           fallback when RCCL cannot come up on every rank.
 *   "ll"    one kernel per call for buckets up to $INCCL_LL_MAX_BYTES (default
 *           1 MiB): quant + local sum into an IPC buffer, arrival flags written into
 *           the peers' memory, every peer's bucket read over xGMI and summed +
 *           dequantised; no host synchronisation (larger buckets: as "p2p")
 *   "mesh"  one persistent kernel per call: each chunk's quantised partial is
 *           pushed into its owner's IPC inbox over xGMI, the owner sums +
 *           dequantises it once every rank's arrival flag is up, and every rank pulls
 *           the result chunks; phases of different chunks overlap, no host
 *           synchronisation
 *   The ll and mesh buffers are fine-grained uncached device memory by default
 *   ($INCCL_IPC_MEM = uncached | finegrained | coarse): their kernels poll flags
 *   that peers write over xGMI while they run.
 *   "meshw" as "mesh", but the owner also pushes each result chunk into every
 *           rank's IPC result inbox, so that every xGMI transfer is a write; each
 *           rank then copies the chunks locally into dst
 *   "ar"    quant+sum -> ncclAllReduce(int32, sum) in place -> dequant
 * Every rank must select the same engine.  $INCCL_ENGINE sets it at creation. */
int inccl_comm_set_engine(struct inccl_communicator *comm, const char *name);
/* "rccl", "ar", "a2a", "p2p", "ll", "mesh", "meshw" or "local" */
const char *inccl_comm_engine(const struct inccl_communicator *comm);
/* Allocation flags (hipDeviceMallocDefault 0 / Finegrained 1 / Uncached 3) of the
 * IPC buffer the named engine ("ll", "mesh" or "p2p") has allocated, or a
 * negative INCCL_ERR_* code if it has none yet. */
int inccl_comm_ipc_mem_kind(struct inccl_communicator *comm, const char *engine);
/* Collective (every rank calls it).  An ll or mesh wait that timed out leaves
 * its call's dst undefined and makes every later call of that engine fail with
 * "timed out".  This returns 1 if such a timeout had been recorded on this rank
 * (0 if not, negative on error) and drops the engines' IPC buffers after a
 * device synchronisation and a group barrier, so that the next call rebuilds
 * them from a clean state.  Check a call's outcome after synchronising its
 * stream: a timeout is reported by the NEXT call or by this function. */
int inccl_comm_clear_error(struct inccl_communicator *comm);
/* on != 0: every later inccl_allreduce_f32 / _bf16 (and _f32_host) of this rank
 * returns the MEAN over the ranks instead of the sum -- the dequantise stage
 * scales by 2^-(k + log2 W), which is exact, so the result is bit-identical to
 * dividing the sum by W, without the extra pass over the bucket.  Only for a
 * power-of-two world size (else INCCL_ERR_ARG).  Set it alike on every rank. */
int inccl_comm_set_average(struct inccl_communicator *comm, int on);
/* What a NaN or +-Inf input does to an INCCL_SCALE_AUTO allreduce of this
 * communicator.  INCCL_NONFINITE_SATURATE (the default, the quantiser's spec):
 * NaN quantises to 0 and +-Inf saturates, so the result stays finite.
 * INCCL_NONFINITE_NAN: if any element of any rank's buckets is NaN or +-Inf,
 * every element of the result is NaN on every rank -- what a mixed-precision
 * loss scaler needs to see to skip the step -- at no extra pass (the flag rides
 * in the auto scale's max word).  A fixed scale exponent is unaffected.  Set it
 * alike on every rank. */
#define INCCL_NONFINITE_SATURATE 0
#define INCCL_NONFINITE_NAN 1
int inccl_comm_set_nonfinite(struct inccl_communicator *comm, int mode);

/* Per-stage timing of this rank's calls (diagnostics; off by default).  on != 0:
 * every later non-captured allreduce / reduce-scatter records a pair of HIP
 * timing events around each of its stages, on the stream the stage runs on
 * (about 2 x 3 us of GPU time per stage: never in a timed loop).  After a call,
 * inccl_comm_stage_times synchronises those events and fills us[kind] with the
 * summed microseconds of each stage kind (us[] of INCCL_STAGE_KINDS entries,
 * chunks of a pipelined call added up) and *wall_us with the first stage's start
 * to the last one's end; sum(us) - wall is the time the stages overlapped (the
 * pipelined rccl path quantises chunk i+1 beside chunk i's collectives).
 * Returns the number of stages recorded (0: none, e.g. timing off or a captured
 * call), negative on error. */
#define INCCL_STAGE_QUANT 0    /* quantise + local sum (+ the tail memset) */
#define INCCL_STAGE_RS 1       /* int32 reduce-scatter (ncclReduceScatter, or the in-process one) */
#define INCCL_STAGE_DEQUANT 2  /* dequantise the own shard */
#define INCCL_STAGE_AG 3       /* all-gather of the result shards (ncclAllGather) */
#define INCCL_STAGE_COPY 4     /* copy out of a workspace (ragged or misaligned buckets) */
#define INCCL_STAGE_AR 5       /* int32 allreduce (ncclAllReduce: "ar" engine, small buckets) */
#define INCCL_STAGE_IPC 6      /* an IPC engine's whole exchange (p2p / ll / mesh kernels) */
#define INCCL_STAGE_KINDS 7
int inccl_comm_set_stage_timing(struct inccl_communicator *comm, int on);
int inccl_comm_stage_times(struct inccl_communicator *comm, double *us, int kinds, double *wall_us);

/* Device-resident fp32 allreduce of R local buckets per rank:
 *   dst = dequant( sum over ranks, sum over r<R  quant(srcs[r]) )
 * world == 1: one fused kernel.  world > 1: quant+local sum -> reduce-scatter
 * (int32, sum) -> dequantise own shard -> all-gather (fp32).  `scale_exp` may be
 * INCCL_SCALE_AUTO (adds an absmax pass and a 4-byte max-allreduce).
 * stream NULL = the communicator's stream.  dst may alias srcs[0].  A
 * communicator's calls (allreduce, reduce-scatter, any format) may come on any
 * stream: one on another stream than the previous call's waits for that call's
 * end on the device, since they share the communicator's workspaces. */
int inccl_allreduce_f32(struct inccl_communicator *comm, const float *const *srcs_dev, int R, float *dst_dev,
                        size_t n, int scale_exp, void *stream);
/* Same with the bucket split into `chunks` pieces pipelined over two streams
 * (compute of chunk c+1 overlaps the collectives of chunk c).  chunks <= 1 is
 * inccl_allreduce_f32. */
int inccl_allreduce_f32_pipelined(struct inccl_communicator *comm, const float *const *srcs_dev, int R,
                                  float *dst_dev, size_t n, int scale_exp, int chunks, void *stream);
/* A prepared inccl_allreduce_f32_pipelined (see inccl_op_create): a fixed scale
 * exponent, the same arguments on every run -- for the small-message regime,
 * where marshalling a call costs as much as the collective.  Collective like
 * the call it prepares: every rank runs its op for every call.  Destroy with
 * inccl_op_destroy before the communicator. */
struct inccl_op *inccl_op_create_allreduce_f32(struct inccl_communicator *comm, const float *const *srcs_dev, int R,
                                               float *dst_dev, size_t n, int scale_exp, int chunks, void *stream);
/* The same for 2-byte buckets: a prepared inccl_allreduce_bf16 (kind
 * INCCL_KIND_BF16) or inccl_allreduce_f16 (INCCL_KIND_F16). */
struct inccl_op *inccl_op_create_allreduce16(struct inccl_communicator *comm, int kind,
                                             const uint16_t *const *srcs_dev, int R, uint16_t *dst_dev, size_t n,
                                             int scale_exp, void *stream);
/* Device int32 allreduce (sum, wrap): the arithmetic of inccl_allreduce_write
 * without the host copies. */
int inccl_allreduce_q32(struct inccl_communicator *comm, const int32_t *src_dev, int32_t *dst_dev, size_t n,
                        void *stream);
/* Register caller host memory with a communicator -- the analogue of the
 * reference's ibv_reg_mr on its payload buffers (api.c:170-176).  It is pinned
 * (hipHostRegister) until inccl_host_deregister or communicator destroy, and
 * inccl_allreduce_write / _sendrecv whose src and dst both lie inside registered
 * ranges DMA them directly from pinned memory.  Unregistered memory is DMAed
 * too, through HIP's pageable copies with the device-to-host copies issued from
 * a helper thread ($INCCL_HOST_STAGING=pool: staging copies through the
 * communicator's pinned buffers instead).  At most 16 ranges per communicator.
 * The memory must stay allocated while registered. */
int inccl_host_register(struct inccl_communicator *comm, void *ptr, size_t bytes);
int inccl_host_deregister(struct inccl_communicator *comm, void *ptr);

/* bfloat16 buckets (uint16_t bit patterns), same arithmetic on the widened
 * values: dst = bf16_rne( (float)( sum over ranks, sum over r<R  quant(srcs[r]) ) * 2^-k ).
 * world == 1: one fused kernel, (R + 1) * 2 * n HBM bytes.  world > 1:
 *   "rccl" and the in-process transport: quant+local sum -> reduce-scatter
 *     (int32) -> dequantise own shard to bf16 -> all-gather (bf16, half the fp32
 *     gather's bytes);
 *   "mesh" / "meshw": the persistent kernel with bf16 sources and bf16 result
 *     chunks;
 *   "p2p" (4-byte aligned dst): int32 shards pulled and reduced, bf16 result
 *     shards gathered;
 *   "ar", "a2a", "ll": quant+local sum -> that engine's int32 allreduce ->
 *     dequantise.
 * dst may alias srcs[0]. */
int inccl_allreduce_bf16(struct inccl_communicator *comm, const uint16_t *const *srcs_dev, int R, uint16_t *dst_dev,
                         size_t n, int scale_exp, void *stream);
/* max |x| over R bf16 buckets into *amax_bits_dev (as fp32 bits; NaN ignored). */
int inccl_absmax_bf16(const uint16_t *const *srcs_dev, int R, size_t n, uint32_t *amax_bits_dev, int zero_first,
                      void *stream);

/* IEEE binary16 buckets (uint16_t bit patterns), the same arithmetic:
 * dst = f16_rne( (float)( sum over ranks, sum over r<R  quant(srcs[r]) ) * 2^-k ).
 * world == 1: one fused kernel, (R + 1) * 2 * n HBM bytes.  world > 1: the
 * engines route it as bf16 (2-byte result exchange on "rccl", the in-process
 * transport, "p2p", "mesh" and "meshw"; "ar", "a2a", "ll": int32 allreduce,
 * then dequantise).  dst may alias srcs[0]. */
int inccl_allreduce_f16(struct inccl_communicator *comm, const uint16_t *const *srcs_dev, int R, uint16_t *dst_dev,
                        size_t n, int scale_exp, void *stream);
/* max |x| over R fp16 buckets into *amax_bits_dev (as fp32 bits; NaN ignored). */
int inccl_absmax_f16(const uint16_t *const *srcs_dev, int R, size_t n, uint32_t *amax_bits_dev, int zero_first,
                     void *stream);

/* Reduce-scatter: the allreduce's first half, for callers that keep their
 * gradients sharded (ZeRO / FSDP-style optimisers).  Every rank passes R local
 * buckets of n = W * shard elements; rank r receives in dst_dev (shard
 * elements) the dequantised sum over every rank and bucket of elements
 * [r * shard, (r + 1) * shard) -- bit-identical to that slice of the
 * allreduce's result (the same scale, average mode and non-finite mode).
 * n % W != 0 is INCCL_ERR_ARG.  Routes: world 1 the fused kernel; "rccl" and
 * the in-process transport quant + local sum -> int32 reduce-scatter ->
 * dequantise the shard; "ll" with an fp32 bucket of at most INCCL_LL_MAX_BYTES
 * (shard % 4 == 0): its one kernel, this rank's shard summed from every peer's
 * published quads; "mesh" / "meshw" with INCCL_MESH_RS=1 (opt-in, shard % 64
 * == 0, dst aligned as below): the persistent kernel, each reduce writing its
 * chunk of the shard into dst -- off by default: it returned wrong shards at 8
 * processes and 256 MiB and faulted at 4 processes on one GPU;
 * "p2p", "ll", "mesh", "meshw" (shard % 4 == 0, dst
 * 16-B aligned for fp32, 8-B for 2-byte kinds) quant + local sum into the IPC
 * buffer -> barrier -> one kernel pulls shard r from every peer, sums and
 * dequantises into dst -> barrier; otherwise the engine's int32 allreduce and
 * the shard dequantised.  dst must not alias any source. */
int inccl_reduce_scatter_f32(struct inccl_communicator *comm, const float *const *srcs_dev, int R, float *dst_dev,
                             size_t n, int scale_exp, void *stream);
int inccl_reduce_scatter_bf16(struct inccl_communicator *comm, const uint16_t *const *srcs_dev, int R,
                              uint16_t *dst_dev, size_t n, int scale_exp, void *stream);
int inccl_reduce_scatter_f16(struct inccl_communicator *comm, const uint16_t *const *srcs_dev, int R,
                             uint16_t *dst_dev, size_t n, int scale_exp, void *stream);

/* Host-memory fp32 allreduce (BASELINE config 3): src/dst in host memory,
 * pipelined H2D / reduce / D2H over `bucket_bytes` buckets on three streams.
 * Synchronous. */
int inccl_allreduce_f32_host(struct inccl_communicator *comm, const float *src_host, float *dst_host, size_t n,
                             int scale_exp, size_t bucket_bytes);

/* ---------- the reference switch's dataplane on the GPU ----------
 * non_termination_switch.c:303-501 (parse, per-PSN first-arrival aggregation,
 * broadcast / replay, ACK reflection) and util.c:331-442 (egress frame build,
 * payload htonl, RoCE ICRC), batched: a batch of ingress frames -> ingress
 * (claim, classify, sum) -> egress, or one inccl_switch_batch call.  Frames live in device memory at a fixed `stride` (multiple of
 * 4 B, at least 64; every read stays inside a frame's row).  Frame order within
 * a batch is the arrival order: the actions are exactly those of the reference
 * processing the batch's frames one at a time (the first copy of a (psn, port)
 * pair is added; a later copy is REPLAYed if the PSN completed before it, else
 * DROPPED).  A batch must not hold two PSNs that are slots/2 or more apart (the
 * reference: window 8 of 16 slots), so that no two share a slot or a recycle. */
#define INCCL_SW_IGNORED 0    /* opcode the switch does not handle             */
#define INCCL_SW_ABSORBED 1   /* first arrival, slot not complete (nts.c:359-363) */
#define INCCL_SW_COMPLETED 2  /* first arrival completing the slot: broadcast (nts.c:365-372) */
#define INCCL_SW_DROPPED 3    /* retransmit into an incomplete slot (nts.c:353) */
#define INCCL_SW_REPLAY 4     /* retransmit of a completed slot: resend to its port (nts.c:354-356) */
#define INCCL_SW_ACK 5        /* UP ACK: egress reflects a 62-B ACK to its port (nts.c:403-406) */
#define INCCL_SW_INVALID 6    /* bad port or payload length (nts.c:350) */
#define INCCL_SW_FORWARD 7    /* non-root: the slot's aggregate to the parent (nts.c:394-397, :476-479;
                               * a resend after a round of retransmits, :381-384, :462-465) */
#define INCCL_SW_DOWN 8       /* non-root: the parent's result, taken and sent to every child (nts.c:412-419) */

/* Non-root switch options (inccl_switch_create_nonroot); 0 is the reference. */
#define INCCL_SW_WIRE_ORDER 1 /* children get the parent's words as sent; the reference reverses
                               * each word's bytes (memcpy of wire words, nts.c:413, then htonl) */
#define INCCL_SW_RECYCLE 2    /* clear slot psn + slots/2 when the parent's result for psn is taken,
                               * as the root does at completion; the reference never recycles a
                               * non-root slot, so its ring serves `slots` PSNs and no more */

/* One child connection (the fields of util.h connection_t that egress uses). */
struct inccl_frame_template {
    uint8_t src_mac[6], dst_mac[6];
    uint32_t src_ip, dst_ip;        /* as stored in the IP header */
    uint16_t src_port, dst_port;    /* host order (util.c:368-370) */
    uint32_t qp;                    /* peer QPN (util.c:384) */
};
struct inccl_switch;

/* fan_in children (1..31), `slots` PSN slots (power of two), on `device` (-1 = current). */
struct inccl_switch *inccl_switch_create(int fan_in, uint32_t slots, int device);
/* A non-root switch (nts.c:376-400, :408-423, :457-499): children on ports 0..fan_in-1 and the
 * parent on port fan_in; `flags` INCCL_SW_WIRE_ORDER | INCCL_SW_RECYCLE.  Ingress and egress as
 * below with fan_in + 1 rows (and templates) per input frame, row fan_in being the parent's:
 *   FORWARD  the parent's row: the aggregate, the frame's opcode, a zeroed RETH for WRITE_FIRST /
 *            ONLY (send_roce_data_with_reth(FAN_IN, NULL), nts.c:464, :478)
 *   DOWN     every child: the parent's result with the parent frame's opcode and the child's
 *            kept RETH; a parent frame arriving before every child's, or after one was taken,
 *            is DROPPED (nts.c:412, :420-422); an ACK from the parent is IGNORED (:424-426)
 *   REPLAY   the retransmitting child: the parent's result (nts.c:378-380)
 * Each slot's frames of a batch are decided in arrival order, one slot per lane, so a batch
 * costs more the more copies one PSN has in it (up to 8 per slot are kept in LDS, more are walked). */
struct inccl_switch *inccl_switch_create_nonroot(int fan_in, uint32_t slots, int device, int flags);
/* device pointer of a non-root's result slot for `psn`: what the reference's aggregator holds once
 * the parent's result is taken (its wire words, or host words with INCCL_SW_WIRE_ORDER); the
 * aggregate sent up stays in inccl_switch_slot.  NULL for a root. */
const int32_t *inccl_switch_result(struct inccl_switch *sw, uint32_t psn);
int inccl_switch_destroy(struct inccl_switch *sw);
int inccl_switch_reset(struct inccl_switch *sw, void *stream);
/* device pointer of the 256-lane aggregator slot of `psn`: the wrap-around sum of the arrivals counted
 * since the slot was last recycled, while its arrival bitmap is non-zero.  A recycle (nts.c:235-242)
 * clears the slot's bitmap, degree and RETH keeper; its words are stale until the next counted
 * arrival rewrites them (the next sum starts from zero without reading them). */
const int32_t *inccl_switch_slot(struct inccl_switch *sw, uint32_t psn);
/* ports_dev[i] = ingress port of frame i.  Writes action_dev[i] (INCCL_SW_*) and psn_dev[i], and
 * recycles slot psn + slots/2 of every psn the batch completes (clear_state_data(psn + WINDOW),
 * nts.c:367, which the reference runs at completion, in its ingress pipeline). */
int inccl_switch_ingress(struct inccl_switch *sw, const uint8_t *frames_dev, size_t stride, size_t count,
                         const int32_t *ports_dev, int32_t *action_dev, uint32_t *psn_dev, void *stream);
/* Rows per input frame: rows = fan_in for a root switch, fan_in + 1 for a
 * non-root switch (the parent's row last, index fan_in).  For every COMPLETED
 * frame i: fan_in egress frames to children c at out_dev[(i*rows + c) *
 * out_stride] with frame i's opcode (and, for a WRITE_FIRST / WRITE_ONLY opcode,
 * child c's kept RETH); for every REPLAY frame: one such frame to its port; for
 * every ACK frame: the 62-B ACK of send_roce_ack (opcode 0x11, its PSN, AETH
 * MSN = PSN + 1) to its port; a non-root switch also uses row fan_in for the
 * frame it sends up.  out_len_dev[i*rows + c] = frame bytes or 0 (bytes past a
 * frame, up to its 16-byte rounded length, are written as zero or left as they
 * were).  templates_dev holds `rows` inccl_frame_template records (device
 * memory): children 0..fan_in-1, then the parent's for a non-root switch.
 * Size out_dev, out_len_dev and templates_dev for `rows`, not fan_in. */
int inccl_switch_egress(struct inccl_switch *sw, const uint8_t *frames_dev, size_t stride, size_t count,
                        const int32_t *ports_dev, const int32_t *action_dev, const uint32_t *psn_dev,
                        const struct inccl_frame_template *templates_dev, uint8_t *out_dev, size_t out_stride,
                        int32_t *out_len_dev, void *stream);
/* inccl_switch_ingress followed by inccl_switch_egress of the same batch, in
 * one call (the reference's pipeline() runs both per frame): the same actions,
 * state, out rows and lengths (`rows` per frame, as for inccl_switch_egress:
 * fan_in + 1 on a non-root switch), from the same kernels on `stream`. */
int inccl_switch_batch(struct inccl_switch *sw, const uint8_t *frames_dev, size_t stride, size_t count,
                       const int32_t *ports_dev, int32_t *action_dev, uint32_t *psn_dev,
                       const struct inccl_frame_template *templates_dev, uint8_t *out_dev, size_t out_stride,
                       int32_t *out_len_dev, void *stream);
/* RoCE ICRC (util.c:250-286) of `count` frames: icrc_dev[i] as the frame would store it (host order). */
int inccl_icrc_frames(const uint8_t *frames_dev, size_t stride, size_t count, uint32_t *icrc_dev, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* INCCL_AMD_H */
