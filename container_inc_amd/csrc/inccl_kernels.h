/* inccl_kernels.h -- the thin C-ABI shim between the C host code and the HIP
 * kernels in inccl_kernels.hip.  Internal to libinccl_amd.so. */
#ifndef INCCL_KERNELS_H
#define INCCL_KERNELS_H

#include <stddef.h>
#include <stdint.h>

#include "inccl_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* out[i] = OUT(sum_r IN(srcs[r][i])), kinds INCCL_KIND_*.  Returns 0 or a hipError_t / INCCL_ERR_ARG. */
int inccl_k_stream(int in_kind, int out_kind, const void *const *srcs, int R, void *dst, size_t n, int scale_exp,
                   const uint32_t *amax_bits_dev, int scale_R, void *stream);
/* the same with the dequantise scaled by 2^-out_shift (inccl_comm_set_average) */
int inccl_k_stream_s(int in_kind, int out_kind, const void *const *srcs, int R, void *dst, size_t n, int scale_exp,
                     const uint32_t *amax_bits_dev, int scale_R, int out_shift, void *stream);
int inccl_k_absmax(const float *const *srcs, int R, size_t n, uint32_t *amax_bits_dev, int zero_first, void *stream);
int inccl_k_absmax_bf16(const uint16_t *const *srcs, int R, size_t n, uint32_t *amax_bits_dev, int zero_first,
                        void *stream);
int inccl_k_absmax_f16(const uint16_t *const *srcs, int R, size_t n, uint32_t *amax_bits_dev, int zero_first,
                        void *stream);
int inccl_k_checksum(const int32_t *q, size_t n, uint64_t index_base, uint32_t *out_dev, int zero_first,
                     void *stream);
void inccl_k_set_tuning(int grid_cap, int nt_loads);
/* p2p engine kernels reading peer memory with system-coherent loads (inccl_peer.hip):
 * dst[i] = dequant(sum_j peers[j][i]), n % 4 == 0, 16-B aligned; and
 * dst[off[j] .. off[j]+cnt[j]) = src[j][0 .. cnt[j]) for j < nseg, one launch */
int inccl_k_peer_reduce(const void *const *peers, int W, float *dst, size_t n, int scale_exp,
                        const uint32_t *amax_bits_dev, int scale_R, int out_shift, void *stream);
int inccl_k_peer_gather(const void *const *src, const int64_t *off, const int64_t *cnt, int nseg, void *dst,
                        void *stream);
/* the pull-reduce with 2-byte results: dst[i] = narrow(dequant(sum_j peers[j][i])), narrow = bf16 (kind
 * INCCL_KIND_BF16) or fp16 (INCCL_KIND_F16) round to nearest even, n % 4 == 0, dst 8-B aligned */
int inccl_k_peer_reduce16(int kind, const void *const *peers, int W, uint16_t *dst, size_t n, int scale_exp,
                          const uint32_t *amax_bits_dev, int scale_R, int out_shift, void *stream);
/* the same gather for 2-byte elements (counts and even offsets in elements; dst 4-B aligned) */
int inccl_k_peer_gather16(const void *const *src, const int64_t *off, const int64_t *cnt, int nseg, void *dst,
                          void *stream);
/* dst[i] = sum_j peers[j][i] (int32, wrapping), n % 4 == 0, 16-B aligned */
int inccl_k_peer_sum_q32(const void *const *peers, int W, int32_t *dst, size_t n, void *stream);

/* the one-kernel small-bucket allreduce (inccl_ll.hip) */
#define INCCL_LL_MAX_BLOCKS 256   /* workgroups per call = flags per rank in a signal array */
struct inccl_ll_launch {
    const float *src[INCCL_MAX_LOCAL_INPUTS];
    int R;
    float *dst;
    size_t n;
    uint32_t *own_data;                                /* own data slot 0; slot 1 at + slot_elems */
    const uint32_t *peer_data[INCCL_MAX_LOCAL_INPUTS]; /* every rank's slot 0, [me] = own_data */
    size_t slot_elems;
    uint32_t *peer_sig[INCCL_MAX_LOCAL_INPUTS];        /* per rank signal arrays (W x MAX_BLOCKS words) */
    const uint32_t *own_sig;
    uint32_t *ctr;                                     /* own device words: [0] calls done, [1] workgroups retired */
    uint32_t *err;                                     /* device view of a host-mapped word */
    int W, me;
    uint64_t timeout_ticks;
    int scale_exp;
    const uint32_t *amax_bits;
    int scale_R;
    int out_shift;                                     /* dequantise with 2^-(k + out_shift) */
    size_t rs_lo, rs_n;                                /* rs_n > 0: reduce-scatter -- dst = elements
                                                        * [rs_lo, rs_lo + rs_n) of the result (both % 4 == 0) */
};
int inccl_k_ll_grid(size_t n);
int inccl_k_ll_oneshot(const struct inccl_ll_launch *l, void *stream);

/* the one-kernel large-bucket allreduce (inccl_mesh.hip): push reduce-scatter,
 * per-chunk arrival flags, pull all-gather */
#define INCCL_MESH_MAX_CHUNKS 1024   /* chunks per shard = flags per source rank */
struct inccl_mesh_launch {
    const float *src[INCCL_MAX_LOCAL_INPUTS];
    int R;
    float *dst;
    size_t n;
    size_t shard;                                      /* elements per rank's shard, multiple of 64 */
    size_t chunk;                                      /* elements per chunk, multiple of 64 */
    size_t inbox_stride;                               /* elements per source slot of an inbox */
    int nchunks, lag, grid;
    uint32_t *peer_inbox[INCCL_MAX_LOCAL_INPUTS];      /* every rank's inbox ([me] = own) */
    const uint32_t *own_inbox;
    uint32_t *own_res;
    const uint32_t *peer_res[INCCL_MAX_LOCAL_INPUTS];  /* every rank's result shard */
    uint32_t *peer_resin[INCCL_MAX_LOCAL_INPUTS];      /* every rank's result inbox (push_res) */
    const uint32_t *own_resin;
    int push_res;                                      /* 1: reduce pushes results, gather copies locally */
    int rs;                                            /* 1: reduce-scatter -- dst is this rank's shard */
    int kind16;                                        /* 0: fp32 src / dst; INCCL_KIND_BF16 / _F16: 2-byte ones */
    uint32_t *peer_sig[INCCL_MAX_LOCAL_INPUTS];        /* every rank's signal array */
    const uint32_t *own_sig;
    uint32_t *ctr;                                     /* own words: calls, retired, ticket, abort */
    uint32_t *err;                                     /* device view of a host-mapped word */
    int W, me;
    uint64_t timeout_ticks;
    int scale_exp;
    const uint32_t *amax_bits;
    int scale_R;
    int out_shift;                                     /* dequantise with 2^-(k + out_shift) */
    /* region sizes for the kernel's per-item bounds check (every rank's regions
     * have the same sizes): a work item whose buffer range falls outside its
     * region stores INCCL_MESH_ERR_BOUNDS | item << 8 | peer << 4 into *err
     * and aborts the call instead of touching memory */
    size_t src_bytes, dst_bytes, inbox_bytes, res_bytes, resin_bytes;
};
#define INCCL_MESH_ERR_TIMEOUT 1u
#define INCCL_MESH_ERR_BOUNDS 2u
int inccl_k_mesh(const struct inccl_mesh_launch *l, void *stream);

#ifdef __cplusplus
}
#endif
#endif
