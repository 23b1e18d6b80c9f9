/* inccl_frames.h -- C-ABI shim between switch.c and the frame kernels in
 * inccl_frames.hip (the reference's switch dataplane on the GPU).  Internal. */
#ifndef INCCL_FRAMES_H
#define INCCL_FRAMES_H

#include <stddef.h>
#include <stdint.h>

#include "inccl_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* device-side state of one root switch (pointers into one allocation) */
typedef struct InccSwitchState {
    int32_t *agg;        /* [slots][256]        non_termination_switch.c:55 */
    uint64_t *arrival;   /* [slots][2]          nts.c:59: {bitmap, tag = the batch that wrote it}, double-buffered:
                          * batch g reads the newer word not tagged g and its leader overwrites the other one,
                          * so every frame of the batch sees the bitmap as it was before it (k_ingress_classify) */
    int32_t *degree;     /* [slots]             nts.c:60 */
    uint32_t *reth;      /* [slots][fan_in][4]  nts.c:57 */
    uint64_t *first;     /* [slots][fan_in]     batch-tagged index of the first copy in a batch:
                          * (~gen << 32) | frame, atomicMin -> the earliest frame of the newest batch */
    uint32_t *gen;       /* gen[0]: batches ingested so far.  A batch's claim tags its first-copy keys with
                          * g = gen[0] + 1 and stores g in gen[1]; its classify reads gen[1] and stores g in
                          * gen[0], so that a captured batch (hipGraph) tags every replay anew */
    uint32_t slots;      /* power of two */
    int fan_in;
    /* a non-root switch (nts.c:376-400, :408-423, :457-499; parent = port fan_in) instead of the
     * root: agg, degree and reth as above; arrival, first and gen unused */
    int nonroot, flags;  /* flags: INCCL_SW_WIRE_ORDER | INCCL_SW_RECYCLE */
    int32_t *res;        /* [slots][256]        the parent's result as the reference's aggregator holds it
                          *                     (nts.c:413: wire words; ntohl'd with INCCL_SW_WIRE_ORDER) */
    uint32_t *bits;      /* [slots]             arrival bitmap: children, bit fan_in = parent's result (nts.c:59) */
    uint32_t *head;      /* [slots]             the batch's frame list of each slot (~0: empty; reset by its owner) */
    uint32_t *work;      /* [inccl_k_nr_work_words]  64 region counters, then per region the records of its
                          *                     classify blocks' slots: PSN | the slot held arrivals before the
                          *                     batch << 31, the parent frame taken, the frame counted for each
                          *                     child (~0: none; bit 31: WRITE_FIRST, payload at byte 70) */
    uint32_t *link;      /* [frames][2]         per frame (one 8-byte word): next frame of its slot's list, port | WF << 8 */
} InccSwitchState;

#define INCCL_FRAME_MIN_STRIDE 64   /* a row must hold the 62-B ACK frame (headers through the BTH) */

typedef struct inccl_frame_template InccFrameTemplate;

int inccl_k_frames_init(void);
/* words of a non-root batch's work records for `count` frames */
size_t inccl_k_nr_work_words(size_t count, int fan_in);
int inccl_k_icrc(const uint8_t *frames, size_t stride, size_t count, uint32_t *out, void *stream);
int inccl_k_switch_ingress(const InccSwitchState *s, const uint8_t *frames, size_t stride, size_t count,
                           const int32_t *ports, int32_t *action, uint32_t *psn_out, void *stream);
int inccl_k_switch_batch(const InccSwitchState *s, const uint8_t *frames, size_t stride, size_t count,
                         const int32_t *ports, int32_t *action, uint32_t *psn_out, const InccFrameTemplate *tmpl,
                         uint8_t *out, size_t out_stride, int32_t *out_len, void *stream);
int inccl_k_switch_egress(const InccSwitchState *s, const uint8_t *in_frames, size_t in_stride, size_t count,
                          const int32_t *ports, const int32_t *action, const uint32_t *psns,
                          const InccFrameTemplate *tmpl, uint8_t *out, size_t out_stride, int32_t *out_len,
                          void *stream);

#ifdef __cplusplus
}
#endif
#endif
