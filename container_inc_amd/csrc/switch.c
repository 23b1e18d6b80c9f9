/* switch.c -- host side of the GPU switch dataplane (inccl_frames.hip), the
 * root switch (inccl_switch_create) and the non-root one
 * (inccl_switch_create_nonroot: children below port fan_in, the parent on it,
 * nts.c:376-400, :408-423, :457-499).
 *
 * The reference's root switch keeps its aggregation state in globals
 * (non_termination_switch.c:55-60) and processes one frame at a time on one
 * CPU thread (nts.c:508-530).  Here the state lives in HBM and frames are
 * processed in batches: ingress launches (claim, classify, sum: parse +
 * idempotent add + the recycle, clear_state_data(psn + window), nts.c:303-483,
 * :235-242, :367) and one egress launch (broadcast / replay frames and ACK
 * reflections, frame build + ICRC, util.c:331-442) -- or one inccl_switch_batch
 * call that issues the same four launches on one stream.  No host state changes per batch,
 * so a batch's launches can be captured in a hipGraph and replayed.  A batch must span
 * fewer than slots/2 PSNs -- the reference's window of 8 packets over 16 slots
 * (nts.c:21-22) has the same ratio. */
#define _GNU_SOURCE
#include <stdlib.h>
#include <string.h>

#include "inccl_frames.h"
#include "inccl_internal.h"

struct inccl_switch {
    InccSwitchState st;
    void *mem;
    size_t bytes;
    size_t first_off;   /* the first-arrival table (root) or the slots' list heads (non-root): all-ones */
    int device;
    size_t link_cap;    /* non-root: frames the per-frame list links hold */
};

static int kerr2(int rc, const char *what)
{
    if (rc == 0) return 0;
    if (rc == INCCL_ERR_ARG) return inccl_set_error(rc, "%s: invalid argument", what);
    return inccl_set_error(INCCL_ERR_HIP, "%s: %s", what, hipGetErrorString((hipError_t)rc));
}

struct inccl_switch *inccl_switch_create(int fan_in, uint32_t slots, int device)
{
    if (fan_in < 1 || fan_in > 31 || slots < 2 || (slots & (slots - 1)) != 0) {
        inccl_set_error(INCCL_ERR_ARG, "switch: fan_in must be 1..31 and slots a power of two >= 2");
        return NULL;
    }
    if (device >= 0 && hipSetDevice(device) != hipSuccess) {
        inccl_set_error(INCCL_ERR_HIP, "switch: hipSetDevice(%d) failed", device);
        return NULL;
    }
    struct inccl_switch *sw = (struct inccl_switch *)calloc(1, sizeof(*sw));
    if (!sw) return NULL;
    const size_t agg = (size_t)slots * 256 * sizeof(int32_t);
    const size_t arr = (size_t)slots * 2 * sizeof(uint64_t);
    const size_t deg = (size_t)slots * sizeof(int32_t);
    const size_t reth = (size_t)slots * (size_t)fan_in * 16;
    const size_t first = (size_t)slots * (size_t)fan_in * 8;
    const size_t gen = 16;   /* the batch-generation words (zeroed with the state) */
    sw->first_off = (agg + arr + deg + reth + gen + 7) & ~(size_t)7;
    sw->bytes = sw->first_off + first;
    hipError_t e = hipMalloc(&sw->mem, sw->bytes);
    if (e == hipSuccess) e = hipMemset(sw->mem, 0, sw->first_off);
    if (e == hipSuccess) e = hipMemset((char *)sw->mem + sw->first_off, 0xFF, first);   /* no batch yet */
    if (e != hipSuccess) {
        inccl_hip_check(e, "switch: hipMalloc");
        if (sw->mem) hipFree(sw->mem);
        free(sw);
        return NULL;
    }
    char *p = (char *)sw->mem;
    sw->st.agg = (int32_t *)p;
    sw->st.arrival = (uint64_t *)(p + agg);
    sw->st.degree = (int32_t *)(p + agg + arr);
    sw->st.reth = (uint32_t *)(p + agg + arr + deg);
    sw->st.gen = (uint32_t *)(p + agg + arr + deg + reth);
    sw->st.first = (uint64_t *)(p + sw->first_off);
    sw->st.slots = slots;
    sw->st.fan_in = fan_in;
    hipGetDevice(&sw->device);
    if (kerr2(inccl_k_frames_init(), "switch: CRC tables")) {
        hipFree(sw->mem);
        free(sw);
        return NULL;
    }
    return sw;
}

struct inccl_switch *inccl_switch_create_nonroot(int fan_in, uint32_t slots, int device, int flags)
{
    if (fan_in < 1 || fan_in > 31 || slots < 2 || (slots & (slots - 1)) != 0 || slots > (1u << 24) ||
        (flags & ~(INCCL_SW_WIRE_ORDER | INCCL_SW_RECYCLE))) {
        inccl_set_error(INCCL_ERR_ARG, "switch: fan_in must be 1..31, slots a power of two in 2..2^24, "
                                       "flags INCCL_SW_WIRE_ORDER | INCCL_SW_RECYCLE");
        return NULL;
    }
    if (device >= 0 && hipSetDevice(device) != hipSuccess) {
        inccl_set_error(INCCL_ERR_HIP, "switch: hipSetDevice(%d) failed", device);
        return NULL;
    }
    struct inccl_switch *sw = (struct inccl_switch *)calloc(1, sizeof(*sw));
    if (!sw) return NULL;
    /* zeroed: agg, res, bits, degree, reth; all-ones: head (the per-batch
     * list links and work records grow with the batch, ensure_batch_mem) */
    const size_t S = slots;
    const size_t agg = S * 256 * sizeof(int32_t), words = S * sizeof(uint32_t);
    const size_t reth = S * (size_t)fan_in * 16;
    const size_t zero_end = (2 * agg + 2 * words + reth + 15) & ~(size_t)15;
    sw->first_off = zero_end;
    sw->bytes = zero_end + words;
    hipError_t e = hipMalloc(&sw->mem, sw->bytes);
    if (e == hipSuccess) e = hipMemset(sw->mem, 0, zero_end);
    if (e == hipSuccess) e = hipMemset((char *)sw->mem + zero_end, 0xFF, words);
    if (e != hipSuccess) {
        inccl_hip_check(e, "switch: hipMalloc");
        if (sw->mem) hipFree(sw->mem);
        free(sw);
        return NULL;
    }
    char *p = (char *)sw->mem;
    sw->st.agg = (int32_t *)p;
    sw->st.res = (int32_t *)(p + agg);
    sw->st.bits = (uint32_t *)(p + 2 * agg);
    sw->st.degree = (int32_t *)(p + 2 * agg + words);
    sw->st.reth = (uint32_t *)(p + 2 * agg + 2 * words);
    sw->st.head = (uint32_t *)(p + zero_end);
    sw->st.slots = slots;
    sw->st.fan_in = fan_in;
    sw->st.nonroot = 1;
    sw->st.flags = flags;
    hipGetDevice(&sw->device);
    if (kerr2(inccl_k_frames_init(), "switch: CRC tables")) {
        hipFree(sw->mem);
        free(sw);
        return NULL;
    }
    return sw;
}

const int32_t *inccl_switch_result(struct inccl_switch *sw, uint32_t psn)
{
    if (!sw || !sw->st.nonroot) return NULL;
    return sw->st.res + (size_t)(psn & (sw->st.slots - 1)) * 256;
}

/* a non-root batch of `count` frames needs count list links and its work
 * records (inccl_k_nr_work_words; grown outside stream capture: a captured
 * batch must follow an uncaptured one as large) */
static int ensure_links(struct inccl_switch *sw, size_t count, void *stream)
{
    if (!sw->st.nonroot || count <= sw->link_cap) return 0;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (stream && hipStreamIsCapturing((hipStream_t)stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
        return inccl_set_error(INCCL_ERR_ARG, "non-root switch: a captured batch of %zu frames needs an earlier "
                                              "uncaptured batch at least as large (list links)", count);
    if (sw->st.link) {
        hipDeviceSynchronize();
        hipFree(sw->st.link);
        sw->st.link = NULL;
        sw->st.work = NULL;
        sw->link_cap = 0;
    }
    const size_t link = count * 2 * sizeof(uint32_t);
    INCCL_HIP(hipMalloc((void **)&sw->st.link, link + inccl_k_nr_work_words(count, sw->st.fan_in) * sizeof(uint32_t)));
    sw->st.work = sw->st.link + count * 2;
    sw->link_cap = count;
    return 0;
}

int inccl_switch_destroy(struct inccl_switch *sw)
{
    if (!sw) return 0;
    hipSetDevice(sw->device);
    hipDeviceSynchronize();
    hipFree(sw->mem);
    if (sw->st.link) hipFree(sw->st.link);
    free(sw);
    return 0;
}

int inccl_switch_reset(struct inccl_switch *sw, void *stream)
{
    if (!sw) return inccl_set_error(INCCL_ERR_ARG, "switch is NULL");
    INCCL_HIP(hipMemsetAsync(sw->mem, 0, sw->first_off, (hipStream_t)stream));
    const size_t ones = sw->st.nonroot ? (size_t)sw->st.slots * sizeof(uint32_t) : sw->bytes - sw->first_off;
    INCCL_HIP(hipMemsetAsync((char *)sw->mem + sw->first_off, 0xFF, ones, (hipStream_t)stream));
    return 0;
}

const int32_t *inccl_switch_slot(struct inccl_switch *sw, uint32_t psn)
{
    if (!sw) return NULL;
    return sw->st.agg + (size_t)(psn & (sw->st.slots - 1)) * 256;
}

int inccl_switch_ingress(struct inccl_switch *sw, const uint8_t *frames_dev, size_t stride, size_t count,
                         const int32_t *ports_dev, int32_t *action_dev, uint32_t *psn_dev, void *stream)
{
    if (!sw) return inccl_set_error(INCCL_ERR_ARG, "switch is NULL");
    if (count && stride < INCCL_FRAME_MIN_STRIDE)
        return inccl_set_error(INCCL_ERR_ARG, "inccl_switch_ingress: stride %zu below %d", stride, INCCL_FRAME_MIN_STRIDE);
    /* a new batch: its first-arrival keys outrank every earlier batch's (the
     * generation is a device word the batch's commit advances, so a captured
     * batch stays correct on replay; switch state is per stream-ordered call
     * sequence, like the reference's globals) */
    const int rc = ensure_links(sw, count, stream);
    if (rc) return rc;
    return kerr2(inccl_k_switch_ingress(&sw->st, frames_dev, stride, count, ports_dev, action_dev, psn_dev, stream),
                 "inccl_switch_ingress");
}

int inccl_switch_batch(struct inccl_switch *sw, const uint8_t *frames_dev, size_t stride, size_t count,
                       const int32_t *ports_dev, int32_t *action_dev, uint32_t *psn_dev,
                       const struct inccl_frame_template *templates_dev, uint8_t *out_dev, size_t out_stride,
                       int32_t *out_len_dev, void *stream)
{
    if (!sw) return inccl_set_error(INCCL_ERR_ARG, "switch is NULL");
    if (count && stride < INCCL_FRAME_MIN_STRIDE)
        return inccl_set_error(INCCL_ERR_ARG, "inccl_switch_batch: stride %zu below %d", stride, INCCL_FRAME_MIN_STRIDE);
    const int rc = ensure_links(sw, count, stream);
    if (rc) return rc;
    return kerr2(inccl_k_switch_batch(&sw->st, frames_dev, stride, count, ports_dev, action_dev, psn_dev,
                                      templates_dev, out_dev, out_stride, out_len_dev, stream),
                 "inccl_switch_batch");
}

int inccl_switch_egress(struct inccl_switch *sw, const uint8_t *frames_dev, size_t stride, size_t count,
                        const int32_t *ports_dev, const int32_t *action_dev, const uint32_t *psn_dev,
                        const struct inccl_frame_template *templates_dev, uint8_t *out_dev, size_t out_stride,
                        int32_t *out_len_dev, void *stream)
{
    if (!sw) return inccl_set_error(INCCL_ERR_ARG, "switch is NULL");
    if (count && stride < INCCL_FRAME_MIN_STRIDE)
        return inccl_set_error(INCCL_ERR_ARG, "inccl_switch_egress: stride %zu below %d", stride, INCCL_FRAME_MIN_STRIDE);
    return kerr2(inccl_k_switch_egress(&sw->st, frames_dev, stride, count, ports_dev, action_dev, psn_dev,
                                       templates_dev, out_dev, out_stride, out_len_dev, stream),
                 "inccl_switch_egress");
}

int inccl_icrc_frames(const uint8_t *frames_dev, size_t stride, size_t count, uint32_t *icrc_dev, void *stream)
{
    if (count && stride < INCCL_FRAME_MIN_STRIDE)
        return inccl_set_error(INCCL_ERR_ARG, "inccl_icrc_frames: stride %zu below %d", stride, INCCL_FRAME_MIN_STRIDE);
    return kerr2(inccl_k_icrc(frames_dev, stride, count, icrc_dev, stream), "inccl_icrc_frames");
}
