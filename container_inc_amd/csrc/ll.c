/* ll.c -- host side of the "ll" engine: the one-kernel allreduce for small
 * buckets (kernel and protocol in inccl_ll.hip).
 *
 * The p2p engine (p2p.c) pays two stream synchronisations and two host
 * barriers per call -- tens of microseconds that dominate below ~1 MiB.  Here a
 * call is one kernel launch: ranks meet through arrival flags that the kernel
 * writes into the peers' memory, the switch's arrival bitmap
 * (non_termination_switch.c:361-365) kept in HBM.
 *
 * Per rank, one device allocation shared over HIP IPC:
 *   [0, 32 KiB)                  signal array: W x INCCL_LL_MAX_BLOCKS words,
 *                                word [j][b] = last call whose block b of rank j arrived
 *   [32 KiB, +8)                 call counter + retired-workgroup count (own use)
 *   [64 KiB, +cap*4)             data slot of even calls (int32 partial sums)
 *   [64 KiB + cap*4, +cap*4)     data slot of odd calls
 * Created collectively on the first ll call (all ranks make the same calls). */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "inccl_internal.h"
#include "inccl_kernels.h"

#define LL_SIG_BYTES ((size_t)65536)   /* signals + counters; keeps the data slots 64 KiB aligned */
#define LL_CTR_OFFSET ((size_t)32768)  /* after the 8 x 256 signal words */

void inccl_ll_release(struct inccl_communicator *c)
{
    const int W = c->group->world_size, me = c->group->rank;
    if (!c->ll_buf) return;
    hipDeviceSynchronize();
    for (int j = 0; j < W && j < INCCL_MAX_LOCAL_INPUTS; ++j) {
        if (j != me && c->ll_peer[j]) hipIpcCloseMemHandle(c->ll_peer[j]);
        c->ll_peer[j] = NULL;
    }
    hipFree(c->ll_buf);
    c->ll_buf = NULL;
    if (c->ll_err_host) hipHostFree(c->ll_err_host);
    c->ll_err_host = NULL;
    c->ll_err_dev = NULL;
    c->ll_cap = 0;
}

static int ll_ensure(struct inccl_communicator *c)
{
    struct inccl_group *g = c->group;
    const int W = g->world_size, me = g->rank;
    if (c->ll_buf) return 0;
    if (W > INCCL_MAX_LOCAL_INPUTS)
        return inccl_set_error(INCCL_ERR_ARG, "ll engine supports up to %d GPUs", INCCL_MAX_LOCAL_INPUTS);
    int rc = 0;
    const size_t cap = (c->ll_max_bytes / 4 + 1023) & ~(size_t)1023;
    hipIpcMemHandle_t mine, all[INCCL_MAX_LOCAL_INPUTS];
    memset(&mine, 0, sizeof(mine));
    /* local failures are carried to the collective outcome check below */
    hipError_t e = inccl_ipc_malloc((void **)&c->ll_buf, LL_SIG_BYTES + 2 * cap * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(c->ll_buf, 0, LL_SIG_BYTES);   /* synchronous: zero before any peer maps it */
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipIpcGetMemHandle(&mine, c->ll_buf);
    if (e == hipSuccess) e = hipHostMalloc((void **)&c->ll_err_host, sizeof(uint32_t), hipHostMallocMapped);
    if (e == hipSuccess) {
        *(volatile uint32_t *)c->ll_err_host = 0;
        e = hipHostGetDevicePointer((void **)&c->ll_err_dev, c->ll_err_host, 0);
    }
    if (e != hipSuccess) rc = inccl_hip_check(e, "ll: buffer setup");
    int rc_x = inccl_boot_allgather(g, &mine, all, sizeof(hipIpcMemHandle_t));
    if (rc_x) {
        inccl_ll_release(c);   /* back to a clean state: the next call starts over */
        return rc_x;
    }
    for (int j = 0; rc == 0 && j < W; ++j) {
        if (j == me) {
            c->ll_peer[j] = c->ll_buf;
            continue;
        }
        void *p = NULL;
        e = hipIpcOpenMemHandle(&p, all[j], hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) rc = inccl_hip_check(e, "ll: hipIpcOpenMemHandle");
        c->ll_peer[j] = (char *)p;
    }
    /* agree on the outcome, so that every rank falls back alike */
    int32_t mine_rc = rc ? 1 : 0, all_rc[INCCL_MAX_LOCAL_INPUTS];
    int rc2 = inccl_boot_allgather(g, &mine_rc, all_rc, sizeof(int32_t));
    if (rc2) return rc2;
    for (int j = 0; j < W; ++j)
        if (all_rc[j]) {
            if (!rc) rc = inccl_set_error(INCCL_ERR_HIP, "ll: rank %d could not map the peer buffers", j);
            inccl_ll_release(c);
            return rc;
        }
    c->ll_cap = cap;
    c->ll_last_stream = NULL;
    if (c->ll_timeout_ticks == 0) c->ll_timeout_ticks = inccl_wait_ticks(g);
    return 0;
}

/* device wall-clock ticks of a bounded in-kernel wait: $INCCL_LL_TIMEOUT_MS (5 s) */
uint64_t inccl_wait_ticks(struct inccl_group *g)
{
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, g->device >= 0 ? g->device : 0) != hipSuccess ||
        khz <= 0)
        khz = 100000;   /* 100 MHz, the CDNA constant clock */
    const char *t = getenv("INCCL_LL_TIMEOUT_MS");
    const double ms = t ? atof(t) : 5000.0;
    return (uint64_t)(ms * (double)khz);
}

int inccl_ll_piece(struct inccl_communicator *c, const float *const *srcs, int R, float *dst, size_t n, int k,
                   const uint32_t *amax, int scale_R, size_t rs_lo, size_t rs_n, hipStream_t st)
{
    const int W = c->group->world_size, me = c->group->rank;
    if (!c->ll_buf) {   /* the collective setup cannot run inside a graph capture */
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        INCCL_HIP(hipStreamIsCapturing(st, &cap));
        if (cap != hipStreamCaptureStatusNone)
            return inccl_set_error(INCCL_ERR_STATE, "ll: make one call outside graph capture first (collective setup)");
    }
    int rc = ll_ensure(c);
    if (rc) return rc;
    if (n > c->ll_cap) return inccl_set_error(INCCL_ERR_ARG, "ll: %zu elements exceed the slot (%zu)", n, c->ll_cap);
    if (*(volatile uint32_t *)c->ll_err_host)
        return inccl_set_error(INCCL_ERR_STATE, "ll: an earlier call timed out waiting for a peer (results invalid)");
    struct inccl_ll_launch l;
    memset(&l, 0, sizeof(l));
    for (int r = 0; r < R; ++r) l.src[r] = srcs[r];
    l.R = R;
    l.dst = dst;
    l.n = n;
    l.own_data = (uint32_t *)(c->ll_buf + LL_SIG_BYTES);
    l.slot_elems = c->ll_cap;
    for (int j = 0; j < W; ++j) {
        l.peer_data[j] = (const uint32_t *)(c->ll_peer[j] + LL_SIG_BYTES);
        l.peer_sig[j] = (uint32_t *)c->ll_peer[j];
    }
    l.own_sig = (const uint32_t *)c->ll_buf;
    l.ctr = (uint32_t *)(c->ll_buf + LL_CTR_OFFSET);
    l.err = c->ll_err_dev;
    l.W = W;
    l.me = me;
    l.timeout_ticks = c->ll_timeout_ticks;
    l.scale_exp = k;
    l.amax_bits = amax;
    l.scale_R = scale_R;
    l.out_shift = c->out_shift;
    l.rs_lo = rs_lo;
    l.rs_n = rs_n;
    /* the parity argument needs this rank's calls in order: chain across streams
     * (inside a graph capture the caller's single capture stream orders them) */
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    INCCL_HIP(hipStreamIsCapturing(st, &cap));
    const int capturing = cap != hipStreamCaptureStatusNone;
    if (!capturing && c->ll_last_stream && c->ll_last_stream != st) INCCL_HIP(hipStreamWaitEvent(st, c->ev[7], 0));
    /* $INCCL_LL_CHECK (debugging aid, eager calls only): wait before and after
     * the call and check that the device call counter advanced by exactly one
     * and the retire counter is back at 0 */
    const int check = !capturing && getenv("INCCL_LL_CHECK") != NULL;
    uint32_t before[2] = {0, 0}, after[2] = {0, 0};
    if (check) {
        INCCL_HIP(hipStreamSynchronize(st));
        INCCL_HIP(hipMemcpy(before, l.ctr, sizeof(before), hipMemcpyDeviceToHost));
    }
    rc = inccl_k_ll_oneshot(&l, st);
    if (rc) return inccl_set_error(INCCL_ERR_HIP, "ll kernel launch failed (%d)", rc);
    if (!capturing) {
        INCCL_HIP(hipEventRecord(c->ev[7], st));
        c->ll_last_stream = st;
    }
    if (check) {
        INCCL_HIP(hipStreamSynchronize(st));
        INCCL_HIP(hipMemcpy(after, l.ctr, sizeof(after), hipMemcpyDeviceToHost));
        if (after[0] != before[0] + 1 || before[1] != 0 || after[1] != 0)
            fprintf(stderr, "[inccl ll rank %d] n %zu grid %d: call counter %u -> %u, retired %u -> %u\n", me, n,
                    inccl_k_ll_grid(n), before[0], after[0], before[1], after[1]);
    }
    return 0;
}
