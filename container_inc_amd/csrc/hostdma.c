/* hostdma.c -- a per-communicator thread that issues the device-to-host copies
 * of the host-memory pipeline (inccl_allreduce_write / _sendrecv on memory the
 * caller did not register; the reference's api.c:403-452 path as host.c calls
 * it, on plain malloc'ed buffers).
 *
 * HIP copies to or from pageable memory return only when the bytes have been
 * moved (HIP stages them itself), so one host thread issuing chunk i+1's H2D and
 * chunk i's D2H runs them one after the other: 25.7 GB/s for a 256 MiB message
 * on MI355X against 56 GB/s for each direction alone
 * (tools/api_write_probe.py SERIES=30).  With the D2Hs issued from this thread,
 * the two directions are in flight together, as with registered memory.
 *
 * Jobs run strictly in posting order.  The caller learns how many have been
 * issued (i.e. finished, for pageable memory) through inccl_d2h_wait_issued. */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "inccl_internal.h"

#define D2H_RING 4

struct d2h_job {
    void *dst;
    const void *src;
    size_t bytes;
    hipEvent_t after, done;
    hipStream_t st;
};

struct inccl_d2h_worker {
    pthread_t th;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    struct d2h_job ring[D2H_RING];
    unsigned long long posted, issued;
    hipError_t err;        /* first failure, sticky until inccl_d2h_reset */
    int device;
    int quit;
};

static void *d2h_main(void *arg)
{
    struct inccl_d2h_worker *w = (struct inccl_d2h_worker *)arg;
    hipSetDevice(w->device);
    pthread_mutex_lock(&w->mu);
    for (;;) {
        while (w->issued == w->posted && !w->quit) pthread_cond_wait(&w->cv, &w->mu);
        if (w->issued == w->posted && w->quit) break;
        const struct d2h_job j = w->ring[w->issued % D2H_RING];
        pthread_mutex_unlock(&w->mu);
        hipError_t e = hipStreamWaitEvent(j.st, j.after, 0);
        if (e == hipSuccess) e = hipMemcpyAsync(j.dst, j.src, j.bytes, hipMemcpyDeviceToHost, j.st);
        if (e == hipSuccess) e = hipEventRecord(j.done, j.st);
        pthread_mutex_lock(&w->mu);
        if (e != hipSuccess && w->err == hipSuccess) w->err = e;
        w->issued++;
        pthread_cond_broadcast(&w->cv);
    }
    pthread_mutex_unlock(&w->mu);
    return NULL;
}

struct inccl_d2h_worker *inccl_d2h_worker_create(int device)
{
    struct inccl_d2h_worker *w = (struct inccl_d2h_worker *)calloc(1, sizeof(*w));
    if (!w) return NULL;
    pthread_mutex_init(&w->mu, NULL);
    pthread_cond_init(&w->cv, NULL);
    w->device = device;
    if (pthread_create(&w->th, NULL, d2h_main, w) != 0) {
        pthread_cond_destroy(&w->cv);
        pthread_mutex_destroy(&w->mu);
        free(w);
        return NULL;
    }
    return w;
}

void inccl_d2h_worker_destroy(struct inccl_d2h_worker *w)
{
    if (!w) return;
    pthread_mutex_lock(&w->mu);
    w->quit = 1;
    pthread_cond_broadcast(&w->cv);
    pthread_mutex_unlock(&w->mu);
    pthread_join(w->th, NULL);   /* drains every posted job first */
    pthread_cond_destroy(&w->cv);
    pthread_mutex_destroy(&w->mu);
    free(w);
}

unsigned long long inccl_d2h_posted(struct inccl_d2h_worker *w)
{
    pthread_mutex_lock(&w->mu);
    const unsigned long long p = w->posted;
    pthread_mutex_unlock(&w->mu);
    return p;
}

void inccl_d2h_post(struct inccl_d2h_worker *w, void *dst, const void *src, size_t bytes, hipEvent_t after,
                    hipEvent_t done, hipStream_t st)
{
    pthread_mutex_lock(&w->mu);
    while (w->posted - w->issued >= D2H_RING) pthread_cond_wait(&w->cv, &w->mu);
    struct d2h_job *j = &w->ring[w->posted % D2H_RING];
    j->dst = dst;
    j->src = src;
    j->bytes = bytes;
    j->after = after;
    j->done = done;
    j->st = st;
    w->posted++;
    pthread_cond_broadcast(&w->cv);
    pthread_mutex_unlock(&w->mu);
}

/* Block until the first `count` jobs ever posted have been issued; returns the
 * first HIP error any job hit (and clears it). */
hipError_t inccl_d2h_wait_issued(struct inccl_d2h_worker *w, unsigned long long count)
{
    pthread_mutex_lock(&w->mu);
    while (w->issued < count) pthread_cond_wait(&w->cv, &w->mu);
    const hipError_t e = w->err;
    w->err = hipSuccess;
    pthread_mutex_unlock(&w->mu);
    return e;
}
