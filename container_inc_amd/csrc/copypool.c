/* copypool.c -- a small persistent thread pool for host memcpy into / out of the
 * pinned staging buffers (the reference's registered MRs, api.c:164-176).
 *
 * The reference encodes and decodes 1024-element messages on the calling thread
 * (api.c:300-302, :428-430).  Here one host thread cannot keep up with PCIe
 * Gen5, so a copy is split over `n` workers that persist for the communicator's
 * lifetime (the reference vendors C-Thread-Pool for its switch; this is the
 * host-side equivalent for the staging copies). */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "inccl_internal.h"

struct inccl_copy_pool {
    int n;
    pthread_t *th;
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    unsigned gen;          /* job generation */
    int pending;           /* workers still copying the current job */
    int quit;
    char *dst;
    const char *src;
    size_t bytes;
};

static void *worker(void *arg)
{
    struct inccl_copy_pool *p = (struct inccl_copy_pool *)arg;
    pthread_mutex_lock(&p->mu);
    int idx = p->pending++;   /* registration order gives each worker its slice index */
    pthread_cond_signal(&p->done);
    unsigned seen = p->gen;
    for (;;) {
        while (p->gen == seen && !p->quit) pthread_cond_wait(&p->go, &p->mu);
        if (p->quit) break;
        seen = p->gen;
        char *dst = p->dst;
        const char *src = p->src;
        const size_t bytes = p->bytes;
        pthread_mutex_unlock(&p->mu);
        /* slice idx of n+1 (the caller copies slice n); 4 KiB-aligned slices */
        const size_t parts = (size_t)p->n + 1;
        size_t per = (bytes + parts - 1) / parts;
        per = (per + 4095) & ~(size_t)4095;
        const size_t lo = per * (size_t)idx;
        if (lo < bytes) memcpy(dst + lo, src + lo, (bytes - lo) < per ? (bytes - lo) : per);
        pthread_mutex_lock(&p->mu);
        if (--p->pending == 0) pthread_cond_signal(&p->done);
    }
    pthread_mutex_unlock(&p->mu);
    return NULL;
}

struct inccl_copy_pool *inccl_copy_pool_create(int n)
{
    if (n < 1) return NULL;
    struct inccl_copy_pool *p = (struct inccl_copy_pool *)calloc(1, sizeof(*p));
    if (!p) return NULL;
    p->n = n;
    p->th = (pthread_t *)calloc((size_t)n, sizeof(pthread_t));
    pthread_mutex_init(&p->mu, NULL);
    pthread_cond_init(&p->go, NULL);
    pthread_cond_init(&p->done, NULL);
    int started = 0;
    for (int i = 0; p->th && i < n; ++i)
        if (pthread_create(&p->th[i], NULL, worker, p) == 0) started++;
    pthread_mutex_lock(&p->mu);
    while (p->pending < started) pthread_cond_wait(&p->done, &p->mu);
    p->pending = 0;
    p->n = started;
    pthread_mutex_unlock(&p->mu);
    if (started == 0) {
        inccl_copy_pool_destroy(p);
        return NULL;
    }
    return p;
}

void inccl_copy_pool_destroy(struct inccl_copy_pool *p)
{
    if (!p) return;
    pthread_mutex_lock(&p->mu);
    p->quit = 1;
    pthread_cond_broadcast(&p->go);
    pthread_mutex_unlock(&p->mu);
    for (int i = 0; p->th && i < p->n; ++i) pthread_join(p->th[i], NULL);
    pthread_cond_destroy(&p->go);
    pthread_cond_destroy(&p->done);
    pthread_mutex_destroy(&p->mu);
    free(p->th);
    free(p);
}

void inccl_copy(struct inccl_copy_pool *p, void *dst, const void *src, size_t bytes)
{
    if (!p || bytes < ((size_t)1 << 20)) {   /* small copies: not worth a wake-up */
        memcpy(dst, src, bytes);
        return;
    }
    pthread_mutex_lock(&p->mu);
    p->dst = (char *)dst;
    p->src = (const char *)src;
    p->bytes = bytes;
    p->pending = p->n;
    p->gen++;
    pthread_cond_broadcast(&p->go);
    pthread_mutex_unlock(&p->mu);
    /* the caller copies the last slice */
    const size_t parts = (size_t)p->n + 1;
    size_t per = (bytes + parts - 1) / parts;
    per = (per + 4095) & ~(size_t)4095;
    const size_t lo = per * (size_t)p->n;
    if (lo < bytes) memcpy((char *)dst + lo, (const char *)src + lo, bytes - lo);
    pthread_mutex_lock(&p->mu);
    while (p->pending > 0) pthread_cond_wait(&p->done, &p->mu);
    pthread_mutex_unlock(&p->mu);
}
