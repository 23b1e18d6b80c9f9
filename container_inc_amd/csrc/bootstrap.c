/* bootstrap.c -- TCP rendezvous of a group (replaces repository/src/api.c:34-144).
 *
 * Reference: rank 0 accepts world_size-1 connections on MASTER_PORT, each
 * rank sends {rank, ip} (api.c:43-76, :112-144), and rank 0 relays controller
 * data to the group.  Here rank 0 accepts the same connections and later
 * broadcasts the RCCL unique id of every communicator over them; there is no
 * controller, topology YAML or switch to configure. */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <fcntl.h>
#include <poll.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "inccl_internal.h"

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static double boot_timeout_s(void)
{
    const char *e = getenv("INCCL_BOOT_TIMEOUT");
    double t = e ? atof(e) : 0.0;
    return t > 0.0 ? t : 300.0;
}

static int send_all(int fd, const void *buf, size_t n)
{
    const char *p = (const char *)buf;
    while (n > 0) {
        ssize_t k = send(fd, p, n, MSG_NOSIGNAL);
        if (k < 0) {
            if (errno == EINTR) continue;
            return -1;
        }
        p += k;
        n -= (size_t)k;
    }
    return 0;
}

static int recv_all(int fd, void *buf, size_t n)
{
    char *p = (char *)buf;
    const double deadline = now_s() + boot_timeout_s();
    while (n > 0) {
        struct pollfd pf = {fd, POLLIN, 0};
        int ms = (int)((deadline - now_s()) * 1000.0);
        if (ms <= 0) return -1;
        int pr = poll(&pf, 1, ms);
        if (pr < 0 && errno == EINTR) continue;
        if (pr <= 0) return -1;
        ssize_t k = recv(fd, p, n, 0);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return -1;
        p += k;
        n -= (size_t)k;
    }
    return 0;
}

static void tune_fd(int fd)
{
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

int inccl_boot_master(struct inccl_group *g)
{
    const int peers = g->world_size - 1;
    g->peer_fds = (int *)calloc((size_t)g->world_size, sizeof(int));
    if (!g->peer_fds) return inccl_set_error(INCCL_ERR_NOMEM, "bootstrap: out of memory");
    for (int i = 0; i < g->world_size; ++i) g->peer_fds[i] = -1;
    if (peers == 0) return 0;

    int ls = socket(AF_INET, SOCK_STREAM, 0);
    if (ls < 0) return inccl_set_error(INCCL_ERR_SYS, "bootstrap: socket: %s", strerror(errno));
    int one = 1;
    setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    struct sockaddr_in addr;
    memset(&addr, 0, sizeof(addr));
    addr.sin_family = AF_INET;
    addr.sin_addr.s_addr = htonl(INADDR_ANY);
    addr.sin_port = htons((uint16_t)g->port);
    /* EADDRINUSE is retried until the boot deadline: a port from the
     * ephemeral range (what a caller's "free port" usually is) can be held for
     * a while as the local end of another connection on this host -- one GPU
     * test run lost a group that way -- or by a peer's own connect attempt
     * that landed on itself (dropped in inccl_boot_worker) */
    const double deadline = now_s() + boot_timeout_s();
    int brc;
    while ((brc = bind(ls, (struct sockaddr *)&addr, sizeof(addr))) < 0 && errno == EADDRINUSE && now_s() < deadline)
        usleep(20000);
    if (brc < 0 || listen(ls, peers + 4) < 0) {
        int rc = inccl_set_error(INCCL_ERR_SYS, "bootstrap: bind/listen port %d: %s", g->port, strerror(errno));
        close(ls);
        return rc;
    }
    int joined = 0;
    while (joined < peers) {
        struct pollfd pf = {ls, POLLIN, 0};
        int ms = (int)((deadline - now_s()) * 1000.0);
        if (ms <= 0) break;
        int pr = poll(&pf, 1, ms);
        if (pr < 0 && errno == EINTR) continue;
        if (pr <= 0) break;
        int fd = accept(ls, NULL, NULL);
        if (fd < 0) continue;
        tune_fd(fd);
        int32_t hello[2];
        /* {rank, world_size}: the reference sends {rank, ip} (api.c:130-134) */
        if (recv_all(fd, hello, sizeof(hello)) != 0 || hello[0] <= 0 || hello[0] >= g->world_size ||
            hello[1] != g->world_size || g->peer_fds[hello[0]] != -1) {
            close(fd);
            continue;
        }
        g->peer_fds[hello[0]] = fd;
        joined++;
    }
    close(ls);
    if (joined < peers) return inccl_set_error(INCCL_ERR_SYS, "bootstrap: only %d of %d ranks joined", joined, peers);
    /* release the workers only once everyone is in */
    const char go = 'G';
    for (int r = 1; r < g->world_size; ++r)
        if (send_all(g->peer_fds[r], &go, 1) != 0)
            return inccl_set_error(INCCL_ERR_SYS, "bootstrap: send to rank %d failed", r);
    return 0;
}

int inccl_boot_worker(struct inccl_group *g)
{
    struct addrinfo hints, *res = NULL;
    memset(&hints, 0, sizeof(hints));
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    char port[16];
    snprintf(port, sizeof(port), "%d", g->port);
    if (getaddrinfo(g->master_ip, port, &hints, &res) != 0 || !res)
        return inccl_set_error(INCCL_ERR_SYS, "bootstrap: cannot resolve %s", g->master_ip);
    const double deadline = now_s() + boot_timeout_s();
    int fd = -1;
    while (now_s() < deadline) {
        fd = socket(AF_INET, SOCK_STREAM, 0);
        if (fd < 0) break;
        if (connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
            /* a connect to a port in the ephemeral range can land on itself
             * (local port == rank 0's port, before rank 0 has bound it): that
             * is no rank 0, and it holds rank 0's port -- drop it and retry */
            struct sockaddr_in la, pa;
            socklen_t ll = sizeof(la), pl = sizeof(pa);
            if (getsockname(fd, (struct sockaddr *)&la, &ll) != 0 || getpeername(fd, (struct sockaddr *)&pa, &pl) != 0 ||
                la.sin_port != pa.sin_port || la.sin_addr.s_addr != pa.sin_addr.s_addr)
                break;
        }
        close(fd);
        fd = -1;
        usleep(20000);   /* rank 0 may not be listening yet */
    }
    freeaddrinfo(res);
    if (fd < 0) return inccl_set_error(INCCL_ERR_SYS, "bootstrap: connect %s:%d failed", g->master_ip, g->port);
    tune_fd(fd);
    int32_t hello[2] = {g->rank, g->world_size};
    char go = 0;
    if (send_all(fd, hello, sizeof(hello)) != 0 || recv_all(fd, &go, 1) != 0 || go != 'G') {
        close(fd);
        return inccl_set_error(INCCL_ERR_SYS, "bootstrap: handshake with rank 0 failed");
    }
    g->master_fd = fd;
    return 0;
}

int inccl_boot_bcast(struct inccl_group *g, void *buf, size_t bytes)
{
    if (g->world_size == 1) return 0;
    if (g->rank == 0) {
        for (int r = 1; r < g->world_size; ++r)
            if (send_all(g->peer_fds[r], buf, bytes) != 0)
                return inccl_set_error(INCCL_ERR_SYS, "bootstrap: bcast to rank %d failed", r);
        return 0;
    }
    if (recv_all(g->master_fd, buf, bytes) != 0) return inccl_set_error(INCCL_ERR_SYS, "bootstrap: bcast recv failed");
    return 0;
}

int inccl_boot_allgather(struct inccl_group *g, const void *mine, void *all, size_t bytes)
{
    char *out = (char *)all;
    memcpy(out + (size_t)g->rank * bytes, mine, bytes);
    if (g->world_size == 1) return 0;
    if (g->rank == 0) {
        for (int r = 1; r < g->world_size; ++r)
            if (recv_all(g->peer_fds[r], out + (size_t)r * bytes, bytes) != 0)
                return inccl_set_error(INCCL_ERR_SYS, "allgather: recv from rank %d failed", r);
        for (int r = 1; r < g->world_size; ++r)
            if (send_all(g->peer_fds[r], out, bytes * (size_t)g->world_size) != 0)
                return inccl_set_error(INCCL_ERR_SYS, "allgather: send to rank %d failed", r);
        return 0;
    }
    if (send_all(g->master_fd, mine, bytes) != 0 ||
        recv_all(g->master_fd, out, bytes * (size_t)g->world_size) != 0)
        return inccl_set_error(INCCL_ERR_SYS, "allgather: exchange with rank 0 failed");
    return 0;
}

int inccl_boot_barrier(struct inccl_group *g)
{
    if (g->world_size == 1) return 0;
    char b = 'B';
    if (g->rank == 0) {
        for (int r = 1; r < g->world_size; ++r)
            if (recv_all(g->peer_fds[r], &b, 1) != 0) return inccl_set_error(INCCL_ERR_SYS, "barrier: recv failed");
        for (int r = 1; r < g->world_size; ++r)
            if (send_all(g->peer_fds[r], &b, 1) != 0) return inccl_set_error(INCCL_ERR_SYS, "barrier: send failed");
        return 0;
    }
    if (send_all(g->master_fd, &b, 1) != 0 || recv_all(g->master_fd, &b, 1) != 0)
        return inccl_set_error(INCCL_ERR_SYS, "barrier: exchange with rank 0 failed");
    return 0;
}

/* ------------------------------------------------------------------ */
/* same-node fast barrier: a sense-reversing counter in POSIX shared memory */
/* ------------------------------------------------------------------ */
struct inccl_shm_bar {
    _Atomic uint32_t count;
    _Atomic uint32_t generation;
    uint32_t world;
    _Atomic uint32_t words[2][64];   /* one word per rank for small host reductions, two banks */
};

int inccl_boot_shm_init(struct inccl_group *g)
{
    if (g->world_size == 1 || g->shm_bar) return 0;
    char name[64];
    memset(name, 0, sizeof(name));
    if (g->rank == 0) {
        struct timespec ts;
        clock_gettime(CLOCK_REALTIME, &ts);
        snprintf(name, sizeof(name), "/inccl-%d-%ld-%d", (int)getpid(), (long)ts.tv_nsec, g->port);
        int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd >= 0) {
            if (ftruncate(fd, sizeof(struct inccl_shm_bar)) != 0) name[0] = 0;
            close(fd);
        } else {
            name[0] = 0;
        }
    }
    int rc = inccl_boot_bcast(g, name, sizeof(name));
    if (rc) return rc;
    int32_t ok = 0;
    void *p = MAP_FAILED;
    if (name[0]) {
        int fd = shm_open(name, O_RDWR, 0600);
        if (fd >= 0) {
            p = mmap(NULL, sizeof(struct inccl_shm_bar), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            close(fd);
            ok = p != MAP_FAILED;
        }
    }
    int32_t all[64];
    if (g->world_size > 64) ok = 0;
    rc = g->world_size <= 64 ? inccl_boot_allgather(g, &ok, all, sizeof(ok)) : 0;
    int every = rc == 0 && g->world_size <= 64;
    for (int j = 0; every && j < g->world_size; ++j) every = every && all[j];
    /* the name is no longer needed once every rank has mapped it */
    int rc2 = inccl_boot_barrier(g);
    if (g->rank == 0 && name[0]) shm_unlink(name);
    if (!every) {   /* not all on one node (or no /dev/shm): keep the TCP barrier */
        if (p != MAP_FAILED) munmap(p, sizeof(struct inccl_shm_bar));
        return rc ? rc : rc2;
    }
    struct inccl_shm_bar *b = (struct inccl_shm_bar *)p;
    if (g->rank == 0) b->world = (uint32_t)g->world_size;
    g->shm_bar = b;
    return inccl_boot_barrier(g);
}

int inccl_group_barrier(struct inccl_group *g)
{
    struct inccl_shm_bar *b = g->shm_bar;
    if (!b) return inccl_boot_barrier(g);
    const uint32_t gen = atomic_load(&b->generation);
    if (atomic_fetch_add(&b->count, 1) + 1 == (uint32_t)g->world_size) {
        atomic_store(&b->count, 0);
        atomic_store(&b->generation, gen + 1);
        return 0;
    }
    const double deadline = now_s() + boot_timeout_s();
    unsigned spins = 0;
    while (atomic_load(&b->generation) == gen) {
        if ((++spins & 1023) == 0) {
            if (now_s() > deadline) return inccl_set_error(INCCL_ERR_SYS, "shm barrier timed out");
            sched_yield();
        }
    }
    return 0;
}

/* max of one word over the group: through the shared-memory segment when the
 * group has one (one barrier, a few microseconds), else the TCP allgather.
 * Calls alternate between two banks of words, so no second barrier is needed:
 * a rank writes bank b again only in the call after next, which it reaches
 * after the next call's barrier -- i.e. after every rank has finished reading
 * bank b in this call.  The bank sequence is per group: calls on one group
 * must not run concurrently (communicators that share a group from different
 * threads serialise their auto-scale calls themselves). */
int inccl_group_allreduce_max_u32(struct inccl_group *g, uint32_t *v)
{
    if (g->world_size == 1) return 0;
    struct inccl_shm_bar *b = g->shm_bar;
    if (b) {
        _Atomic uint32_t *words = b->words[g->max_seq++ & 1u];
        atomic_store(&words[g->rank], *v);
        int rc = inccl_group_barrier(g);   /* every word of this bank written */
        if (rc) return rc;
        uint32_t m = 0;
        for (int j = 0; j < g->world_size; ++j) {
            const uint32_t w = atomic_load(&words[j]);
            m = w > m ? w : m;
        }
        *v = m;
        return 0;
    }
    uint32_t all[64];
    if (g->world_size > 64) return inccl_set_error(INCCL_ERR_ARG, "max-allreduce: world too large");
    int rc = inccl_boot_allgather(g, v, all, sizeof(*v));
    if (rc) return rc;
    uint32_t m = 0;
    for (int j = 0; j < g->world_size; ++j) m = all[j] > m ? all[j] : m;
    *v = m;
    return 0;
}

void inccl_boot_close(struct inccl_group *g)
{
    if (g->shm_bar) {
        munmap(g->shm_bar, sizeof(struct inccl_shm_bar));
        g->shm_bar = NULL;
    }
    if (g->peer_fds) {
        for (int r = 0; r < g->world_size; ++r)
            if (g->peer_fds[r] >= 0) close(g->peer_fds[r]);
        free(g->peer_fds);
        g->peer_fds = NULL;
    }
    if (g->master_fd >= 0) {
        close(g->master_fd);
        g->master_fd = -1;
    }
}
