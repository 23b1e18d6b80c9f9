/*
 * api.h -- drop-in replacement for the INCCL host API of In-NetLab/container_inc
 *          (reference: repository/include/api.h), served by libinccl_amd.so.
 *
 * The six entry points keep the reference's exact C signatures so an
 * application such as repository/src/host.c links against this library
 * unchanged.  What differs is below the surface: the reduction runs on an
 * MI355X (HIP kernels + RCCL over xGMI) instead of a software RoCE switch.
 *
 * The structs are opaque here.  The reference exposes libibverbs types in them
 * (api.h:42-91, which need <infiniband/verbs.h>); its only caller, host.c:39-47,
 * uses them through pointers alone.
 *
 * Error behaviour (kept from the reference, api.c):
 *   - inccl_group_create returns NULL on socket / setup errors (api.c:82-98).
 *   - collectives are void; diagnostics go to stderr.  The additive API in
 *     inccl_amd.h returns error codes for every call instead.
 */
#ifndef INCCL_AMD_API_H
#define INCCL_AMD_API_H

/* The system headers the reference api.h:1-18 hands to its callers (host.c
 * uses printf, atoi, clock_t, clock() and CLOCKS_PER_SEC through them, never
 * including them itself), minus <infiniband/verbs.h>, plus <time.h>, which
 * the reference gets transitively from verbs.h. */
#include <netinet/in.h>
#include <arpa/inet.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <stdint.h>
#include <inttypes.h>
#include <endian.h>
#include <byteswap.h>
#include <stdbool.h>
#include <getopt.h>
#include <sys/time.h>
#include <sys/types.h>
#include <sys/socket.h>
#include <netdb.h>
#include <time.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Reference constants (api.h:32-40, util.h:85). */
#define TCP_PORT_1 31324
#define TCP_PORT_2 31325
#define INCCL_HEADER_LEN 8
#define GID_IDX 1
#ifndef PAYLOAD_LEN
#define PAYLOAD_LEN 1024
#endif
#define WINDOW_SIZE 8192
#define MESSAGE_SIZE (4 * (PAYLOAD_LEN))
#define PAYLOAD_COUNT ((MESSAGE_SIZE) / (sizeof(int)))
/* parameter.h:1 -- rank 0's rendezvous port (override with INCCL_MASTER_PORT). */
#define MASTER_PORT 52223

struct inccl_group;          /* reference api.h:42-70  */
struct inccl_communicator;   /* reference api.h:79-91  */

/* Replaces api.c:5-149.  Rank 0 listens on master_ip:MASTER_PORT, the other
 * ranks connect and register; rank 0 then distributes the RCCL unique id for
 * each communicator.  master_ip "local" selects the in-process transport
 * (ranks are threads of one process sharing one GPU, see inccl_amd.h). */
struct inccl_group *inccl_group_create(int world_size, int rank, const char *master_ip);
/* Replaces api.c:151-154 (which freed nothing and returned 1).  Closes the
 * control sockets and frees the group; returns 1 like the reference. */
int inccl_group_destroy(struct inccl_group *group);

/* Replaces api.c:156-287.  `size` is in bytes (host.c:41); staging buffers of
 * 2*size bytes are allocated pinned (the reference's registered MRs,
 * api.c:164-176) plus device buffers of the same size. */
struct inccl_communicator *inccl_communicator_create(struct inccl_group *group, uint32_t size);
/* Declared but never defined by the reference (api.h:97, api.c:290).  Frees
 * device and pinned buffers and the RCCL communicator; returns 0. */
int inccl_communicator_destroy(struct inccl_communicator *comm);

/* Replace api.c:330-401 and api.c:403-452.  len = number of int32 elements.
 * dst[i] = sum over ranks of src[i], two's-complement wrap (nts.c:361-363).
 * As in the reference only whole 1024-element messages are reduced
 * (message_num = len / PAYLOAD_COUNT, api.c:406); dst[message_num*1024 ..
 * len) is left untouched.  Blocking; one call at a time per communicator. */
void inccl_allreduce_sendrecv(struct inccl_communicator *comm, int32_t *src_data, uint32_t len, int32_t *dst_data);
void inccl_allreduce_write(struct inccl_communicator *comm, int32_t *src_data, uint32_t len, int32_t *dst_data);

#ifdef __cplusplus
}
#endif
#endif /* INCCL_AMD_API_H */
