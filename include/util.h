/*
 * util.h -- drop-in stand-in for the reference's repository/include/util.h,
 * so that an application written against the reference (host.c:2 includes
 * it) builds against this include directory unchanged.
 *
 * The reference header declares the switch's RoCEv2 frame structs and
 * builders (util.h:10-139) over <pcap.h>.  Those belong to the software
 * switch, which this library replaces; its GPU dataplane has its own frame
 * interface in inccl_amd.h (inccl_switch_*, struct inccl_frame_template).
 * What remains here are the wire constants a host program may name.
 */
#ifndef INCCL_AMD_UTIL_H
#define INCCL_AMD_UTIL_H

#include <stdint.h>
#include <arpa/inet.h>
#include <sys/time.h>

/* util.h:79-86 */
#define PACKET_TYPE_DATA 0
#define PACKET_TYPE_ACK 1
#define PACKET_TYPE_NAK 2
#define PACKET_TYPE_DATA_SINGLE 3
#define PACKET_TYPE_RETH 4
#ifndef PAYLOAD_LEN
#define PAYLOAD_LEN 1024 /* bytes of int32 payload per RoCE packet (256 lanes) */
#endif
#define ELEMENT_SIZE sizeof(int32_t)

#endif /* INCCL_AMD_UTIL_H */
