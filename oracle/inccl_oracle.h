/*
 * inccl_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the host-side allreduce hot path of In-NetLab/container_inc
 * (INCCL), written from scratch in plain C11.  It is the parity checker for the
 * MI355X engine in container_inc_amd/: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product library never links it.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the reference checkout's repository/ directory).
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - integer sum + wire codec + windowed driver: pinned by the reference's own
 *     known-answer test src/host.c:20-25,51-55 (in[i] = i*(rank+1), two ranks,
 *     dst[i] == 3*i) -> tests/golden/host_known_answer.*
 *   - ICRC: pinned by the canned RoCEv2 ACK frame in src/test.c:4-22 whose
 *     captured ICRC bytes are kept at src/test.c:21 (e8 b0 bb 30).
 *   - fp32 quantise / dequantise: NOT present in the reference (no float in its
 *     data path).  Pinned by the spec below plus known-answer vectors
 *     (powers of two, ties-to-even, saturation, NaN/Inf, denormals).
 * The reference itself is unbuildable in this image (needs infiniband/verbs.h
 * and pcap.h, both absent), so there is no oracle/_ref build.
 */
#ifndef INCCL_ORACLE_H
#define INCCL_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Size constants of the reference (repository/include/api.h:38-40,
 * repository/include/util.h:85, repository/src/non_termination_switch.c:21-24). */
#define ORC_PAYLOAD_LEN      1024   /* bytes per RoCE packet payload  (util.h:85)        */
#define ORC_LANES            256    /* int32 lanes per packet          (nts.c:55)         */
#define ORC_MESSAGE_SIZE     4096   /* bytes per RDMA WRITE message    (api.h:39)         */
#define ORC_PAYLOAD_COUNT    1024   /* int32 per message               (api.h:40)         */
#define ORC_WINDOW_SIZE      8192   /* host window in bytes            (api.h:38)         */
#define ORC_PKTS_PER_MSG     4      /* MESSAGE_SIZE / PAYLOAD_LEN                         */
#define ORC_SW_WINDOW        8      /* switch window in packets        (nts.c:21)         */
#define ORC_SW_SLOTS         16     /* N = 2*WINDOW_SIZE slots         (nts.c:22)         */
#define ORC_MAX_FAN_IN       31     /* bitmap bit FAN_IN marks "result known" (nts.c:29-30,366) */
#define ORC_ETH_HDR          14
#define ORC_IP_HDR           20
#define ORC_UDP_HDR          8
#define ORC_BTH_HDR          12
#define ORC_RETH_HDR         16
#define ORC_AETH_HDR         4
#define ORC_ICRC_LEN         4

/* Quantiser scale exponents accepted by the engine (spec). */
#define ORC_SCALE_MIN        (-64)
#define ORC_SCALE_MAX        64

/* ---------------- byte order (wire codec) ---------------- */
/* api.c:300-302 post_send: send_payload[i] = htonl(src[i]) */
void orc_encode_be32(const int32_t *src, uint32_t *wire, size_t n);
/* api.c:428-430 / :377-379: dst[j] = ntohl(receive_payload[j]) */
void orc_decode_be32(const uint32_t *wire, int32_t *dst, size_t n);

/* ---------------- fp32 <-> fixed point (new front/back stages) ---------------- */
/* q = sat_i32(round_half_even(x * 2^k)); NaN -> 0; +Inf -> INT32_MAX; -Inf -> INT32_MIN. */
int32_t orc_quantise_one(float x, int k);
void    orc_quantise_f32(const float *x, int32_t *q, size_t n, int k);
/* f = (float)q * 2^-k  ((float)q rounds to nearest even; the scaling is exact). */
float   orc_dequantise_one(int32_t q, int k);
void    orc_dequantise_q32(const int32_t *q, float *f, size_t n, int k);

/* ---------------- reduction ---------------- */
/* nts.c:361-363: aggregator[slot][i] += ntohl(data[i]) -- two's-complement wrap
 * (done in uint32 here: the reference's signed int accumulator is UB on overflow). */
void orc_sum_q32(const int32_t *const *srcs, int R, int32_t *dst, size_t n);
/* Fused spec of the engine's single-GPU path: dst = dequant(sum_r quant(src_r)). */
void orc_reduce_f32(const float *const *srcs, int R, float *dst, size_t n, int k);
/* Local quantise+sum to int32 (first stage of the multi-GPU path). */
void orc_quant_sum(const float *const *srcs, int R, int32_t *dst, size_t n, int k);
/* max |x| over R buckets; NaN lanes ignored. */
float orc_absmax_f32(const float *const *srcs, int R, size_t n);
/* bfloat16 buckets (uint16_t bit patterns): quantise the exactly widened fp32
 * value; dequantise to fp32 as above, then round to nearest even bf16 */
float orc_bf16_to_f32(uint16_t h);
uint16_t orc_f32_to_bf16(float f);
void orc_reduce_bf16(const uint16_t *const *srcs, int R, uint16_t *dst, size_t n, int k);
void orc_quant_sum_bf16(const uint16_t *const *srcs, int R, int32_t *dst, size_t n, int k);
void orc_sum_dequant_bf16(const int32_t *const *srcs, int R, uint16_t *dst, size_t n, int k);
float orc_absmax_bf16(const uint16_t *const *srcs, int R, size_t n);
/* IEEE binary16 buckets: widening exact; narrowing to nearest even, +-Inf past
 * 65504, subnormals below 2^-14 (pinned against numpy's float16 in
 * tests/test_oracle_f16.py) */
float orc_f16_to_f32(uint16_t h);
uint16_t orc_f32_to_f16(float f);
void orc_f16_to_f32_n(const uint16_t *h, float *f, size_t n);
void orc_f32_to_f16_n(const float *f, uint16_t *h, size_t n);
void orc_reduce_f16(const uint16_t *const *srcs, int R, uint16_t *dst, size_t n, int k);
void orc_quant_sum_f16(const uint16_t *const *srcs, int R, int32_t *dst, size_t n, int k);
void orc_sum_dequant_f16(const int32_t *const *srcs, int R, uint16_t *dst, size_t n, int k);
float orc_absmax_f16(const uint16_t *const *srcs, int R, size_t n);
/* Largest k with R*absmax*2^k <= 2^30 (one bit of headroom), clamped to
 * [ORC_SCALE_MIN, ORC_SCALE_MAX]; absmax == 0 -> ORC_SCALE_MAX; Inf -> ORC_SCALE_MIN. */
int   orc_choose_scale(float absmax, int R);
/* Position-weighted linear checksum: sum_i (2i+1) * (uint32)q[i]  mod 2^32. */
uint32_t orc_checksum_q32(const int32_t *q, size_t n, uint64_t index_base);

/* ---------------- switch aggregation pipeline (root switch) ---------------- */
/* State of nts.c:55-60 restated for one root switch with fan_in children.  The
 * reference's ring is N = 16 slots with window 8 (nts.c:21-22); the ring here
 * may be any power of two up to ORC_SW_MAX_SLOTS, with window = slots / 2. */
#define ORC_SW_MAX_SLOTS 1024
typedef struct orc_switch {
    int      fan_in;
    uint32_t slots, window;
    int32_t  aggregator[ORC_SW_MAX_SLOTS][ORC_LANES];                      /* nts.c:55 */
    uint32_t arrival_state[ORC_SW_MAX_SLOTS];                              /* nts.c:59 bitmap */
    int      degree[ORC_SW_MAX_SLOTS];                                     /* nts.c:60 */
    uint8_t  reth_keeper[ORC_SW_MAX_SLOTS][ORC_MAX_FAN_IN][ORC_RETH_HDR];  /* nts.c:57 */
    uint64_t adds;                                                         /* packets actually summed */
    uint64_t replays;                                                      /* retransmits answered from the slot */
    int      root;                                                         /* nts.c:68: 1 root, 0 non-root */
    int      flags;                                                        /* non-root: ORC_SW_WIRE_ORDER | ORC_SW_RECYCLE */
} orc_switch;

/* A non-root switch (nts.c:376-400, :408-423, :457-499): children on ports
 * 0..fan_in-1, the parent on port fan_in.  flags 0 is the reference exactly:
 * the parent's result is copied into the aggregator as wire bytes (nts.c:413,
 * :489) and re-encoded with htonl on the way down (util.c:403-405), so every
 * downstream word has its bytes reversed, and no slot is ever recycled
 * (clear_state_data runs only at the root, :367, :449).  ORC_SW_WIRE_ORDER
 * stores the result ntohl'd (children get the parent's words as sent);
 * ORC_SW_RECYCLE clears slot psn + window when the parent's result for psn is
 * taken, as the root does at completion. */
#define ORC_SW_WIRE_ORDER 1
#define ORC_SW_RECYCLE    2
int orc_switch_init_nonroot(orc_switch *sw, int fan_in, uint32_t slots, int flags);

size_t orc_switch_bytes(void);                      /* sizeof(orc_switch), for callers that allocate it */
const int32_t *orc_switch_slot(const orc_switch *sw, uint32_t psn);   /* aggregator[Idx(psn)] (nts.c:55) */
void orc_switch_init(orc_switch *sw, int fan_in);   /* the reference's 16-slot ring */
/* 0, or -1 for fan_in outside 1..31 or slots not a power of two in 2..ORC_SW_MAX_SLOTS */
int orc_switch_init_ring(orc_switch *sw, int fan_in, uint32_t slots);
/* One UP data packet from child `port` with PSN `psn` and a big-endian payload of
 * ORC_LANES words (nts.c:347-374 / :427-455, root branch).
 * Returns:  ORC_SW_ABSORBED  first arrival, aggregate not complete yet
 *           ORC_SW_BROADCAST first arrival completed the slot; egress_be holds the
 *                            big-endian aggregate to send to EVERY child (nts.c:369-371)
 *           ORC_SW_REPLAY    retransmit of a completed slot; egress_be holds the aggregate
 *                            to send back to `port` only (nts.c:353-356)
 *           ORC_SW_DROPPED   retransmit of an incomplete slot (nts.c:353 with no result) */
enum { ORC_SW_ABSORBED = 0, ORC_SW_BROADCAST = 1, ORC_SW_REPLAY = 2, ORC_SW_DROPPED = 3,
       ORC_SW_ACK = 4, ORC_SW_IGNORED = 5, ORC_SW_INVALID = 6,
       ORC_SW_FORWARD = 7,   /* non-root: the aggregate to the parent (nts.c:394-397, :476-479, resend :381-384, :462-465) */
       ORC_SW_DOWN = 8 };    /* non-root: the parent's result taken and broadcast (nts.c:412-419, :488-495) */
int orc_switch_ingress(orc_switch *sw, int port, uint32_t psn,
                       const uint32_t *payload_be, uint32_t *egress_be);

/* A child connection: the util.h connection_t fields that send_roce_data /
 * _with_reth / send_roce_ack hand to build_eth_packet (nts.c:252-298) -- src =
 * my_*, dst = peer_*, BTH QPN = peer_qp.  Same 28-byte layout as the engine's
 * struct inccl_frame_template. */
typedef struct orc_conn {
    uint8_t  my_mac[6], peer_mac[6];
    uint32_t my_ip, peer_ip;        /* as stored in the IP header */
    uint16_t my_port, peer_port;    /* host order */
    uint32_t peer_qp;
} orc_conn;

/* The whole of pipeline() (nts.c:303-501, root branch) for one frame from child
 * `port`, frames in -> frames out: parse (opcode, PSN :311-344), UP_DATA and
 * UP_WRITE_FIRST_ONLY aggregation with the RETH keeper (:347-374, :427-455),
 * UP_ACK reflection (:403-406).  Row c of `out` (stride out_stride) receives
 * the frame sent to child c and out_len[c] its length (0: none sent):
 *   ORC_SW_BROADCAST  every child: the aggregate with the completing packet's
 *                     opcode, with child c's kept RETH if that opcode is
 *                     WRITE_FIRST / WRITE_ONLY (send_roce_data_with_reth)
 *   ORC_SW_REPLAY     child `port`: the same, with the retransmit's opcode
 *   ORC_SW_ACK        child `port`: the 62-B ACK (opcode 0x11, AETH) for the PSN
 *   ORC_SW_ABSORBED / DROPPED  nothing
 *   ORC_SW_IGNORED    opcode the pipeline has no case for: nothing, no state
 *   ORC_SW_INVALID    port >= fan_in (the root has no parent) or a payload
 *                     length other than 1024 B (the reference asserts, :350)
 * row_len bounds the frame's bytes (a payload past it is INVALID).
 * A non-root switch (orc_switch_init_nonroot) has fan_in + 1 rows and conns,
 * row fan_in being the parent's:
 *   ORC_SW_FORWARD    the parent: the aggregate with this packet's opcode (a
 *                     WRITE_FIRST / WRITE_ONLY one with a zeroed RETH, :464, :478)
 *   ORC_SW_DOWN       a packet from the parent whose result was taken: every
 *                     child, the aggregator's words with the parent packet's
 *                     opcode and child c's kept RETH for WRITE_FIRST / ONLY
 *   ORC_SW_REPLAY     child `port`: the aggregator after the parent's result
 *   ORC_SW_DROPPED    also a parent packet that is not taken (:420-422)
 *   ORC_SW_IGNORED    also an ACK from the parent (DOWN_ACK, :424-426) */
int orc_switch_pipeline(orc_switch *sw, const orc_conn *conns, int port, const uint8_t *frame, size_t row_len,
                        uint8_t *out, size_t out_stride, int *out_len);

/* ---------------- RoCEv2 framing + ICRC ---------------- */
/* util.c:141-195: reflected CRC-32 (poly 0xEDB88320), init ~0, final ~. */
uint32_t orc_crc32(const void *data, size_t len);
/* util.c:250-286: ICRC over 8 x 0xFF || IP..payload with tos/ttl/ipcsum/udpcsum/qpn-low-byte masked. */
uint32_t orc_icrc(const uint8_t *frame);
/* util.c:106-127 */
uint16_t orc_ipv4_checksum(const uint8_t *ip_hdr);
/* util.c:331-442 build_eth_packet for PACKET_TYPE_DATA (reth == NULL, with_reth == 0)
 * and PACKET_TYPE_RETH (with_reth != 0; reth may be NULL -> zeroed).  `payload_host`
 * holds host-order words; they are written big-endian.  Returns the frame length. */
typedef struct orc_frame_hdr {
    uint8_t  src_mac[6], dst_mac[6];
    uint32_t src_ip, dst_ip;      /* network order, as util.c:362-363 stores them */
    uint16_t src_port, dst_port;  /* host order */
    uint32_t qp, psn;
    uint8_t  opcode;
} orc_frame_hdr;
size_t orc_build_data_frame(uint8_t *frame, const orc_frame_hdr *h, const int32_t *payload_host,
                            int n_words, int with_reth, const uint8_t *reth16);
/* util.c:331-442 for PACKET_TYPE_ACK (send_roce_ack, nts.c:284-298): opcode 0x11,
 * BTH PSN without the ack-request bit, AETH syn_msn = htonl(msn | 0x1f000000)
 * (util.c:342-343, :379-380, :387-388, :391-395); h->opcode is not used.  62 B. */
size_t orc_build_ack_frame(uint8_t *frame, const orc_frame_hdr *h, uint32_t msn);

/* ---------------- windowed host driver + switch, single-process loopback ---------------- */
/* Drives R ranks through api.c:403-452 (inccl_allreduce_write: 2-message window,
 * encode, completion-ordered decode) against one root switch (nts.c:303-501).
 * Each RDMA WRITE of 4096 B is four 1 KiB packets with consecutive PSNs.
 * `dup_every` > 0 re-injects every dup_every-th packet as a retransmit (idempotence).
 * Elements [message_num*1024, len) of dst are left untouched, as in the reference.
 * Returns the number of messages decoded per rank. */
int orc_allreduce_write_loopback(int R, const int32_t *const *src, uint32_t len,
                                 int32_t *const *dst, int dup_every,
                                 uint64_t *frames_out, int with_icrc);

#ifdef __cplusplus
}
#endif
#endif /* INCCL_ORACLE_H */
