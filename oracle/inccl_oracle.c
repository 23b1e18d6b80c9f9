/*
 * inccl_oracle.c -- TEST INFRASTRUCTURE ONLY (see inccl_oracle.h).
 *
 * Plain-C restatement of the INCCL hot path.  Scalar on purpose: it mirrors the
 * reference's per-element loops so it can also serve as the single-core CPU
 * baseline ("port") in bench.py.  Compiled with the reference's flags
 * (-O3 -march=native -funroll-loops, repository/CMakeLists.txt:30).
 */
#include "inccl_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* byte order                                                           */
/* ------------------------------------------------------------------ */
static inline uint32_t bswap32(uint32_t v)
{
    return (v >> 24) | ((v >> 8) & 0x0000FF00u) | ((v << 8) & 0x00FF0000u) | (v << 24);
}

/* htonl on a little-endian host (x86-64 and the MI355X hosts are LE). */
static inline uint32_t to_be(uint32_t v) { return bswap32(v); }

void orc_encode_be32(const int32_t *src, uint32_t *wire, size_t n)
{
    /* api.c:300-302 */
    for (size_t i = 0; i < n; ++i) wire[i] = to_be((uint32_t)src[i]);
}

void orc_decode_be32(const uint32_t *wire, int32_t *dst, size_t n)
{
    /* api.c:428-430 */
    for (size_t i = 0; i < n; ++i) dst[i] = (int32_t)to_be(wire[i]);
}

/* ------------------------------------------------------------------ */
/* quantise / dequantise (engine spec; no reference counterpart)       */
/* ------------------------------------------------------------------ */
static inline float pow2f(int k)
{
    /* exact 2^k for k in [-126, 127] built from the exponent field */
    union { uint32_t u; float f; } c;
    c.u = (uint32_t)(k + 127) << 23;
    return c.f;
}

int32_t orc_quantise_one(float x, int k)
{
    if (x != x) return 0;                       /* NaN -> 0 */
    /* For |k| <= 64 the product is exact whenever it is a normal number; a
     * subnormal product has magnitude < 2^-126 and rounds to 0 below. */
    float y = x * pow2f(k);
    if (y >= 2147483648.0f) return INT32_MAX;   /* saturate (also +Inf) */
    if (y <= -2147483648.0f) return INT32_MIN;  /* saturate (also -Inf) */
    return (int32_t)nearbyintf(y);              /* round half to even */
}

void orc_quantise_f32(const float *x, int32_t *q, size_t n, int k)
{
    for (size_t i = 0; i < n; ++i) q[i] = orc_quantise_one(x[i], k);
}

float orc_dequantise_one(int32_t q, int k)
{
    return (float)q * pow2f(-k);
}

void orc_dequantise_q32(const int32_t *q, float *f, size_t n, int k)
{
    const float s = pow2f(-k);
    for (size_t i = 0; i < n; ++i) f[i] = (float)q[i] * s;
}

/* ------------------------------------------------------------------ */
/* reduction                                                            */
/* ------------------------------------------------------------------ */
void orc_sum_q32(const int32_t *const *srcs, int R, int32_t *dst, size_t n)
{
    /* nts.c:361-363, accumulated in uint32 (exact mod 2^32 wrap) */
    for (size_t i = 0; i < n; ++i) {
        uint32_t acc = 0;
        for (int r = 0; r < R; ++r) acc += (uint32_t)srcs[r][i];
        dst[i] = (int32_t)acc;
    }
}

void orc_quant_sum(const float *const *srcs, int R, int32_t *dst, size_t n, int k)
{
    for (size_t i = 0; i < n; ++i) {
        uint32_t acc = 0;
        for (int r = 0; r < R; ++r) acc += (uint32_t)orc_quantise_one(srcs[r][i], k);
        dst[i] = (int32_t)acc;
    }
}

void orc_reduce_f32(const float *const *srcs, int R, float *dst, size_t n, int k)
{
    const float s = pow2f(-k);
    for (size_t i = 0; i < n; ++i) {
        uint32_t acc = 0;
        for (int r = 0; r < R; ++r) acc += (uint32_t)orc_quantise_one(srcs[r][i], k);
        dst[i] = (float)(int32_t)acc * s;
    }
}

float orc_absmax_f32(const float *const *srcs, int R, size_t n)
{
    float m = 0.0f;
    for (int r = 0; r < R; ++r)
        for (size_t i = 0; i < n; ++i) {
            float a = fabsf(srcs[r][i]);
            if (a > m) m = a;   /* NaN compares false: ignored */
        }
    return m;
}

/* bfloat16: the top half of an fp32 word.  Widening is exact; narrowing rounds
 * to nearest even (NaN kept quiet; the dequantised sums are always finite). */
float orc_bf16_to_f32(uint16_t h)
{
    union { uint32_t u; float f; } c;
    c.u = (uint32_t)h << 16;
    return c.f;
}

uint16_t orc_f32_to_bf16(float f)
{
    union { uint32_t u; float f; } c;
    c.f = f;
    if (f != f) return (uint16_t)((c.u >> 16) | 0x40u);
    const uint32_t lsb = (c.u >> 16) & 1u;
    return (uint16_t)((c.u + 0x7fffu + lsb) >> 16);
}

void orc_reduce_bf16(const uint16_t *const *srcs, int R, uint16_t *dst, size_t n, int k)
{
    const float s = pow2f(-k);
    for (size_t i = 0; i < n; ++i) {
        uint32_t acc = 0;
        for (int r = 0; r < R; ++r) acc += (uint32_t)orc_quantise_one(orc_bf16_to_f32(srcs[r][i]), k);
        dst[i] = orc_f32_to_bf16((float)(int32_t)acc * s);
    }
}

void orc_quant_sum_bf16(const uint16_t *const *srcs, int R, int32_t *dst, size_t n, int k)
{
    for (size_t i = 0; i < n; ++i) {
        uint32_t acc = 0;
        for (int r = 0; r < R; ++r) acc += (uint32_t)orc_quantise_one(orc_bf16_to_f32(srcs[r][i]), k);
        dst[i] = (int32_t)acc;
    }
}

void orc_sum_dequant_bf16(const int32_t *const *srcs, int R, uint16_t *dst, size_t n, int k)
{
    const float s = pow2f(-k);
    for (size_t i = 0; i < n; ++i) {
        uint32_t acc = 0;
        for (int r = 0; r < R; ++r) acc += (uint32_t)srcs[r][i];
        dst[i] = orc_f32_to_bf16((float)(int32_t)acc * s);
    }
}

float orc_absmax_bf16(const uint16_t *const *srcs, int R, size_t n)
{
    float m = 0.0f;
    for (int r = 0; r < R; ++r)
        for (size_t i = 0; i < n; ++i) {
            float a = fabsf(orc_bf16_to_f32(srcs[r][i]));
            if (a > m) m = a;
        }
    return m;
}

/* IEEE binary16: widening is exact; narrowing rounds to nearest even, past
 * 65504 to +-Inf (the halfway point 65520 rounds to Inf: 65504's last mantissa
 * bit is odd), below 2^-14 to subnormals (gradual underflow), NaN kept quiet. */
float orc_f16_to_f32(uint16_t h)
{
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
    union { uint32_t u; float f; } c;
    if (e == 0x1F) c.u = sign | 0x7F800000u | (m << 13);
    else if (e == 0) {
        c.f = (float)m * 5.9604644775390625e-08f;   /* m * 2^-24, exact */
        c.u |= sign;
    } else c.u = sign | ((e + 112u) << 23) | (m << 13);
    return c.f;
}

uint16_t orc_f32_to_f16(float f)
{
    union { uint32_t u; float f; } c;
    c.f = f;
    const uint32_t sign = (c.u >> 16) & 0x8000u, ax = c.u & 0x7FFFFFFFu;
    if (ax > 0x7F800000u) return (uint16_t)(sign | 0x7E00u | ((ax >> 13) & 0x3FFu));
    if (ax >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u);        /* >= 65520: Inf */
    const uint32_t e = ax >> 23, m = ax & 0x7FFFFFu;
    if (ax >= 0x38800000u) {                                          /* normal half */
        uint32_t h = ((e - 112u) << 10) | (m >> 13);
        const uint32_t rem = m & 0x1FFFu;
        if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;       /* a carry moves into the exponent */
        return (uint16_t)(sign | h);
    }
    if (ax <= 0x33000000u) return (uint16_t)sign;                     /* <= 2^-25: zero (2^-25 ties to even) */
    const uint32_t mm = m | 0x800000u, sh = 126u - e;                 /* subnormal: 14 <= sh <= 24 */
    uint32_t h = mm >> sh;
    const uint32_t rem = mm & ((1u << sh) - 1u), half = 1u << (sh - 1u);
    if (rem > half || (rem == half && (h & 1u))) ++h;
    return (uint16_t)(sign | h);
}

void orc_f16_to_f32_n(const uint16_t *h, float *f, size_t n)
{
    for (size_t i = 0; i < n; ++i) f[i] = orc_f16_to_f32(h[i]);
}

void orc_f32_to_f16_n(const float *f, uint16_t *h, size_t n)
{
    for (size_t i = 0; i < n; ++i) h[i] = orc_f32_to_f16(f[i]);
}

void orc_reduce_f16(const uint16_t *const *srcs, int R, uint16_t *dst, size_t n, int k)
{
    const float s = pow2f(-k);
    for (size_t i = 0; i < n; ++i) {
        uint32_t acc = 0;
        for (int r = 0; r < R; ++r) acc += (uint32_t)orc_quantise_one(orc_f16_to_f32(srcs[r][i]), k);
        dst[i] = orc_f32_to_f16((float)(int32_t)acc * s);
    }
}

void orc_quant_sum_f16(const uint16_t *const *srcs, int R, int32_t *dst, size_t n, int k)
{
    for (size_t i = 0; i < n; ++i) {
        uint32_t acc = 0;
        for (int r = 0; r < R; ++r) acc += (uint32_t)orc_quantise_one(orc_f16_to_f32(srcs[r][i]), k);
        dst[i] = (int32_t)acc;
    }
}

void orc_sum_dequant_f16(const int32_t *const *srcs, int R, uint16_t *dst, size_t n, int k)
{
    const float s = pow2f(-k);
    for (size_t i = 0; i < n; ++i) {
        uint32_t acc = 0;
        for (int r = 0; r < R; ++r) acc += (uint32_t)srcs[r][i];
        dst[i] = orc_f32_to_f16((float)(int32_t)acc * s);
    }
}

float orc_absmax_f16(const uint16_t *const *srcs, int R, size_t n)
{
    float m = 0.0f;
    for (int r = 0; r < R; ++r)
        for (size_t i = 0; i < n; ++i) {
            float a = fabsf(orc_f16_to_f32(srcs[r][i]));
            if (a > m) m = a;
        }
    return m;
}

int orc_choose_scale(float absmax, int R)
{
    if (!(absmax > 0.0f)) return ORC_SCALE_MAX;
    if (isinf(absmax)) return ORC_SCALE_MIN;
    double t = (double)absmax * (double)R;   /* exact: 24-bit mantissa x small int */
    int e;
    double m = frexp(t, &e);                 /* t = m * 2^e, m in [0.5, 1) */
    int k = (m == 0.5) ? (31 - e) : (30 - e);
    if (k < ORC_SCALE_MIN) k = ORC_SCALE_MIN;
    if (k > ORC_SCALE_MAX) k = ORC_SCALE_MAX;
    return k;
}

uint32_t orc_checksum_q32(const int32_t *q, size_t n, uint64_t index_base)
{
    uint32_t cs = 0;
    for (size_t i = 0; i < n; ++i)
        cs += (uint32_t)(2u * (uint32_t)(index_base + i) + 1u) * (uint32_t)q[i];
    return cs;
}

/* ------------------------------------------------------------------ */
/* root-switch aggregation (nts.c:231-250, :303-501)                    */
/* ------------------------------------------------------------------ */
#define SLOT(sw, psn) ((psn) & ((sw)->slots - 1))    /* nts.c:25 Idx(): psn % N, N a power of two */

size_t orc_switch_bytes(void) { return sizeof(orc_switch); }

const int32_t *orc_switch_slot(const orc_switch *sw, uint32_t psn) { return sw->aggregator[SLOT(sw, psn)]; }

int orc_switch_init_ring(orc_switch *sw, int fan_in, uint32_t slots)
{
    if (fan_in < 1 || fan_in > ORC_MAX_FAN_IN || slots < 2 || slots > ORC_SW_MAX_SLOTS || (slots & (slots - 1)))
        return -1;
    memset(sw, 0, sizeof(*sw));
    sw->fan_in = fan_in;
    sw->slots = slots;
    sw->window = slots / 2;                                    /* nts.c:21-22: N = 2 * WINDOW_SIZE */
    sw->root = 1;
    return 0;
}

int orc_switch_init_nonroot(orc_switch *sw, int fan_in, uint32_t slots, int flags)
{
    /* the parent's port is bit fan_in of the bitmap, as the result bit (nts.c:59, :366) */
    if ((flags & ~(ORC_SW_WIRE_ORDER | ORC_SW_RECYCLE)) || orc_switch_init_ring(sw, fan_in, slots) != 0)
        return -1;
    sw->root = 0;
    sw->flags = flags;
    return 0;
}

void orc_switch_init(orc_switch *sw, int fan_in)
{
    orc_switch_init_ring(sw, fan_in, ORC_SW_SLOTS);            /* the reference's ring: 16 slots, window 8 */
}

static void sw_clear(orc_switch *sw, uint32_t psn)
{
    /* nts.c:235-242 clear_state_data */
    const uint32_t s = SLOT(sw, psn);
    sw->arrival_state[s] = 0;
    sw->degree[s] = 0;
    memset(sw->reth_keeper[s], 0, sizeof(sw->reth_keeper[s]));
    memset(sw->aggregator[s], 0, sizeof(sw->aggregator[s]));
}

static inline int sw_all_fan_in(const orc_switch *sw, uint32_t s)
{
    const uint32_t mask = 0xffffffffu >> (32 - sw->fan_in);   /* nts.c:29 */
    return (sw->arrival_state[s] & mask) == mask;              /* nts.c:244-246 */
}

/* The root branch of nts.c:347-374 / :427-455 for one counted-or-not data
 * packet; the RETH of a WRITE_FIRST packet (NULL otherwise) goes into the
 * keeper with the first transmission (nts.c:442). */
static int sw_data(orc_switch *sw, int port, uint32_t psn, const uint8_t *payload_be_bytes, const uint8_t *reth)
{
    const uint32_t s = SLOT(sw, psn);
    const uint32_t port_bit = 1u << port;
    const uint32_t result_bit = 1u << sw->fan_in;              /* bit FAN_IN (nts.c:366) */
    sw->degree[s] += 1;                                        /* nts.c:351, :431 */

    if (sw->arrival_state[s] & port_bit) {                     /* nts.c:353 / :435 retransmit */
        if (sw->arrival_state[s] & result_bit) {               /* nts.c:354-356 / :436-438 replay */
            sw->replays++;
            return ORC_SW_REPLAY;
        }
        return ORC_SW_DROPPED;
    }
    /* first transmission: nts.c:359-363 / :441-445 */
    sw->arrival_state[s] |= port_bit;
    if (reth) memcpy(sw->reth_keeper[s][port], reth, ORC_RETH_HDR);
    {
        uint32_t *acc = (uint32_t *)sw->aggregator[s];
        for (int i = 0; i < ORC_LANES; ++i) {
            uint32_t w;
            memcpy(&w, payload_be_bytes + 4 * i, 4);
            acc[i] += to_be(w);                                /* ntohl */
        }
    }
    sw->adds++;
    if (sw_all_fan_in(sw, s)) {                                /* nts.c:365-372 / :447-453 */
        sw->arrival_state[s] |= result_bit;
        sw_clear(sw, psn + sw->window);                        /* nts.c:367 / :449 */
        return ORC_SW_BROADCAST;
    }
    return ORC_SW_ABSORBED;
}

/* The non-root branch of nts.c:376-400 / :457-482 for one UP data packet. */
static int sw_data_nonroot(orc_switch *sw, int port, uint32_t psn, const uint8_t *payload_be_bytes,
                           const uint8_t *reth)
{
    const uint32_t s = SLOT(sw, psn);
    const uint32_t port_bit = 1u << port;
    const uint32_t result_bit = 1u << sw->fan_in;              /* "received from the parent" (nts.c:378) */
    sw->degree[s] += 1;                                        /* nts.c:351, :431 */

    if (sw->arrival_state[s] & port_bit) {                     /* nts.c:377 / :458 retransmission */
        if (sw->arrival_state[s] & result_bit) {               /* :378-380 / :459-461 replay to the port */
            sw->replays++;
            return ORC_SW_REPLAY;
        }
        /* :381-384 / :462-465: every child retransmits when none got the
         * result, so the aggregate goes up again once per round of them */
        if (sw_all_fan_in(sw, s) && sw->degree[s] % sw->fan_in == 0) return ORC_SW_FORWARD;
        return ORC_SW_DROPPED;
    }
    /* first transmission: nts.c:388-392 / :469-474 */
    sw->arrival_state[s] |= port_bit;
    if (reth) memcpy(sw->reth_keeper[s][port], reth, ORC_RETH_HDR);
    {
        uint32_t *acc = (uint32_t *)sw->aggregator[s];
        for (int i = 0; i < ORC_LANES; ++i) {
            uint32_t w;
            memcpy(&w, payload_be_bytes + 4 * i, 4);
            acc[i] += to_be(w);                                /* ntohl */
        }
    }
    sw->adds++;
    return sw_all_fan_in(sw, s) ? ORC_SW_FORWARD : ORC_SW_ABSORBED;   /* :394-397 / :476-479 */
}

/* DOWN_DATA / DOWN_WRITE_FIRST_ONLY from the parent (nts.c:408-423 / :484-499) */
static int sw_down(orc_switch *sw, uint32_t psn, const uint8_t *payload_be_bytes)
{
    const uint32_t s = SLOT(sw, psn);
    const uint32_t result_bit = 1u << sw->fan_in;
    /* :412 / :488: taken only once, and only after every child's arrival */
    if ((sw->arrival_state[s] & result_bit) || !sw_all_fan_in(sw, s)) return ORC_SW_DROPPED;   /* :420-422 */
    if (sw->flags & ORC_SW_WIRE_ORDER) {
        for (int i = 0; i < ORC_LANES; ++i) {
            uint32_t w;
            memcpy(&w, payload_be_bytes + 4 * i, 4);
            sw->aggregator[s][i] = (int32_t)to_be(w);          /* ntohl, as the UP path adds */
        }
    } else {
        memcpy(sw->aggregator[s], payload_be_bytes, ORC_PAYLOAD_LEN);   /* :413 / :489, wire bytes as they are */
    }
    sw->arrival_state[s] |= result_bit;                        /* :414 / :490 */
    if (sw->flags & ORC_SW_RECYCLE) sw_clear(sw, psn + sw->window);
    return ORC_SW_DOWN;
}

int orc_switch_ingress(orc_switch *sw, int port, uint32_t psn,
                       const uint32_t *payload_be, uint32_t *egress_be)
{
    const int rc = sw_data(sw, port, psn, (const uint8_t *)payload_be, NULL);
    if (rc == ORC_SW_REPLAY || rc == ORC_SW_BROADCAST) {
        /* egress re-encode (util.c:403-405) */
        const uint32_t s = SLOT(sw, psn);
        for (int i = 0; i < ORC_LANES; ++i) egress_be[i] = to_be((uint32_t)sw->aggregator[s][i]);
    }
    return rc;
}

/* ------------------------------------------------------------------ */
/* CRC32 / ICRC / framing (util.c:106-195, :250-286, :331-442)          */
/* ------------------------------------------------------------------ */
static uint32_t crc_tab[8][256];
static int crc_ready;

static void crc_init(void)
{
    /* util.c:141-159: reflected table for poly 0xEDB88320, then the seven
     * derived slice-by-8 tables */
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int j = 0; j < 8; ++j) c = (c >> 1) ^ ((c & 1u) ? 0xEDB88320u : 0u);
        crc_tab[0][i] = c;
    }
    for (int t = 1; t < 8; ++t)
        for (int i = 0; i < 256; ++i)
            crc_tab[t][i] = (crc_tab[t - 1][i] >> 8) ^ crc_tab[0][crc_tab[t - 1][i] & 0xFFu];
    crc_ready = 1;
}

uint32_t orc_crc32(const void *data, size_t len)
{
    if (!crc_ready) crc_init();
    const uint8_t *p = (const uint8_t *)data;
    uint32_t c = 0xFFFFFFFFu;
    /* slice-by-8 main loop (util.c:165-187) */
    while (len >= 8) {
        uint32_t lo = ((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24)) ^ c;
        c = crc_tab[7][lo & 0xFF] ^ crc_tab[6][(lo >> 8) & 0xFF] ^ crc_tab[5][(lo >> 16) & 0xFF] ^
            crc_tab[4][lo >> 24] ^ crc_tab[3][p[4]] ^ crc_tab[2][p[5]] ^ crc_tab[1][p[6]] ^
            crc_tab[0][p[7]];
        p += 8;
        len -= 8;
    }
    while (len--) c = (c >> 8) ^ crc_tab[0][(c ^ *p++) & 0xFFu];   /* util.c:190-192 */
    return c ^ 0xFFFFFFFFu;
}

uint32_t orc_icrc(const uint8_t *frame)
{
    /* util.c:250-286 */
    const uint8_t *ip = frame + ORC_ETH_HDR;
    const int len = (int)(((uint32_t)ip[2] << 8) | ip[3]) - ORC_ICRC_LEN;  /* IP total length - ICRC */
    uint8_t buf[8 + 4096];
    if (len < 0 || len > 4096) return 0;
    memset(buf, 0xFF, 8);
    memcpy(buf + 8, ip, (size_t)len);
    uint8_t *mip = buf + 8;
    mip[1] = 0xFF;                                   /* tos        (util.c:266) */
    mip[8] = 0xFF;                                   /* ttl        (util.c:267) */
    mip[10] = 0xFF; mip[11] = 0xFF;                  /* ip csum    (util.c:268) */
    uint8_t *udp = mip + ORC_IP_HDR;
    udp[6] = 0xFF; udp[7] = 0xFF;                    /* udp csum   (util.c:269) */
    uint8_t *bth = udp + ORC_UDP_HDR;
    bth[4] = 0xFF;                                   /* BTH resv8a (util.c:270) */
    return orc_crc32(buf, (size_t)len + 8);
}

uint16_t orc_ipv4_checksum(const uint8_t *ip_hdr)
{
    /* util.c:106-127, checksum field treated as 0; result in network order bytes */
    const int ihl = (ip_hdr[0] & 0x0F) * 4;
    uint32_t sum = 0;
    for (int i = 0; i < ihl; i += 2) {
        if (i == 10) continue;
        sum += ((uint32_t)ip_hdr[i] << 8) | ip_hdr[i + 1];
    }
    while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
    return (uint16_t)~sum;   /* host-order value; caller stores it big-endian */
}

static inline void put16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static inline void put32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

/* util.c:331-442 build_eth_packet, for its three packet types the switch
 * sends: PACKET_TYPE_DATA (payload, no RETH), PACKET_TYPE_RETH (RETH +
 * payload) and PACKET_TYPE_ACK (AETH, no payload). */
enum { PKT_DATA, PKT_RETH, PKT_ACK };

static size_t build_frame(uint8_t *frame, int type, const orc_frame_hdr *h, const int32_t *payload_host, int n_words,
                          uint32_t msn, const uint8_t *reth16)
{
    const int data_len = type == PKT_ACK ? 0 : n_words * 4;
    size_t total = ORC_ETH_HDR + ORC_IP_HDR + ORC_UDP_HDR + ORC_BTH_HDR + (size_t)data_len + ORC_ICRC_LEN;
    if (type == PKT_ACK) total += ORC_AETH_HDR;                         /* util.c:342-343 */
    else if (type == PKT_RETH) total += ORC_RETH_HDR;                   /* util.c:344-345 */
    uint8_t *eth = frame;
    memcpy(eth, h->dst_mac, 6);                                         /* util.c:349-351 */
    memcpy(eth + 6, h->src_mac, 6);
    put16(eth + 12, 0x0800);
    uint8_t *ip = frame + ORC_ETH_HDR;                                  /* util.c:354-364 */
    ip[0] = 0x45; ip[1] = 0x00;
    put16(ip + 2, (uint16_t)(total - ORC_ETH_HDR));
    ip[4] = 0x11; ip[5] = 0x11;
    put16(ip + 6, 0x4000);
    ip[8] = 0x40; ip[9] = 0x11;
    memcpy(ip + 12, &h->src_ip, 4);
    memcpy(ip + 16, &h->dst_ip, 4);
    ip[10] = 0; ip[11] = 0;
    put16(ip + 10, orc_ipv4_checksum(ip));
    uint8_t *udp = ip + ORC_IP_HDR;                                     /* util.c:367-372 */
    put16(udp + 0, h->src_port);
    put16(udp + 2, h->dst_port);
    put16(udp + 4, (uint16_t)(total - ORC_ETH_HDR - ORC_IP_HDR));
    udp[6] = 0; udp[7] = 0;
    uint8_t *bth = udp + ORC_UDP_HDR;                                   /* util.c:376-388 */
    bth[0] = type == PKT_ACK ? 0x11 : h->opcode; bth[1] = 0x00; bth[2] = 0xFF; bth[3] = 0xFF;
    put32(bth + 4, h->qp & 0x00FFFFFFu);
    put32(bth + 8, type == PKT_ACK ? h->psn : (h->psn | 0x80000000u)); /* ack request on data (util.c:385-388) */
    uint8_t *d = bth + ORC_BTH_HDR;
    if (type == PKT_ACK) {                                              /* util.c:391-397 */
        put32(d, msn | 0x1f000000u);
    } else {
        if (type == PKT_RETH) {                                         /* util.c:409-417 */
            if (reth16) memcpy(d, reth16, ORC_RETH_HDR); else memset(d, 0, ORC_RETH_HDR);
            d += ORC_RETH_HDR;
        }
        for (int i = 0; i < n_words; ++i) put32(d + 4 * i, (uint32_t)payload_host[i]);   /* util.c:403-405, :419-421 */
    }
    const uint32_t icrc = orc_icrc(frame);                              /* util.c:425-426 */
    memcpy(frame + total - ORC_ICRC_LEN, &icrc, 4);                     /* stored host order */
    return total;
}

size_t orc_build_data_frame(uint8_t *frame, const orc_frame_hdr *h, const int32_t *payload_host,
                            int n_words, int with_reth, const uint8_t *reth16)
{
    return build_frame(frame, with_reth ? PKT_RETH : PKT_DATA, h, payload_host, n_words, 0, reth16);
}

size_t orc_build_ack_frame(uint8_t *frame, const orc_frame_hdr *h, uint32_t msn)
{
    return build_frame(frame, PKT_ACK, h, NULL, 0, msn, NULL);
}

/* nts.c:252-298: the connection's fields as build_eth_packet takes them (src =
 * my_*, dst = peer_*, QPN = peer_qp) */
static void conn_hdr(orc_frame_hdr *h, const orc_conn *c, uint32_t psn, uint8_t opcode)
{
    memcpy(h->src_mac, c->my_mac, 6);
    memcpy(h->dst_mac, c->peer_mac, 6);
    h->src_ip = c->my_ip;
    h->dst_ip = c->peer_ip;
    h->src_port = c->my_port;
    h->dst_port = c->peer_port;
    h->qp = c->peer_qp;
    h->psn = psn;
    h->opcode = opcode;
}

static int is_data_op(uint8_t op) { return op == 0x00 || op == 0x01 || op == 0x02 || op == 0x04 || op == 0x07 || op == 0x08; }
static int is_wf_op(uint8_t op) { return op == 0x06 || op == 0x0A; }

/* pipeline() of a non-root switch (root == 0, nts.c:303-501): ports below
 * fan_in are children (UP_*), port fan_in the parent (DOWN_*, :320-343). */
static int pipeline_nonroot(orc_switch *sw, const orc_conn *conns, int port, const uint8_t *frame, size_t row_len,
                            uint8_t *out, size_t out_stride, int *out_len)
{
    const int F = sw->fan_in, up = port < F;
    const uint8_t op = frame[42];
    const uint32_t psn = ((uint32_t)frame[51] << 16) | ((uint32_t)frame[52] << 8) | frame[53];   /* :311 */
    const int udp_len = ((int)frame[38] << 8) | frame[39];
    orc_frame_hdr h;
    if (op == 0x11) {
        if (!up) return ORC_SW_IGNORED;                        /* DOWN_ACK: "impossible" (:424-426) */
        conn_hdr(&h, &conns[port], psn, 0x11);                 /* UP_ACK: reflect (:403-406) */
        out_len[port] = (int)orc_build_ack_frame(out + (size_t)port * out_stride, &h, psn + 1);
        return ORC_SW_ACK;
    }
    if (!is_data_op(op) && !is_wf_op(op)) return ORC_SW_IGNORED;
    const int wf = is_wf_op(op);
    const int data_len = udp_len - ORC_BTH_HDR - ORC_UDP_HDR - ORC_ICRC_LEN - (wf ? ORC_RETH_HDR : 0);   /* :349, :410 */
    const size_t doff = 54 + (wf ? ORC_RETH_HDR : 0);
    if (data_len != ORC_PAYLOAD_LEN || doff + ORC_PAYLOAD_LEN > row_len) return ORC_SW_INVALID;   /* :350, :411 */
    const int rc = up ? sw_data_nonroot(sw, port, psn, frame + doff, wf ? frame + 54 : NULL)
                      : sw_down(sw, psn, frame + doff);
    if (rc != ORC_SW_FORWARD && rc != ORC_SW_REPLAY && rc != ORC_SW_DOWN) return rc;
    /* the aggregator words re-encoded with htonl (send_roce_data[_with_reth],
     * util.c:403-405, :419-421) and this packet's opcode */
    const uint32_t s = SLOT(sw, psn);
    int32_t agg[ORC_LANES];
    memcpy(agg, sw->aggregator[s], sizeof(agg));
    int c0 = port, c1 = port + 1;                               /* REPLAY: the retransmitting child */
    if (rc == ORC_SW_FORWARD) c0 = F, c1 = F + 1;               /* the parent, RETH NULL (:464, :478) */
    if (rc == ORC_SW_DOWN) c0 = 0, c1 = F;                      /* every child (:416-418, :492-494) */
    for (int c = c0; c < c1; ++c) {
        conn_hdr(&h, &conns[c], psn, op);
        out_len[c] = (int)orc_build_data_frame(out + (size_t)c * out_stride, &h, agg, ORC_LANES, wf,
                                               wf && c < F ? sw->reth_keeper[s][c] : NULL);
    }
    return rc;
}

int orc_switch_pipeline(orc_switch *sw, const orc_conn *conns, int port, const uint8_t *frame, size_t row_len,
                        uint8_t *out, size_t out_stride, int *out_len)
{
    const int rows = sw->fan_in + (sw->root ? 0 : 1);          /* a non-root's row fan_in: its parent */
    for (int c = 0; c < rows; ++c) out_len[c] = 0;
    /* the root has children only: a port outside them (the reference's DOWN_*
     * path, nts.c:408-426, :484-499, is a non-root switch's) is refused */
    if (port < 0 || port >= rows || row_len < 64) return ORC_SW_INVALID;
    if (!sw->root) return pipeline_nonroot(sw, conns, port, frame, row_len, out, out_stride, out_len);
    /* parser, nts.c:307-344 */
    const uint8_t op = frame[42];
    const uint32_t psn = ((uint32_t)frame[51] << 16) | ((uint32_t)frame[52] << 8) | frame[53];   /* :311 */
    const int udp_len = ((int)frame[38] << 8) | frame[39];
    orc_frame_hdr h;
    if (op == 0x11) {                                          /* UP_ACK: reflect (nts.c:403-406, :284-298) */
        conn_hdr(&h, &conns[port], psn, 0x11);
        out_len[port] = (int)orc_build_ack_frame(out + (size_t)port * out_stride, &h, psn + 1);
        return ORC_SW_ACK;
    }
    if (!is_data_op(op) && !is_wf_op(op)) return ORC_SW_IGNORED;
    const int wf = is_wf_op(op);
    const int data_len = udp_len - ORC_BTH_HDR - ORC_UDP_HDR - ORC_ICRC_LEN - (wf ? ORC_RETH_HDR : 0);   /* :349, :429 */
    const size_t doff = 54 + (wf ? ORC_RETH_HDR : 0);
    if (data_len != ORC_PAYLOAD_LEN || doff + ORC_PAYLOAD_LEN > row_len) return ORC_SW_INVALID;   /* assert, :350 */
    const int rc = sw_data(sw, port, psn, frame + doff, wf ? frame + 54 : NULL);
    if (rc != ORC_SW_BROADCAST && rc != ORC_SW_REPLAY) return rc;
    /* send_roce_data (no RETH) for a data packet, send_roce_data_with_reth with
     * the child's kept RETH for a WRITE_FIRST one; both with THIS packet's
     * opcode (nts.c:355, :370, :437, :452) */
    const uint32_t s = SLOT(sw, psn);
    int32_t agg[ORC_LANES];
    memcpy(agg, sw->aggregator[s], sizeof(agg));
    const int c0 = rc == ORC_SW_BROADCAST ? 0 : port, c1 = rc == ORC_SW_BROADCAST ? sw->fan_in : port + 1;
    for (int c = c0; c < c1; ++c) {
        conn_hdr(&h, &conns[c], psn, op);
        out_len[c] = (int)orc_build_data_frame(out + (size_t)c * out_stride, &h, agg, ORC_LANES, wf,
                                               wf ? sw->reth_keeper[s][c] : NULL);
    }
    return rc;
}

/* ------------------------------------------------------------------ */
/* loopback: api.c:293-327 + :403-452 against nts.c pipeline()          */
/* ------------------------------------------------------------------ */
typedef struct { int rank; uint32_t psn; } pkt_t;

int orc_allreduce_write_loopback(int R, const int32_t *const *src, uint32_t len,
                                 int32_t *const *dst, int dup_every,
                                 uint64_t *frames_out, int with_icrc)
{
    if (R < 1 || R > ORC_MAX_FAN_IN) return -1;
    const int message_num = (int)(len / ORC_PAYLOAD_COUNT);                 /* api.c:406 */
    const int window_msgs = ORC_WINDOW_SIZE / ORC_MESSAGE_SIZE;             /* api.c:408 */
    if (message_num < window_msgs) return -1;   /* the reference would read past src */
    const size_t buf_words = (size_t)message_num * ORC_PAYLOAD_COUNT;

    uint32_t **send_payload = calloc((size_t)R, sizeof(*send_payload));
    uint32_t **recv_payload = calloc((size_t)R, sizeof(*recv_payload));
    uint8_t **delivered = calloc((size_t)R, sizeof(*delivered));   /* per (msg) packet bitmap */
    int *send_num = calloc((size_t)R, sizeof(int));
    int *recv_num = calloc((size_t)R, sizeof(int));
    const size_t qcap = (size_t)R * (size_t)message_num * ORC_PKTS_PER_MSG * 2 + 16;
    pkt_t *q = malloc(qcap * sizeof(pkt_t));
    orc_switch *sw = malloc(sizeof(orc_switch));
    uint32_t egress[ORC_LANES];
    int32_t egress_host[ORC_LANES];
    uint8_t frame[2048];
    uint64_t frames = 0, ingress_count = 0;
    size_t qh = 0, qt = 0;
    int ok = 1;

    for (int r = 0; r < R; ++r) {
        send_payload[r] = malloc(buf_words * 4);
        recv_payload[r] = calloc(buf_words, 4);
        delivered[r] = calloc((size_t)message_num, 1);
        if (!send_payload[r] || !recv_payload[r] || !delivered[r]) ok = 0;
    }
    if (!send_payload || !recv_payload || !delivered || !send_num || !recv_num || !q || !sw) ok = 0;
    if (!ok) goto out;
    orc_switch_init(sw, R);

#define POST_SEND(r, idx)                                                                     \
    do {                                                                                      \
        orc_encode_be32(src[r] + (size_t)(idx) * ORC_PAYLOAD_COUNT,                           \
                        send_payload[r] + (size_t)(idx) * ORC_PAYLOAD_COUNT, ORC_PAYLOAD_COUNT); \
        for (int p_ = 0; p_ < ORC_PKTS_PER_MSG; ++p_) {                                       \
            q[qt].rank = (r); q[qt].psn = (uint32_t)((idx) * ORC_PKTS_PER_MSG + p_); ++qt;    \
        }                                                                                     \
    } while (0)

    for (int r = 0; r < R; ++r)
        for (int i = 0; i < window_msgs; ++i) { POST_SEND(r, i); send_num[r]++; }   /* api.c:408-411 */

    while (qh < qt) {
        const pkt_t pk = q[qh++];
        const uint32_t msg = pk.psn / ORC_PKTS_PER_MSG, part = pk.psn % ORC_PKTS_PER_MSG;
        const uint32_t *payload = send_payload[pk.rank] + (size_t)pk.psn * ORC_LANES;
        int passes = (dup_every > 0 && (++ingress_count % (uint64_t)dup_every) == 0) ? 2 : 1;
        for (int pass = 0; pass < passes; ++pass) {      /* pass 1 = immediate retransmit */
            const int rc = orc_switch_ingress(sw, pk.rank, pk.psn, payload, egress);
            if (rc != ORC_SW_BROADCAST && rc != ORC_SW_REPLAY) continue;
            const int c0 = (rc == ORC_SW_BROADCAST) ? 0 : pk.rank;
            const int c1 = (rc == ORC_SW_BROADCAST) ? R : pk.rank + 1;
            for (int c = c0; c < c1; ++c) {
                if (with_icrc) {
                    orc_frame_hdr h;
                    memset(&h, 0, sizeof(h));
                    h.qp = 0x11; h.psn = pk.psn; h.opcode = part == 0 ? 0x06 : (part == 3 ? 0x08 : 0x07);
                    h.src_port = 4791; h.dst_port = 4791;
                    orc_decode_be32(egress, egress_host, ORC_LANES);
                    orc_build_data_frame(frame, &h, egress_host, ORC_LANES, part == 0, NULL);
                }
                frames++;
                /* the NIC writes the payload at the RETH address = own receive_payload + idx*4096 */
                memcpy(recv_payload[c] + (size_t)pk.psn * ORC_LANES, egress, ORC_PAYLOAD_LEN);
                const uint8_t bit = (uint8_t)(1u << part);
                if (delivered[c][msg] & bit) continue;
                delivered[c][msg] |= bit;
                if (delivered[c][msg] != 0x0F) continue;
                /* completion of WRITE wr_id = msg: api.c:422-438 */
                orc_decode_be32(recv_payload[c] + (size_t)msg * ORC_PAYLOAD_COUNT,
                                dst[c] + (size_t)recv_num[c] * ORC_PAYLOAD_COUNT, ORC_PAYLOAD_COUNT);
                recv_num[c]++;
                if (send_num[c] < message_num) { POST_SEND(c, send_num[c]); send_num[c]++; }
            }
        }
    }
#undef POST_SEND
    for (int r = 0; r < R; ++r)
        if (recv_num[r] != message_num) ok = 0;

out:
    if (frames_out) *frames_out = frames;
    for (int r = 0; r < R && send_payload && recv_payload && delivered; ++r) {
        free(send_payload[r]); free(recv_payload[r]); free(delivered[r]);
    }
    free(send_payload); free(recv_payload); free(delivered);
    free(send_num); free(recv_num); free(q); free(sw);
    return ok ? message_num : -1;
}
