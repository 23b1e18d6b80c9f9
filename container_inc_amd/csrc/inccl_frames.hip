// inccl_frames.hip -- the reference's switch dataplane on the GPU (gfx950):
// RoCEv2 frame parse, per-PSN idempotent aggregation, egress frame build and
// the RoCE ICRC (CRC-32).  Reference: repository/src/non_termination_switch.c
// (nts.c) :303-501 for the pipeline and :55-60 / :231-250 for its state;
// repository/src/util.c:331-442 (build_eth_packet), :250-286 (compute_icrc),
// :141-195 (crc32), :106-127 (ipv4_checksum).
//
// A batch of frames (frame index = arrival order) goes through
//   k_ingress_claim   a lane per frame: parse + validate, and the first copy of
//                     every (slot, port) by a batch-tagged atomicMin
//   k_ingress_classify  a lane per frame: classify in the reference's serial
//                     order (nts.c:353-372), the arrival bitmap, the RETH keeper
//                     (:442), the recycle (:235-242, :367)
//   k_ingress_sum     a wave per two consecutive frames: each completed or
//                     absorbed PSN's counted arrivals summed into its aggregate
//                     (:361-363), every data frame counted in its slot's degree
//                     (:351)
//   k_egress<F>       persistent, a wave per 4 input frames at a time: the COMPLETED
//                     broadcasts (:447-453) and REPLAY resends (:353-356) from the
//                     state ingress left, and the ACK reflections (:403-406),
//                     frames per util.c:331-442
// inccl_switch_ingress runs the first three, inccl_switch_egress the last,
// inccl_switch_batch all four.  A non-root switch (nts.c:376-400, :408-423,
// :457-499) runs k_nr_claim / k_nr_classify / k_nr_sum for ingress (each
// slot's frames decided in arrival order by one lane) and k_egress<F, O, true>,
// whose row fan_in per input frame is the parent's.  The ICRC is linear over GF(2), so every CRC
// here is a XOR of table lookups reduced over the wave with DPP -- no serial
// byte loop.
//
// State on the GPU (slots = PSN ring size, power of two; the reference uses 16):
//   agg[slots][256] int32        aggregator        (nts.c:55)
//   arrival[slots][2] uint64     port bitmap + bit fan_in = "result known" (nts.c:59, :366),
//                                tagged with the batch that wrote it, double-buffered by
//                                batch parity (k_ingress_classify)
//   degree[slots] int32          arrivals incl. retransmits (nts.c:60, :351)
//   reth[slots][fan_in][16 B]    RETH of each child's WRITE_FIRST (nts.c:57, :442)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <mutex>

#include "inccl_frames.h"

namespace {

constexpr int kWave = 64;
constexpr int kWin = 1088;            // ICRC window: the longest message (1098-B frame from byte 10)
constexpr int kFrameMax = 1152;
constexpr int kLanes = 256;           // int32 lanes per packet (nts.c:55)
constexpr int kAuxNt = 2;   // buffer instruction cache policy: nt (streaming, not re-read)
constexpr int kAuxSc1 = 16;   // buffer instruction cache policy: sc1 (write-through)
constexpr int kOobOffset = 0x7FFFFFF0;   // past any row: a buffer store there is dropped, a load returns 0

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

// frame bytes that read as 0xFF while the ICRC runs: 10-13 carry the CRC init
// (the 4 x 0xFF prefix), the rest are the ICRC masks of util.c:266-270 (tos,
// ttl, IP checksum, UDP checksum, BTH resv8a)
constexpr int kNumMasked = 11;
__device__ __forceinline__ int masked_pos(int i)
{
    constexpr uint64_t lo = 10ull | 11ull << 8 | 12ull << 16 | 13ull << 24 | 15ull << 32 | 22ull << 40 | 24ull << 48 |
                            25ull << 56;
    constexpr uint32_t hi = 40u | 41u << 8 | 46u << 16;
    return i < 8 ? (int)((lo >> (8 * i)) & 0xFF) : (int)((hi >> (8 * (i - 8))) & 0xFF);
}

// a value whose bits the compiler may not reason about: keeps a nibble plane's
// byte extracts as byte extracts (one SDWA select each) instead of folding them
// back into a shift + mask of the original word
__device__ __forceinline__ uint32_t opaque_u32(uint32_t v)
{
    asm("" : "+v"(v));
    return v;
}

__device__ __forceinline__ uint64_t opaque64(uint64_t v)
{
    asm("" : "+v"(v));
    return v;
}

// a value nothing reads on the path where it is left so (no instruction sets it)
__device__ __forceinline__ uint32_t unset() { return __builtin_nondeterministic_value(0u); }
__device__ __forceinline__ u4 unset4() { return u4{unset(), unset(), unset(), unset()}; }

// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// an ICRC is computed only for an IP length the window holds and whose frame
// lies inside its row: a header claiming more bytes than the row has reads as
// malformed (ICRC 0), never as the next row's bytes
__device__ __forceinline__ bool icrc_len_ok(int ipt, int64_t stride)
{
    return ipt >= 28 && ipt <= kWin && 14 + ipt <= kFrameMax && 14 + ipt <= stride;
}

// ---------------------------------------------------------------------------
// Standalone ICRC (inccl_icrc_frames; util.c:250-286 for any frame), two frames
// per wave: lanes 0-31 take frame 2p, lanes 32-63 frame 2p+1, each lane a
// 34-byte segment of the frame's ICRC message right-aligned in a 1088-byte
// window (32 x 34; leading zeros do not change a raw CRC).  Each lane loads its
// segment straight from the frame (two dwordx4 + two dword buffer loads at the
// segment's dword offset), sets the mask bytes and clears the bytes before the
// message with one (AND, OR) LDS table lookup per dword, computes the segment's
// CRC as 68 independent nibble lookups, shifts it to the window's end
// (Z_{34 (31 - lane')}, 8 lookups in a lane-major table) and the 32-lane halves
// XOR-reduce with DPP.  Every memory instruction runs on every pass (a frame
// past the end, or malformed, gets a zero-size buffer: its loads return 0 and
// its store is dropped), so the waits stay one pass deep.  The variants this
// was chosen over (LDS-staged frames, one frame per wave, byte tables, two pairs
// per pass, the VALU mask) live in tools/tune/tune_icrc.hip.
// ---------------------------------------------------------------------------
constexpr int kSeg2 = 34;
__device__ uint32_t g_seg34[kSeg2][2][16];          // [byte j][nibble][value] = Z_{33-j}(T[value << 4 nibble])
__device__ uint32_t g_lane_shift32[8][16][32];      // [nibble][value][lane'] = Z_{34 (31 - lane')}(value << 4 nibble)

struct IcrcLds {
    uint32_t seg[kSeg2][2][16];
    uint32_t lane_sh[8][16][32];
    uint32_t andor[32][2];   // [nibble | 16 (frame dword <= 2)] -> (AND, OR)
};

// the masked byte positions (10-13, 15, 22, 24, 25, 40, 41, 46) as a bitmap
constexpr uint64_t kIcrcMaskBits = (1ull << 10) | (1ull << 11) | (1ull << 12) | (1ull << 13) | (1ull << 15) |
                                   (1ull << 22) | (1ull << 24) | (1ull << 25) | (1ull << 40) | (1ull << 41) |
                                   (1ull << 46);

// dw[k] = frame dword d0 + k -> (dw & AND) | OR from the 32-entry table,
// indexed by the dword's mask nibble and a "dword <= 2" bit: the mask bytes set
// to 0xFF and frame bytes 0-9 cleared (bytes 10-11 of dword 2 are then set by
// its OR), so the CRC needs no per-byte zeroing of the leading bytes.  The
// bitmap shift is clamped: a segment far before a short frame would shift it by
// 64 or more, which the hardware takes modulo 64.
__device__ __forceinline__ void icrc_mask_regs(uint32_t (&dw)[10], int d0, const IcrcLds& t)
{
    const int s4 = 4 * d0;
    const uint64_t x = (d0 >= 12 || d0 <= -16) ? 0ull : (s4 >= 0 ? kIcrcMaskBits >> s4 : kIcrcMaskBits << (-s4));
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    const int cnt = min(max(3 - d0, 0), 10);           // dwords k with d0 + k <= 2
    const uint32_t zbits = (1u << cnt) - 1u;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const uint32_t i = __builtin_amdgcn_ubfe(k < 8 ? lo : hi, 4 * (k & 7), 4) | (((zbits >> k) & 1u) << 4);
        dw[k] = (dw[k] & t.andor[i][0]) | t.andor[i][1];
    }
}

// The raw CRC contribution of this lane's 34-byte segment (frame byte o on;
// dw[k] = frame dword (o >> 2) + k, masked), shifted to the window's end.
__device__ __forceinline__ uint32_t icrc_segment(const uint32_t (&dw)[10], int o, const IcrcLds& t, int l)
{
    const uint32_t sh = (uint32_t)o & 3u;
    uint32_t a[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) a[k] = __builtin_amdgcn_alignbyte(dw[k + 1], dw[k], sh);
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t lo = opaque_u32(a[k] & 0x0F0F0F0Fu), hi = opaque_u32((a[k] >> 4) & 0x0F0F0F0Fu);
        uint32_t v[8];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            v[2 * b] = t.seg[4 * k + b][0][(uint8_t)(lo >> (8 * b))];
            v[2 * b + 1] = t.seg[4 * k + b][1][(uint8_t)(hi >> (8 * b))];
        }
        c = xor3(xor3(xor3(c, v[0], v[1]), v[2], v[3]), xor3(v[4], v[5], v[6]), v[7]);
    }
    // bytes 32 and 33 of the segment
    c = xor3(c, t.seg[32][0][a[8] & 15u], t.seg[32][1][(a[8] >> 4) & 15u]);
    c = xor3(c, t.seg[33][0][(a[8] >> 8) & 15u], t.seg[33][1][(a[8] >> 12) & 15u]);
    const uint32_t clo = opaque_u32(c & 0x0F0F0F0Fu), chi = opaque_u32((c >> 4) & 0x0F0F0F0Fu);
    uint32_t v[8];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        v[2 * b] = t.lane_sh[2 * b][(uint8_t)(clo >> (8 * b))][l];
        v[2 * b + 1] = t.lane_sh[2 * b + 1][(uint8_t)(chi >> (8 * b))][l];
    }
    return xor3(xor3(v[0], v[1], v[2]), xor3(v[3], v[4], v[5]), v[6]) ^ v[7];
}

// Out-of-range segment words: a load partly before the frame covers only bytes
// below 10 (cleared or masked), and the segment's last byte o + 33 <= 14 +
// ip_total - 5 keeps both dwordx4 inside the frame.
template <int kW>
__global__ __launch_bounds__(kWave* kW) void k_icrc(const uint8_t* __restrict__ frames, int64_t stride, int64_t count,
                                                     uint32_t* __restrict__ out)
{
    __shared__ IcrcLds t;
    for (int i = threadIdx.x; i < kSeg2 * 2 * 16; i += blockDim.x) (&t.seg[0][0][0])[i] = (&g_seg34[0][0][0])[i];
    for (int i = threadIdx.x; i < 8 * 16 * 32; i += blockDim.x) (&t.lane_sh[0][0][0])[i] = (&g_lane_shift32[0][0][0])[i];
    if (threadIdx.x < 32) {
        const uint32_t m = ((threadIdx.x & 15u) * 0x00204081u) & 0x01010101u;   // nibble bit i -> byte i
        t.andor[threadIdx.x][0] = threadIdx.x & 16u ? 0u : 0xFFFFFFFFu;
        t.andor[threadIdx.x][1] = (m << 8) - m;
    }
    __syncthreads();
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    const int half = lane >> 5, l = lane & 31;
    const int64_t pairs = (count + 1) >> 1, step = (int64_t)gridDim.x * kW;
    int64_t q = (int64_t)blockIdx.x * kW + w;
    if (q >= pairs) return;
    // one buffer per pair (wave-uniform): its two rows, one for a last odd frame, none past the end
    auto pair_rsrc = [&](int64_t pp) {
        const int64_t rows = count - 2 * pp;
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(frames) + (rows > 0 ? 2 * pp : 0) * stride, 0,
                                                 rows >= 2 ? (int)(2 * stride) : rows == 1 ? (int)stride : 0, 0x00020000);
    };
    const int row_off = half * (int)stride;
    // bytes 16-19 of this half's frame (the IP total length), 0 past the end
    auto hdr = [&](int64_t pp) -> uint32_t {
        return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(pair_rsrc(pp), stride >= 20 ? row_off + 16 : kOobOffset, 0, 0);
    };
    auto fetch = [&](int64_t pp, uint32_t h, uint32_t (&dw)[10], int& o, bool& ok) {
        const int64_t f = 2 * pp + half;
        const int ipt = (int)(((h & 0xFFu) << 8) | ((h >> 8) & 0xFFu));
        ok = f < count && icrc_len_ok(ipt, stride);
        o = 10 + l * kSeg2 - (kWin - ipt);
        // the segment's dwords, inside this frame's row: a dword before the row (a
        // lane whose segment starts before byte 10) or past the frame's last dword
        // reads 0; the two dwordx4 never reach past the frame (above)
        const int d = o >> 2, words = (14 + ipt + 3) >> 2;
        const __amdgpu_buffer_rsrc_t rs = pair_rsrc(pp);
        // (each offset a VGPR the compiler cannot see through: a select it could
        // split into two loads on two paths would bring back the joined waits)
        auto at = [&](int k) {
            return (int)opaque_u32((uint32_t)(ok && d + k >= 0 && d + k < words ? row_off + 4 * (d + k) : kOobOffset));
        };
        const u4 a = __builtin_amdgcn_raw_buffer_load_b128(
            rs, (int)opaque_u32((uint32_t)(ok && d >= 0 ? row_off + 4 * d : kOobOffset)), 0, 0);
        const u4 b = __builtin_amdgcn_raw_buffer_load_b128(rs, at(4), 0, 0);
        dw[8] = __builtin_amdgcn_raw_buffer_load_b32(rs, at(8), 0, 0);
        dw[9] = __builtin_amdgcn_raw_buffer_load_b32(rs, at(9), 0, 0);
        dw[0] = a.x; dw[1] = a.y; dw[2] = a.z; dw[3] = a.w;
        dw[4] = b.x; dw[5] = b.y; dw[6] = b.z; dw[7] = b.w;
    };
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)(4 * count), 0x00020000);
    uint32_t cur[10];
    int o;
    bool ok;
    fetch(q, hdr(q), cur, o, ok);
    uint32_t hn = hdr(q + step);
    // a dropped store: the loop is entered with its back edge's memory history
    __builtin_amdgcn_raw_buffer_store_b32(0u, ors, kOobOffset, 0, 0);
    for (;;) {
        const int64_t qn = q + step;
        uint32_t nxt[10];
        int on;
        bool okn;
        fetch(qn, hn, nxt, on, okn);
        hn = hdr(qn + step);
        icrc_mask_regs(cur, o >> 2, t);
        uint32_t x = ok ? icrc_segment(cur, o, t, l) : 0u;
        // XOR-reduce each 32-lane half: quads, half-rows, rows, then row 0 into
        // row 1 and row 2 into row 3 (lanes 31 and 63 end with the two frames)
        x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);
        x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);
        x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);
        x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false);
        x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
        const uint32_t ca = ~(uint32_t)__builtin_amdgcn_readlane((int)x, 31);
        const uint32_t cb = ~(uint32_t)__builtin_amdgcn_readlane((int)x, 63);
        // lane 0 writes frame 2 q, lane 32 frame 2 q + 1 (past the end: dropped)
        __builtin_amdgcn_raw_buffer_store_b32(ok ? (half ? cb : ca) : 0u, ors,
                                              l == 0 && q < pairs ? (int)(4 * (2 * q + half)) : kOobOffset, 0, 0);
        q = qn;
        if (q >= pairs) break;
#pragma unroll
        for (int k = 0; k < 10; ++k) cur[k] = nxt[k];
        o = on;
        ok = okn;
    }
}

__device__ __forceinline__ bool is_data_opcode(uint8_t op)
{
    return op == 0x00 || op == 0x01 || op == 0x02 || op == 0x04 || op == 0x07 || op == 0x08;   // nts.c:314-319
}
__device__ __forceinline__ bool is_write_first(uint8_t op) { return op == 0x06 || op == 0x0A; }   // nts.c:327-328

// payload word i of the frame at `fr`, its payload at byte 54 + 16*wf (2-byte
// aligned), network order -> host order (nts.c:361-363)
__device__ __forceinline__ uint32_t payload_word(const uint8_t* fr, uint32_t wf, int i)
{
    const uint16_t* d16 = reinterpret_cast<const uint16_t*>(fr + 54 + 16 * wf);
    return __builtin_bswap32((uint32_t)d16[2 * i] | ((uint32_t)d16[2 * i + 1] << 16));
}

// Payload words 4 lane .. 4 lane + 3, host order, from the 16-byte chunks that
// hold them: the payload starts at byte 54 or 70, both 6 mod 16, so lane l's
// words are bytes 6-15 of chunk `lo` and bytes 0-5 of chunk `hi` (the next one).
__device__ __forceinline__ void payload_from_chunks(u4 lo, uint32_t hi0, uint32_t hi1, uint32_t (&w)[4])
{
    w[0] = __builtin_bswap32(__builtin_amdgcn_alignbyte(lo.z, lo.y, 2));
    w[1] = __builtin_bswap32(__builtin_amdgcn_alignbyte(lo.w, lo.z, 2));
    w[2] = __builtin_bswap32(__builtin_amdgcn_alignbyte(hi0, lo.w, 2));
    w[3] = __builtin_bswap32(__builtin_amdgcn_alignbyte(hi1, hi0, 2));
}

// Payload words 4 lane .. 4 lane + 3, host order, loaded.  With 16-byte aligned
// rows (`wide`) lane l loads the aligned chunk holding payload bytes 16 l - 6 ..
// 16 l + 9 in ONE dwordx4 and takes bytes 16 l + 10 .. 16 l + 15 from lane l+1's
// chunk (lane 63 reads those six bytes, still inside the frame, as two dwords).
// The 2-byte-load fallback takes eight loads per lane.  Call in uniform control flow.
__device__ __forceinline__ void payload16(const uint8_t* fr, uint32_t wf, int lane, bool wide, uint32_t (&w)[4])
{
    if (wide) {
        const u4* c = reinterpret_cast<const u4*>(fr) + (3 + wf);
        const u4 a = c[lane];
        uint32_t n0 = (uint32_t)__shfl_down((int)a.x, 1, kWave), n1 = (uint32_t)__shfl_down((int)a.y, 1, kWave);
        if (lane == kWave - 1) {
            const uint32_t* t = reinterpret_cast<const uint32_t*>(c + kWave);
            n0 = t[0];
            n1 = t[1];
        }
        payload_from_chunks(a, n0, n1, w);
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = payload_word(fr, wf, 4 * lane + j);
    }
}

__device__ __forceinline__ void put16(uint8_t* p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

// Header image of child c's egress frames (util.c:348-388) with opcode and PSN
// left zero: identical for every frame of that child and kind, so each block
// builds the 3*fan_in images once into LDS and frames copy them word-wise.
// Kinds: data (PACKET_TYPE_DATA), RETH (PACKET_TYPE_RETH) and ACK
// (PACKET_TYPE_ACK: opcode 0x11 in the image, PSN and AETH left zero).
constexpr int kHdrImg = 80;   // 70 header bytes (with RETH slot), rows 16-byte aligned (read as 16-byte chunks)
constexpr int kImgReth = 1, kImgAck = 2;   // (kind 0: data)
constexpr int kAckLen = 14 + 20 + 8 + 12 + 4 + 4;   // 62 B: headers, AETH, ICRC (util.c:341-343)

__device__ void build_header_image(uint32_t (&w)[kHdrImg / 4], const InccFrameTemplate& h, int kind)
{
    // built in registers (every index a constant once unrolled), stored as words
    uint8_t fr[kHdrImg];
    const int total = kind == kImgAck ? kAckLen : 14 + 20 + 8 + 12 + (kind == kImgReth ? 16 : 0) + kLanes * 4 + 4;   // util.c:341-345
#pragma unroll
    for (int i = 0; i < kHdrImg; ++i) fr[i] = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {                                    // util.c:348-351
        fr[i] = h.dst_mac[i];
        fr[6 + i] = h.src_mac[i];
    }
    fr[12] = 0x08; fr[13] = 0x00;
    uint8_t* ip = fr + 14;                                           // util.c:354-364
    ip[0] = 0x45; ip[1] = 0x00;
    put16(ip + 2, (uint32_t)(total - 14));
    ip[4] = 0x11; ip[5] = 0x11;
    put16(ip + 6, 0x4000);
    ip[8] = 0x40; ip[9] = 0x11;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        ip[12 + i] = (uint8_t)(h.src_ip >> (8 * i));                 // stored as-is (network order value)
        ip[16 + i] = (uint8_t)(h.dst_ip >> (8 * i));
    }
    uint32_t sum = 0;                                                // util.c:106-127
#pragma unroll
    for (int i = 0; i < 20; i += 2) sum += ((uint32_t)ip[i] << 8) | ip[i + 1];
    while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
    put16(ip + 10, (~sum) & 0xFFFF);
    uint8_t* udp = ip + 20;                                          // util.c:367-372
    put16(udp + 0, h.src_port);
    put16(udp + 2, h.dst_port);
    put16(udp + 4, (uint32_t)(total - 14 - 20));
    uint8_t* bth = udp + 8;                                          // util.c:376-388
    bth[0] = kind == kImgAck ? 0x11 : 0x00;                          // util.c:377-380
    bth[2] = 0xFF; bth[3] = 0xFF;
    const uint32_t q = h.qp & 0x00FFFFFFu;
    bth[4] = (uint8_t)(q >> 24); bth[5] = (uint8_t)(q >> 16); bth[6] = (uint8_t)(q >> 8); bth[7] = (uint8_t)q;
#pragma unroll
    for (int i = 0; i < kHdrImg / 4; ++i)
        w[i] = (uint32_t)fr[4 * i] | ((uint32_t)fr[4 * i + 1] << 8) | ((uint32_t)fr[4 * i + 2] << 16) |
               ((uint32_t)fr[4 * i + 3] << 24);
}

// Egress ICRC by linearity.  The raw CRC (init 0, no final XOR) of a message
// of fixed length is linear over GF(2) in its bytes, so an egress frame's ICRC
// message -- [4 x 0xFF][masked IP .. BTH (.. RETH)][1024-B payload], L =
// doff + 1014 bytes -- splits into parts computed at different rates:
//   P   the payload (shared by every child of an input frame): 64 lanes x 16 B,
//       each lane's segment CRC (32 nibble lookups) shifted past the segments
//       after it (Z_{16 (63 - lane)}, 8 lookups), XOR over the wave -- once per
//       input frame, from registers;
//   H_c the header with opcode, PSN and RETH zeroed: constant per (child,
//       RETH flag), computed once per block at start-up;
//   V   opcode + PSN (5 bytes, shared by the children) and each child's RETH
//       (16 bytes): one table lookup pair per byte from tables that hold each
//       byte position's contribution already shifted to the message end.
// ICRC = ~(P ^ V_op,psn ^ H_c ^ V_reth,c): the per-child CRC work is one RETH
// reduction (RETH frames only), not a pass over the 1 KiB frame.
constexpr int kVarBytes = 21;   // opcode, 4 PSN bytes, 16 RETH bytes
__device__ uint32_t g_lane16[8][16][kWave];            // [nibble][value][lane] = Z_{16 (63 - lane)}(value << 4 nibble)
__device__ uint32_t g_var[5 + kVarBytes][2][16];     // [var_row(reth, byte)][nibble][value]: contribution at the message end
__device__ uint32_t g_z1024[8][16];                   // Z_1024(value << 4 nibble)
// The ACK's ICRC message is frame bytes 10-57 (48 B, no payload): its variable
// bytes are the PSN (frame 51-53) and the AETH (54-57, util.c:391-395)
constexpr int kAckVar = 7, kAckMsg = 48;
__device__ uint32_t g_ackvar[kAckVar][2][16];       // [byte 51 + k][nibble][value]: contribution at the message end

// variable-byte rows: a RETH-less frame's 5 (opcode, PSN) at rows 0-4, a RETH
// frame's 21 (opcode, PSN, RETH) at rows 5-25
constexpr int kVarRows = 5 + kVarBytes;
__device__ __forceinline__ constexpr int var_row(int wf, int k) { return wf ? 5 + k : k; }

__device__ __forceinline__ uint32_t wave_xor(uint32_t c)
{
    // the DPP XOR-reduction of icrc_wave: lane 63 ends with the whole wave's XOR
    c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0xB1, 0xF, 0xF, false);
    c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x4E, 0xF, 0xF, false);
    c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x141, 0xF, 0xF, false);
    c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x140, 0xF, 0xF, false);
    c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x142, 0xA, 0xF, false);
    c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x143, 0xC, 0xF, false);
    return (uint32_t)__builtin_amdgcn_readlane((int)c, 63);
}

// a variable byte's ICRC term (k: 0 opcode, 1-4 PSN, 5-20 RETH), already shifted to the message end
template <class L>
__device__ __forceinline__ uint32_t var_crc(const L& t, int wf, int k, uint32_t b)
{
    return t.var[var_row(wf, k)][0][b & 15u] ^ t.var[var_row(wf, k)][1][(b >> 4) & 15u];
}

// ---------------------------------------------------------------------------
// Ingress (nts.c:303-483, root branch) reproduces the reference's one-frame-at-
// a-time order: frame index within the batch = arrival order.  What a serial
// switch decides for frame f depends on which copies of its (psn, port) and of
// its PSN's other ports came BEFORE f, so:
//   claim   (a lane per frame) parse + validate; per (slot, port) an atomicMin
//           of a batch-tagged frame index finds the first copy in the batch
//   classify + sum   the first copy of a pair whose port bit was not set
//           before the batch is the arrival that counts: it adds its payload
//           (nts.c:359-363) and keeps its RETH (:442).  The PSN completes at the LAST of
//           its ports' counted arrivals (the max over ports of the first index;
//           ports already in before the batch count as earlier than every
//           frame): that frame is COMPLETED (:365-372), the others ABSORBED.
//           Every other copy is a retransmit (:353): REPLAY if the slot completed
//           before the batch or at an earlier frame of it (:354-356), else
//           DROPPED.
// Batch generation: claim tags its first-copy keys with g = gen[0] + 1 and
// publishes g in gen[1]; classify reads g from gen[1] and stores it to gen[0]
// for the next batch.  Each word is written while no kernel of the batch reads it,
// and nothing changes on the host per batch, so a captured batch (hipGraph)
// tags every replay anew.
// ---------------------------------------------------------------------------
// claim -> classify: a data frame still to classify: kActPending | WRITE_FIRST << 9 |
// opcode (the final actions are all below 0x100; classify replaces the word,
// and the same bit then marks a leader for the sum, kActLeader)
constexpr int kActPending = 0x100;
constexpr int kClaimBlock = 256;

// (~gen << 32) | (frame << 1) | wf: the minimum over a (slot, port)'s keys is the
// newest batch's earliest copy (the frame index dominates bit 0), and bit 0 tells
// classify and the sum where that copy's payload starts (byte 54, or 70 after a RETH) without
// another dependent load.  Frame indices stay below 2^31.
__device__ __forceinline__ uint64_t first_key(uint32_t gen, int64_t f, bool wf)
{
    return ((uint64_t)(~gen) << 32) | ((uint64_t)(uint32_t)f << 1) | (wf ? 1u : 0u);
}

__global__ __launch_bounds__(kClaimBlock) void k_ingress_claim(InccSwitchState s, const uint8_t* __restrict__ frames,
                                                               int64_t stride, int64_t count,
                                                               const int32_t* __restrict__ ports,
                                                               int32_t* __restrict__ action,
                                                               uint32_t* __restrict__ psn_out)
{
    const uint32_t g = *s.gen + 1u;   // this batch's generation
    if (blockIdx.x == 0 && threadIdx.x == 0) s.gen[1] = g;
    const int64_t f = (int64_t)blockIdx.x * kClaimBlock + threadIdx.x;
    if (f >= count) return;
    // rows are 4-byte aligned and at least 64 bytes: the header fields from four
    // dword loads (bytes 36-43 and 48-55 of the row) instead of byte loads
    const uint32_t* fw = reinterpret_cast<const uint32_t*>(frames + f * stride);
    // (all five loads issued before the first use, one wait: through opaque
    // copies, since the compiler would otherwise sink some into the branches
    // below and wait for them one after another)
    const uint32_t w9 = opaque_u32(fw[9]), w10 = opaque_u32(fw[10]), w12 = opaque_u32(fw[12]);
    const uint32_t w13 = opaque_u32(fw[13]);
    const int port = (int)opaque_u32((uint32_t)ports[f]);
    const uint8_t op = (uint8_t)(w10 >> 16);                                    // byte 42
    const uint32_t psn = ((w12 >> 24) << 16) | ((w13 & 0xFFu) << 8) | ((w13 >> 8) & 0xFFu);   // bytes 51-53, nts.c:311
    const int udp_len = (int)(((w9 >> 16) & 0xFFu) << 8 | (w9 >> 24));          // bytes 38-39
    int act = INCCL_SW_IGNORED;
    if (port < 0 || port >= s.fan_in) act = INCCL_SW_INVALID;
    else if (op == 0x11) act = INCCL_SW_ACK;                    // nts.c:336-342, :403-406 (reflect)
    else if (is_data_opcode(op) || is_write_first(op)) {
        const bool wf = is_write_first(op);
        const int data_len = udp_len - 12 - 8 - 4 - (wf ? 16 : 0);   // nts.c:349, :429
        // nts.c:350 asserts the length; the payload must also lie inside the row
        if (data_len != kLanes * 4 || 54 + (wf ? 16 : 0) + kLanes * 4 > stride) act = INCCL_SW_INVALID;
        else {
            const uint32_t slot = psn & (s.slots - 1);
            // (the slot's degree counts this arrival in k_ingress_sum)
            atomicMin(reinterpret_cast<unsigned long long*>(&s.first[(size_t)slot * s.fan_in + port]),
                      (unsigned long long)first_key(g, f, wf));
            act = kActPending | (wf ? 0x200 : 0) | op;
        }
    }
    action[f] = act;
    psn_out[f] = psn;
}

// ---------------------------------------------------------------------------
// Classify + sum (after claim).
//
// Arrival bitmap: every frame classifies against the bitmap as it was before
// the batch, while the PSN's leader writes the new one in the same launch.  A
// slot holds two 64-bit words {bits, tag = the batch that wrote them}.  Batch g
// reads the newer of the words whose tag is not g (arrival_before), and its
// leader overwrites the OTHER word -- the one arrival_before did not select --
// with tag g.  The selected word is then never touched during batch g, so a
// reader gets the pre-batch bitmap whether it loads before or after the
// leader's store (64-bit accesses are single-copy atomic; after the store the
// overwritten word carries tag g and is skipped).  Overwriting a fixed word
// (say g & 1) would be wrong: when the slot's last arrivals came in batch g - 2
// and none in g - 1, word g & 1 IS the pre-batch bitmap, and a reader after the
// store would fall back to the older word.  The recycle writes both words (no
// frame of the batch reads that slot).
// ---------------------------------------------------------------------------
constexpr int kApplyWaves = 8;    // the sum kernel: 8-wave blocks (1, 2, 4, 16: 35.1-36.4 us, no better)
// consecutive frames per sum wave.  Groups of 4 read a fan-in-2 PSN's copies
// from registers even with an ACK between them (ACK batch: sum 40.8-42.0 us
// against 56.6-57.2) but cost 2.2 us on data-only batches (37.5-37.7 against
// 35.2-35.5): not kept (profiles/r05/switch/sum_variants.txt)
constexpr int kSumGroup = 2;

struct ApplyArgs {
    InccSwitchState s;
    const uint8_t* frames;
    int64_t stride, count;
    const int32_t* ports;
    int32_t* action;
    const uint32_t* psns;
    int wide;                        // 16-byte aligned rows
};

// which of a slot's two tagged words holds the arrival bitmap as it was before
// batch g (nts.c:59): the newer of those whose tag is not g (0 or 1)
__device__ __forceinline__ uint32_t arrival_sel(uint64_t w0, uint64_t w1, uint32_t g)
{
    const uint32_t t0 = (uint32_t)(w0 >> 32), t1 = (uint32_t)(w1 >> 32);
    const uint32_t d0 = t0 == g ? 0xFFFFFFFFu : g - t0, d1 = t1 == g ? 0xFFFFFFFFu : g - t1;
    return d0 <= d1 ? 0u : 1u;
}

__device__ __forceinline__ uint32_t arrival_before(uint64_t w0, uint64_t w1, uint32_t g)
{
    return arrival_sel(w0, w1, g) ? (uint32_t)w1 : (uint32_t)w0;
}

// A buffer resource over [base, base + bytes) whose fields are wave-uniform by
// construction: a resource the compiler cannot prove uniform is used through a
// readfirstlane "waterfall" loop around every load and store.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, int64_t bytes)
{
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
    const int n = __builtin_amdgcn_readfirstlane((int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}

// A row's payload tail that lane 63 needs past its own chunk (chunk 67, and
// with a RETH the first half of chunk 68), as 8-byte loads on lanes 0-2: lane 0
// chunk 67 dwords 0-1, lane 1 its dwords 2-3, lane 2 chunk 68 dwords 0-1
__device__ __forceinline__ u2 tail_chunks(__amdgpu_buffer_rsrc_t rs, int rb, int lane)
{
    return __builtin_bit_cast(u2, __builtin_amdgcn_raw_buffer_load_b64(rs, lane < 3 ? rb + 1072 + 8 * lane : kOobOffset,
                                                                      0, 0));
}

// lane l + 1's value (lane 63 gets lane 0's), through a precomputed address
__device__ __forceinline__ uint32_t from_next(uint32_t v, int next4)
{
    return (uint32_t)__builtin_amdgcn_ds_bpermute(next4, (int)v);
}

// ---------------------------------------------------------------------------
// The classification in a lane-per-frame kernel, the payload sums in a kernel
// whose waves need one dependent round trip (the per-pair kernel that did both
// waited on three: claim results, then keys and arrival words, then payloads;
// 50.2 us against 5.5 + 34.5 us per 131 072-frame batch, profiles/r04/).
//
// k_ingress_classify, a lane per frame, decides everything but the sums: each
// lane reads its slot's two tagged arrival words and the first-copy keys of
// all fan_in ports, classifies its frame (nts.c:353-372), writes
// a counted WRITE_FIRST copy's RETH into the keeper (:442), and the lane of the
// PSN's leader (the lowest counted port's first copy) writes the slot's new
// arrival word and recycles slot psn + slots/2 on completion (:235-242, :367).
// A leader's action word carries what its sum needs until k_ingress_sum
// rewrites it: kActLeader, kActPartial (the slot held arrivals before the
// batch), kActOwnWf (its own WRITE_FIRST flag), and for fan_in <= 8 the counted
// ports (bits 16-23) and each counted copy's WRITE_FIRST flag (bits 24-31);
// above 8 ports kActKeys: the sum takes the counted ports from the slot's two
// arrival words and each other copy from its key.  Every other frame's action
// is final here.
//
// k_ingress_sum, a wave per two consecutive frames: the rows' payload chunks
// are loaded with the action words, before anything is known (lane l the
// 16-byte chunk 3 + l of each row, lanes 0 and 1 also chunks 67 and 68: the
// payload starts 6 bytes into chunk 3 or 4, whichever the opcode says, so both
// placements are covered); a leader then sums its counted copies -- its own payload, the
// other frame of the pair if that is a counted copy of the PSN (the common
// case: a PSN's ports arriving as consecutive frames), else the copy the key
// names -- and the slot's partial, stores the sum and its final action.
// ---------------------------------------------------------------------------
constexpr int kActLeader = 0x100, kActPartial = 0x200, kActOwnWf = 0x400, kActKeys = 0x800;
constexpr int kClassifyBlock = 256;

__global__ __launch_bounds__(kClassifyBlock) void k_ingress_classify(InccSwitchState s,
                                                                     const uint8_t* __restrict__ frames,
                                                                     int64_t stride, int64_t count,
                                                                     const int32_t* __restrict__ ports,
                                                                     int32_t* __restrict__ action,
                                                                     const uint32_t* __restrict__ psns)
{
    const uint32_t g = s.gen[1];   // this batch's generation (claim's)
    const int64_t f = (int64_t)blockIdx.x * kClassifyBlock + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x == 0) s.gen[0] = g;   // the next batch's claim adds one
    if (f >= count) return;
    // round trip 1: the claim results; round trip 2: the slot's arrival words,
    // the first-copy keys (fan_in <= 8 at once) and, for a WRITE_FIRST frame,
    // its RETH (frame bytes 54-69, 4-byte aligned row) before it is known to count
    const int act = (int)opaque_u32((uint32_t)action[f]);
    const int port = (int)opaque_u32((uint32_t)ports[f]);
    const uint32_t psn = opaque_u32(psns[f]);
    if (!(act & kActPending)) return;   // ACK, INVALID, IGNORED: final at claim
    const int fan = s.fan_in;
    const uint32_t slot = psn & (s.slots - 1), wf = ((uint32_t)act >> 9) & 1u;
    const uint32_t tag = ~g, result_bit = 1u << fan;
    const uint64_t a0 = s.arrival[2 * (size_t)slot], a1 = s.arrival[2 * (size_t)slot + 1];
    constexpr int kKeys = 8;
    uint64_t key[kKeys];
#pragma unroll
    for (int p = 0; p < kKeys; ++p) key[p] = p < fan ? s.first[(size_t)slot * fan + p] : 0ull;
    uint32_t rw[5] = {0u, 0u, 0u, 0u, 0u};
    if (wf) {
        const uint32_t* fw = reinterpret_cast<const uint32_t*>(frames + f * stride);
#pragma unroll
        for (int j = 0; j < 5; ++j) rw[j] = fw[13 + j];
    }
    const uint32_t sel = arrival_sel(opaque64(a0), opaque64(a1), g);
    const uint32_t pre = (uint32_t)(sel ? a1 : a0);
    // the PSN's ports: which count in this batch (first copy, not in before),
    // when each counts (1 + frame index; 0 = before the batch, ~0 = not yet)
    uint32_t cports = 0, wfs = 0, done = 0, mine = 0xFFFFFFFFu;
    auto port_key = [&](int p, uint64_t k) {
        const bool in_batch = (uint32_t)(k >> 32) == tag, before = (pre >> p) & 1u;
        const uint32_t ef = (uint32_t)k >> 1;
        done = max(done, before ? 0u : (in_batch ? ef + 1u : 0xFFFFFFFFu));
        if (in_batch && !before) {
            cports |= 1u << p;
            wfs |= ((uint32_t)k & 1u) << p;
        }
        if (p == port) mine = in_batch ? ef : 0xFFFFFFFFu;
    };
#pragma unroll
    for (int p = 0; p < kKeys; ++p)
        if (p < fan) port_key(p, key[p]);
    for (int p = kKeys; p < fan; ++p) port_key(p, s.first[(size_t)slot * fan + p]);
    const uint32_t fi = (uint32_t)f;
    const bool counted = !((pre >> port) & 1u) && mine == fi;   // nts.c:359-363
    int fin;
    if (counted) {
        fin = done == fi + 1u ? INCCL_SW_COMPLETED : INCCL_SW_ABSORBED;   // nts.c:365
        if (wf) {   // the RETH into the keeper (nts.c:442)
            uint32_t* kp = s.reth + ((size_t)slot * fan + port) * 4;
            kp[0] = __builtin_amdgcn_alignbyte(rw[1], rw[0], 2);
            kp[1] = __builtin_amdgcn_alignbyte(rw[2], rw[1], 2);
            kp[2] = __builtin_amdgcn_alignbyte(rw[3], rw[2], 2);
            kp[3] = __builtin_amdgcn_alignbyte(rw[4], rw[3], 2);
        }
    } else {   // retransmit: nts.c:353-357
        const bool done_before = (pre & result_bit) != 0;
        const bool done_earlier = done != 0u && done != 0xFFFFFFFFu && done - 1u < fi;
        fin = (done_before || done_earlier) ? INCCL_SW_REPLAY : INCCL_SW_DROPPED;
    }
    if (!(counted && port == __builtin_ctz(cports))) {
        action[f] = fin;
        return;
    }
    // the leader: the slot's new arrival word (over the word that does NOT hold
    // the pre-batch bitmap, see above), the recycle, the sum's orders
    const bool complete = done != 0xFFFFFFFFu;
    s.arrival[2 * (size_t)slot + (sel ^ 1u)] =
        ((uint64_t)g << 32) | (pre | cports | (complete ? result_bit : 0u));   // nts.c:359, :366
    if (complete) {   // clear_state_data(psn + WINDOW), nts.c:235-242, :367
        const uint32_t rs = (psn + (s.slots >> 1)) & (s.slots - 1);
        for (int i = 0; i < fan * 4; ++i) s.reth[(size_t)rs * fan * 4 + i] = 0u;
        s.arrival[2 * (size_t)rs] = (uint64_t)g << 32;
        s.arrival[2 * (size_t)rs + 1] = (uint64_t)g << 32;
        s.degree[rs] = 0;
    }
    action[f] = fin | kActLeader | (pre ? kActPartial : 0) | (wf ? kActOwnWf : 0) |
                (fan <= 8 ? (int)((cports << 16) | (wfs << 24)) : kActKeys);
}

// the sum kernel: one group of kSumGroup consecutive frames per wave, short-lived blocks
__global__ __launch_bounds__(kWave* kApplyWaves) void k_ingress_sum(ApplyArgs A, const int32_t* __restrict__ act_in,
                                                                    const int32_t* __restrict__ ports_in,
                                                                    const uint32_t* __restrict__ psns_in)
{
    constexpr int G = kSumGroup;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    const int next4 = ((lane + 1) & (kWave - 1)) * 4;
    const InccSwitchState& s = A.s;
    const int fan = s.fan_in;
    const int64_t count = A.count, stride = A.stride, gidx = (int64_t)blockIdx.x * kApplyWaves + w;
    const int64_t f0 = G * gidx < count ? G * gidx : 0;
    const int nin = G * gidx < count ? (int)(count - f0 < G ? count - f0 : G) : 0;   // frames of the group (0: none)
    // round trip 1: the action words (scalar).  Round trip 2: the payload
    // chunks of the rows that hold a counted copy (lane l chunk 3 + l, and the
    // tail past lane 63's) -- an ACK, retransmit or invalid row gets a
    // zero-size buffer, so its loads move no bytes.  (One round trip with every
    // row loaded speculatively costs the same on data-only batches, 35.1-35.4
    // against 35.2-35.5 us, and reads every ACK row too: 65.3-66.1 against
    // 56.6-57.2 us with an ACK after every data frame;
    // profiles/r05/switch/sum_variants.txt)
    int act[G];
    uint32_t psn[G];
#pragma unroll
    for (int k = 0; k < G; ++k) {
        act[k] = k < nin ? act_in[f0 + k] : 0;
        psn[k] = k < nin ? psns_in[f0 + k] : 0u;
    }
    u4 x[G] = {};
    u2 e[G] = {};
    if (A.wide) {
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int fk = act[k] & 0xFF;
            const bool counted = (act[k] & kActLeader) || fk == INCCL_SW_ABSORBED || fk == INCCL_SW_COMPLETED;
            const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(A.frames + (f0 + k) * stride, counted ? stride : 0);
            x[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, 48 + 16 * lane, 0, 0);
            e[k] = tail_chunks(rs, 0, lane);
        }
    }
    // every data frame's arrival into its slot's degree (nts.c:351 / :431,
    // retransmits included), as the wave's last memory instructions: atomics
    // issued before a wait would be waited for with it
    auto degrees = [&]() {
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int a = act[k] & 0xFF;
            if (k < nin && a >= INCCL_SW_ABSORBED && a <= INCCL_SW_REPLAY && lane == 0)
                atomicAdd(&s.degree[psn[k] & (s.slots - 1)], 1);
        }
    };
    int any = 0;
#pragma unroll
    for (int k = 0; k < G; ++k) any |= act[k];
    if (!(any & kActLeader)) {
        degrees();
        return;
    }
    int port[G];
#pragma unroll
    for (int k = 0; k < G; ++k) port[k] = k < nin ? ports_in[f0 + k] : -1;
    // payload words 4 lane .. 4 lane + 3 of a row, from its chunks: xx = chunk
    // 3 + lane, ee = chunks 67, 68 on lanes 0, 1 (payload at byte 54 + 16 wf)
    // (ee: the tail chunks' dwords, tail_chunks: lane 0 chunk 67 dwords 0-1,
    // lane 1 its dwords 2-3, lane 2 chunk 68 dwords 0-1)
    auto extract = [&](const u4& xx, const u2& ee, uint32_t wf, uint32_t (&P)[4]) {
        const bool last = lane == kWave - 1;
        uint32_t y0 = from_next(xx.x, next4), y1 = from_next(xx.y, next4);
        y0 = last ? (uint32_t)__builtin_amdgcn_readlane((int)ee.x, 0) : y0;
        y1 = last ? (uint32_t)__builtin_amdgcn_readlane((int)ee.y, 0) : y1;
        if (wf) {
            uint32_t y2 = from_next(xx.z, next4), y3 = from_next(xx.w, next4);
            uint32_t z0 = from_next(y0, next4), z1 = from_next(y1, next4);
            y2 = last ? (uint32_t)__builtin_amdgcn_readlane((int)ee.x, 1) : y2;
            y3 = last ? (uint32_t)__builtin_amdgcn_readlane((int)ee.y, 1) : y3;
            z0 = last ? (uint32_t)__builtin_amdgcn_readlane((int)ee.x, 2) : z0;
            z1 = last ? (uint32_t)__builtin_amdgcn_readlane((int)ee.y, 2) : z1;
            payload_from_chunks(u4{y0, y1, y2, y3}, z0, z1, P);
        } else {
            payload_from_chunks(xx, y0, y1, P);
        }
    };
    auto payload_of = [&](int k, uint32_t wf, uint32_t (&P)[4]) {
        if (A.wide) extract(x[k], e[k], wf, P);
        else payload16(A.frames + (f0 + k) * stride, wf, lane, false, P);
    };
    auto add = [](u4& acc, const uint32_t (&q)[4]) {
        acc.x += q[0];
        acc.y += q[1];
        acc.z += q[2];
        acc.w += q[3];
    };
    const uint32_t g = s.gen[0];   // this batch's generation (classify stored it)
#pragma unroll
    for (int k = 0; k < G; ++k) {
        if (!(act[k] & kActLeader)) continue;
        const uint32_t slot = psn[k] & (s.slots - 1);
        const bool keys = (act[k] & kActKeys) != 0;
        uint32_t cports, wfs;
        if (!keys) {
            cports = ((uint32_t)act[k] >> 16) & 0xFFu;
            wfs = (uint32_t)act[k] >> 24;
        } else {   // fan_in > 8: the counted ports are the new arrival word's bits that the old one lacks
            const uint64_t w0 = s.arrival[2 * (size_t)slot], w1 = s.arrival[2 * (size_t)slot + 1];
            const uint32_t now = (uint32_t)((uint32_t)(w0 >> 32) == g ? w0 : w1);
            cports = now & ~arrival_before(w0, w1, g) & ((1u << fan) - 1u);
            wfs = 0;   // unused: every port but the leader's own is read through its key
        }
        const uint32_t own_wf = (act[k] & kActOwnWf) ? 1u : 0u;
        u4 acc = {0u, 0u, 0u, 0u};
        if (act[k] & kActPartial) acc = reinterpret_cast<const u4*>(s.agg + (size_t)slot * kLanes)[lane];
        uint32_t rest = cports, q[4];
        // the leader's own copy and every counted copy of this PSN among the
        // group's other frames: already in registers (a PSN's ports arriving
        // close together, with or without an ACK between them, is the common
        // case).  A counted copy is the only frame of its (psn, port) whose
        // action is ABSORBED or COMPLETED.
        if ((rest >> port[k]) & 1u) {
            payload_of(k, own_wf, q);
            add(acc, q);
            rest &= ~(1u << port[k]);
        }
#pragma unroll
        for (int o = 0; o < G; ++o) {
            if (o == k || keys || o >= nin) continue;
            const int fo = act[o] & 0xFF;
            // (a counted copy's port is one of the switch's: the shift is in range)
            if ((fo == INCCL_SW_ABSORBED || fo == INCCL_SW_COMPLETED) && psn[o] == psn[k] &&
                ((rest >> (port[o] & 31)) & 1u)) {
                payload_of(o, (wfs >> port[o]) & 1u, q);
                add(acc, q);
                rest &= ~(1u << port[o]);
            }
        }
        // every other counted copy, two at a time: both keys in one round
        // trip, both rows' chunks in the next (not two round trips per copy)
        while (rest) {
            const int pa = __builtin_ctz(rest);
            rest &= rest - 1;
            const int pb = rest ? __builtin_ctz(rest) : pa;
            const bool two = rest != 0;
            rest &= rest - 1;
            const uint64_t ka = s.first[(size_t)slot * fan + pa], kb = s.first[(size_t)slot * fan + pb];
            // a counted port's key is this batch's (tag ~g) by construction; any
            // other key's frame index would name a row of an earlier batch --
            // possibly past this one's end -- so it is never read
            const bool va = (uint32_t)(ka >> 32) == ~g, vb = two && (uint32_t)(kb >> 32) == ~g;
            const uint32_t fa = va ? (uint32_t)ka >> 1 : 0u, fb = vb ? (uint32_t)kb >> 1 : 0u;
            if (A.wide) {
                const __amdgpu_buffer_rsrc_t ra = uniform_rsrc(A.frames + (int64_t)fa * stride, va ? stride : 0);
                const __amdgpu_buffer_rsrc_t rb = uniform_rsrc(A.frames + (int64_t)fb * stride, vb ? stride : 0);
                const u4 xa = __builtin_amdgcn_raw_buffer_load_b128(ra, 48 + 16 * lane, 0, 0);
                const u2 ea = tail_chunks(ra, 0, lane);
                const u4 xb = __builtin_amdgcn_raw_buffer_load_b128(rb, 48 + 16 * lane, 0, 0);
                const u2 eb = tail_chunks(rb, 0, lane);
                extract(xa, ea, (uint32_t)ka & 1u, q);
                add(acc, q);
                if (two) {
                    extract(xb, eb, (uint32_t)kb & 1u, q);
                    add(acc, q);
                }
            } else {
                if (va) {
                    payload16(A.frames + (int64_t)fa * stride, (uint32_t)ka & 1u, lane, false, q);
                    add(acc, q);
                }
                if (vb) {
                    payload16(A.frames + (int64_t)fb * stride, (uint32_t)kb & 1u, lane, false, q);
                    add(acc, q);
                }
            }
        }
        // write-through (sc1): the sum goes to memory and stays in the caches
        // for egress, which reads it next (49.7-50.0 vs 51.8-52.1 us for egress
        // against non-temporal stores; the sum kernel itself unchanged,
        // profiles/r04/switch/agg_store_policy.txt)
        __builtin_amdgcn_raw_buffer_store_b128(acc, uniform_rsrc(s.agg + (size_t)slot * kLanes, kLanes * 4), 16 * lane, 0,
                                               kAuxSc1);
        if (lane == 0) A.action[f0 + k] = act[k] & 0xFF;
    }
    degrees();
}

// ---------------------------------------------------------------------------
// Non-root ingress (nts.c:376-400, :408-423, :457-499: `root` false).  A
// non-root decides a frame from everything before it in its slot -- the
// degree test of a resend (:382, :463) counts every earlier copy -- so each
// slot's frames of the batch are put in arrival order and taken through the
// reference's branches one at a time, by one lane:
//   k_nr_claim     a lane per frame: parse + validate as the root's claim, the
//                  parent on port fan_in; each data frame pushed onto its slot's
//                  list (atomicExch on the slot's head: the frame that found the
//                  list empty owns the slot for the batch)
//   k_nr_classify  a lane per owner: the slot's frames in index order through
//                  UP first copy / resend / replay and DOWN taken / ignored,
//                  the RETH keeper (:470), bitmap and degree, the recycle
//                  (INCCL_SW_RECYCLE); the slot's work record: which frames'
//                  payloads count
//   k_nr_sum       a wave per work item: the counted payloads added to the
//                  aggregate (:390-392, :472-474) and the parent's result into
//                  res (:413, :489)
// A slot holds few frames of a batch (a copy per child, a resend or two, the
// parent's): its owner keeps up to kNrList of them in its own LDS row (not a
// register array: per-lane indices would make every access a waterfall) and
// sorts them; a longer list is walked once per frame (same result, slower).
// Every index read from the lists is checked against the batch's frame count,
// so a list can never send a lane outside the batch.
// ---------------------------------------------------------------------------
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kNrList = 8;
// work records go to kNrShards regions, classify block b into region b % kNrShards,
// each region with its own counter (work[0 .. kNrShards-1]): one counter for
// all serialised the waves' atomics at one L2 channel (28 us per 131 072-frame
// batch, 2 048 atomics)
constexpr int kNrShards = 64;
__host__ __device__ constexpr uint32_t nr_region_cap(int64_t count)
{
    return (uint32_t)((((count + kClassifyBlock - 1) / kClassifyBlock) + kNrShards - 1) / kNrShards) * kClassifyBlock;
}

// A run of consecutive frames of one slot in a wave (a PSN's copies arriving
// together, the common case) is pushed with ONE atomicExch by its last frame:
// each frame links to the frame before it and the run's first frame to what
// the exchange returned (an atomic per frame, two to one address for a fan-in-2
// PSN: 12.6 us per 131 072-frame batch).
__global__ __launch_bounds__(kClaimBlock) void k_nr_claim(InccSwitchState s, const uint8_t* __restrict__ frames,
                                                          int64_t stride, int64_t count,
                                                          const int32_t* __restrict__ ports,
                                                          int32_t* __restrict__ action, uint32_t* __restrict__ psn_out)
{
    if (blockIdx.x == 0 && threadIdx.x < kNrShards) s.work[threadIdx.x] = 0u;   // classify (the next launch) appends
    const int64_t f = (int64_t)blockIdx.x * kClaimBlock + threadIdx.x;
    const bool in = f < count;
    const int64_t fr = in ? f : 0;   // (every lane stays for the wave-wide steps below)
    const uint32_t* fw = reinterpret_cast<const uint32_t*>(frames + fr * stride);
    const uint32_t w9 = opaque_u32(fw[9]), w10 = opaque_u32(fw[10]), w12 = opaque_u32(fw[12]);
    const uint32_t w13 = opaque_u32(fw[13]);
    const int port = (int)opaque_u32((uint32_t)ports[fr]);
    const uint8_t op = (uint8_t)(w10 >> 16);                                    // byte 42
    const uint32_t psn = ((w12 >> 24) << 16) | ((w13 & 0xFFu) << 8) | ((w13 >> 8) & 0xFFu);   // nts.c:311
    const int udp_len = (int)(((w9 >> 16) & 0xFFu) << 8 | (w9 >> 24));
    const bool wf = is_write_first(op);
    int act = INCCL_SW_IGNORED;
    if (port < 0 || port > s.fan_in) act = INCCL_SW_INVALID;
    else if (op == 0x11) act = port < s.fan_in ? INCCL_SW_ACK : INCCL_SW_IGNORED;   // UP_ACK / DOWN_ACK (:424-426)
    else if (is_data_opcode(op) || wf) {
        const int data_len = udp_len - 12 - 8 - 4 - (wf ? 16 : 0);   // nts.c:349, :410, :429, :486
        act = (data_len != kLanes * 4 || 54 + (wf ? 16 : 0) + kLanes * 4 > stride) ? INCCL_SW_INVALID : kActPending;
    }
    const bool linked = in && act == kActPending;
    const uint32_t slot = psn & (s.slots - 1);
    const int lane = threadIdx.x % kWave;
    const uint32_t pslot = (uint32_t)__shfl_up((int)slot, 1, kWave), nslot = (uint32_t)__shfl_down((int)slot, 1, kWave);
    const uint64_t lk = __ballot(linked);
    const bool same_prev = linked && lane > 0 && ((lk >> (lane - 1)) & 1u) && pslot == slot;
    const bool same_next = linked && lane < kWave - 1 && ((lk >> (lane + 1)) & 1u) && nslot == slot;
    const uint64_t ends = __ballot(linked && !same_next) >> lane;
    const int end_lane = ends ? lane + __builtin_ctzll(ends) : lane;   // this frame's run's last frame
    uint32_t old = kNone;
    if (linked && !same_next) old = atomicExch(&s.head[slot], (uint32_t)f);
    const uint32_t run_next = (uint32_t)__shfl((int)old, end_lane, kWave);
    if (linked)
        reinterpret_cast<u2*>(s.link)[f] = u2{same_prev ? (uint32_t)f - 1u : run_next, (uint32_t)port | (wf ? 1u << 8 : 0u)};
    if (in) {
        action[f] = act;
        psn_out[f] = psn;
    }
}

__global__ __launch_bounds__(kClassifyBlock) void k_nr_classify(InccSwitchState s, const uint8_t* __restrict__ frames,
                                                                int64_t stride, int64_t count,
                                                                int32_t* __restrict__ action,
                                                                const uint32_t* __restrict__ psns)
{
    const int64_t f = (int64_t)blockIdx.x * kClassifyBlock + threadIdx.x;
    if (f >= count) return;
    const u2* link = reinterpret_cast<const u2*>(s.link);
    // one round trip: the claim result, the frame's own link, its PSN
    const int a = (int)opaque_u32((uint32_t)action[f]);
    const u2 own = link[f];
    const uint32_t psn = opaque_u32(psns[f]);
    if (a != kActPending || own.x != kNone) return;   // owners only (next = none)
    const uint32_t slot = psn & (s.slots - 1);
    const uint32_t h0 = s.head[slot];
    uint32_t B = s.bits[slot], D = (uint32_t)s.degree[slot], downf = kNone;   // (loaded while the list is walked)
    s.head[slot] = kNone;   // empty for the next batch
    // the slot's work record for the sum: {psn | partial << 31, parent frame,
    // counted frame per child}, in this block's region (the compiler makes the
    // wave's owners one atomic).  Every word is stored inverted, so that the
    // sum's range-checked loads (0 past a record) read kNone
    const int fan = s.fan_in;
    const uint32_t k = blockIdx.x % kNrShards;
    const uint32_t idx = atomicAdd(&s.work[k], 1u);
    uint32_t* rec = s.work + kNrShards + ((size_t)k * nr_region_cap(count) + idx) * (fan + 2);
    // the list: (frame, port | WF << 8) pairs, each hop one 8-byte load; the
    // owner's own entry (the list's end) is already in registers
    __shared__ u2 lds_list[kClassifyBlock][kNrList + 1];   // (+1: lanes' rows spread over the banks)
    u2* L = lds_list[threadIdx.x];
    const uint32_t nfr = (uint32_t)count;
    int n = 0;
    for (uint32_t g = h0; g < nfr;) {
        const u2 e = g == (uint32_t)f ? own : link[g];
        if (n < kNrList) L[n] = u2{g, e.y};
        ++n;
        g = e.x;
    }
    const bool kept = n <= kNrList;
    if (kept)
        for (int i = 1; i < n; ++i)   // insertion sort: arrival order
            for (int j = i; j > 0 && L[j - 1].x > L[j].x; --j) {
                const u2 t = L[j];
                L[j] = L[j - 1];
                L[j - 1] = t;
            }
    const uint32_t cmask = 0xFFFFFFFFu >> (32 - fan), rbit = 1u << fan;   // nts.c:29, :366
    const bool partial = (B & cmask) != 0u;
    uint32_t* cnt = rec + 2;
    for (int q = 0; q < fan; ++q) cnt[q] = ~kNone;
    int64_t prev = -1;
    for (int i = 0; i < n; ++i) {
        uint32_t g = kNone, info = 0u;
        if (kept) {
            g = L[i].x;
            info = L[i].y;
        } else {   // the earliest frame after the previous one
            for (uint32_t h = h0; h < nfr;) {
                const u2 e = link[h];
                if ((int64_t)h > prev && h < g) {
                    g = h;
                    info = e.y;
                }
                h = e.x;
            }
        }
        if (g >= nfr) break;
        prev = g;
        const uint32_t port = info & 0xFFu, wf = (info >> 8) & 1u;
        int act;
        if ((int)port < fan) {
            D += 1u;   // nts.c:351, :431
            const uint32_t pb = 1u << port;
            if (B & pb)   // resend (:377-385, :458-466)
                act = (B & rbit) ? INCCL_SW_REPLAY
                                 : (((B & cmask) == cmask && D % (uint32_t)fan == 0u) ? INCCL_SW_FORWARD
                                                                                         : INCCL_SW_DROPPED);
            else {   // first transmission (:387-398, :468-480)
                B |= pb;
                cnt[port] = ~(g | (wf << 31));
                if (wf) {   // the RETH into the keeper (:470): frame bytes 54-69
                    const uint32_t* fw = reinterpret_cast<const uint32_t*>(frames + (int64_t)g * stride);
                    uint32_t rw[5];
#pragma unroll
                    for (int j = 0; j < 5; ++j) rw[j] = fw[13 + j];
                    uint32_t* kp = s.reth + ((size_t)slot * fan + port) * 4;
#pragma unroll
                    for (int j = 0; j < 4; ++j) kp[j] = __builtin_amdgcn_alignbyte(rw[j + 1], rw[j], 2);
                }
                act = (B & cmask) == cmask ? INCCL_SW_FORWARD : INCCL_SW_ABSORBED;
            }
        } else if (!(B & rbit) && (B & cmask) == cmask) {   // the parent's result, taken once (:412-419)
            B |= rbit;
            downf = g | (wf << 31);
            act = INCCL_SW_DOWN;
            if (s.flags & INCCL_SW_RECYCLE) {   // clear_state_data(psn + WINDOW) as at the root (:235-242)
                const uint32_t rs = (psn + (s.slots >> 1)) & (s.slots - 1);
                for (int j = 0; j < fan * 4; ++j) s.reth[(size_t)rs * fan * 4 + j] = 0u;
                s.bits[rs] = 0u;
                s.degree[rs] = 0;
            }
        } else {
            act = INCCL_SW_DROPPED;   // :420-422
        }
        action[g] = act;
    }
    s.bits[slot] = B;
    s.degree[slot] = (int32_t)D;
    rec[0] = ~((psn & 0x00FFFFFFu) | (partial ? 1u << 31 : 0u));
    rec[1] = ~downf;
}

constexpr int kNrSumWaves = 4;
constexpr int kNrSumRows = 2;   // rows whose payload chunks a wave has in flight at once

// Payload words 4 lane .. 4 lane + 3 of a row (host order) from its 16-byte
// chunks: xx = chunk 3 + lane, ee = the tail chunks lane 63 needs
// (tail_chunks); the payload starts 6 bytes into chunk 3 + wf (as k_ingress_sum)
__device__ __forceinline__ void chunks_payload(const u4& xx, const u2& ee, uint32_t wf, int lane, int next4,
                                               uint32_t (&P)[4])
{
    const bool last = lane == kWave - 1;
    uint32_t y0 = from_next(xx.x, next4), y1 = from_next(xx.y, next4);
    y0 = last ? (uint32_t)__builtin_amdgcn_readlane((int)ee.x, 0) : y0;
    y1 = last ? (uint32_t)__builtin_amdgcn_readlane((int)ee.y, 0) : y1;
    if (wf) {
        uint32_t y2 = from_next(xx.z, next4), y3 = from_next(xx.w, next4);
        uint32_t z0 = from_next(y0, next4), z1 = from_next(y1, next4);
        y2 = last ? (uint32_t)__builtin_amdgcn_readlane((int)ee.x, 1) : y2;
        y3 = last ? (uint32_t)__builtin_amdgcn_readlane((int)ee.y, 1) : y3;
        z0 = last ? (uint32_t)__builtin_amdgcn_readlane((int)ee.x, 2) : z0;
        z1 = last ? (uint32_t)__builtin_amdgcn_readlane((int)ee.y, 2) : z1;
        payload_from_chunks(u4{y0, y1, y2, y3}, z0, z1, P);
    } else {
        payload_from_chunks(xx, y0, y1, P);
    }
}

// A wave per two work records at a time (lane j: word j of each), the next two
// in flight while they are summed: each record's rows' payload chunks
// kNrSumRows at a time (the children's counted copies, then the parent's
// result) with the slot's partial, the second record's rows loading while the
// first's are added.  A wave waits on one payload round trip per pair, not per
// record.
//
// The waits are counts (vmcnt), so every memory instruction of the common
// path is issued unconditionally: range-checked buffer accesses at an
// out-of-range offset where there is nothing to load or store (a conditional
// one makes the compiler wait for everything, vmcnt(0)).  The loop is entered
// with as many (dropped) stores after the first records' loads as a pass
// issues after its prefetch, its four stores.
constexpr int kNrSumTail = 4;

template <bool kWide>
__global__ __launch_bounds__(kWave* kNrSumWaves) void k_nr_sum(InccSwitchState s, const uint8_t* __restrict__ frames,
                                                              int64_t stride, int64_t count)
{
    const int lane = threadIdx.x % kWave, fan = s.fan_in;
    const int next4 = ((lane + 1) & (kWave - 1)) * 4;
    // wave w takes region w % kNrShards, its records w / kNrShards, + nw / kNrShards, ...
    const uint32_t wid = blockIdx.x * kNrSumWaves + threadIdx.x / kWave;
    const uint32_t k = wid % kNrShards, nw = gridDim.x * kNrSumWaves / kNrShards, nfr = (uint32_t)count;
    const uint32_t n = s.work[k];
    const bool wire = (s.flags & INCCL_SW_WIRE_ORDER) != 0;
    const int rw = fan + 2;   // record words
    const __amdgpu_buffer_rsrc_t rrec =
        uniform_rsrc(s.work + kNrShards + (size_t)k * nr_region_cap(count) * rw, (int64_t)n * rw * 4);
    // record i's word `lane`, inverted as classify stored it (past the region's
    // n records or the record's rw words: 0, i.e. kNone once inverted back)
    auto rec = [&](uint32_t i) {
        return __builtin_amdgcn_raw_buffer_load_b32(rrec, lane < rw ? (int)((i * (uint32_t)rw + (uint32_t)lane) * 4u)
                                                                    : kOobOffset,
                                                    0, 0);
    };
    struct Rec {
        uint32_t cq, d;
        uint64_t m;   // counted rows left (record lanes)
        bool down;    // the parent's row left
        bool any, has_down;
        __amdgpu_buffer_rsrc_t ragg, rres;
        u4 acc, vres;
    };
    struct Rows {
        uint32_t row[kNrSumRows];
        int kind[kNrSumRows];   // 0 none, 1 a child's counted copy, 2 the parent's result
        u4 x[kNrSumRows];
        u2 e[kNrSumRows];
    };
    // a record (a past-the-end one is all kNone: no rows, both stores dropped)
    auto open = [&](uint32_t rn) {
        Rec R;
        R.cq = ~rn;
        const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)R.cq, 0), slot = w & (s.slots - 1);
        R.d = (uint32_t)__builtin_amdgcn_readlane((int)R.cq, 1);
        R.ragg = uniform_rsrc(s.agg + (size_t)slot * kLanes, kLanes * 4);
        R.rres = uniform_rsrc(s.res + (size_t)slot * kLanes, kLanes * 4);
        R.m = __ballot(lane >= 2 && lane < rw && (R.cq & 0x7FFFFFFFu) < nfr);
        R.any = R.m != 0;
        // the partial, or 0 -- and not read at all without a counted row (a
        // down batch's records: the aggregate is neither summed nor stored)
        R.acc = __builtin_amdgcn_raw_buffer_load_b128(R.ragg, ((w >> 31) && R.any) ? 16 * lane : kOobOffset, 0, 0);
        R.vres = u4{0u, 0u, 0u, 0u};
        R.has_down = (R.d & 0x7FFFFFFFu) < nfr;
        R.down = R.has_down;
        return R;
    };
    // the record's next kNrSumRows rows, their loads issued (16-byte rows)
    auto take = [&](Rec& R) {
        Rows L;
#pragma unroll
        for (int r = 0; r < kNrSumRows; ++r) {
            if (R.m) {
                L.row[r] = (uint32_t)__builtin_amdgcn_readlane((int)R.cq, __builtin_ctzll(R.m));
                R.m &= R.m - 1;
                L.kind[r] = 1;
            } else if (R.down) {
                L.row[r] = R.d;
                R.down = false;
                L.kind[r] = 2;
            } else {
                L.row[r] = 0u;
                L.kind[r] = 0;
            }
            if (kWide) {
                const __amdgpu_buffer_rsrc_t rs =
                    uniform_rsrc(frames + (int64_t)(L.row[r] & 0x7FFFFFFFu) * stride, L.kind[r] ? stride : 0);
                L.x[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, 48 + 16 * lane, 0, 0);
                L.e[r] = tail_chunks(rs, 0, lane);
            }
        }
        return L;
    };
    auto add = [&](Rec& R, const Rows& L) {
        uint32_t P[kNrSumRows][4];
#pragma unroll
        for (int r = 0; r < kNrSumRows; ++r) {
            if (kWide)
                chunks_payload(L.x[r], L.e[r], L.row[r] >> 31, lane, next4, P[r]);
            else if (L.kind[r])
                payload16(frames + (int64_t)(L.row[r] & 0x7FFFFFFFu) * stride, L.row[r] >> 31, lane, false, P[r]);
            else
                P[r][0] = P[r][1] = P[r][2] = P[r][3] = 0u;
            if (L.kind[r] == 1) {
                R.acc.x += P[r][0];
                R.acc.y += P[r][1];
                R.acc.z += P[r][2];
                R.acc.w += P[r][3];
            } else if (L.kind[r] == 2) {
                // the reference keeps the wire bytes (memcpy, :413): the host words back to wire order
                R.vres = wire ? u4{P[r][0], P[r][1], P[r][2], P[r][3]}
                              : u4{__builtin_bswap32(P[r][0]), __builtin_bswap32(P[r][1]),
                                   __builtin_bswap32(P[r][2]), __builtin_bswap32(P[r][3])};
            }
        }
    };
    // the rest of its rows (fan_in > kNrSumRows, resends), then the aggregate and
    // the parent's result, write-through as the root's sum: egress reads them next
    auto close = [&](Rec& R) {
        while (R.m || R.down) {
            const Rows L = take(R);
            add(R, L);
        }
        __builtin_amdgcn_raw_buffer_store_b128(R.acc, R.ragg, R.any ? 16 * lane : kOobOffset, 0, kAuxSc1);
        __builtin_amdgcn_raw_buffer_store_b128(R.vres, R.rres, R.has_down ? 16 * lane : kOobOffset, 0, kAuxSc1);
    };
    uint32_t i = wid / kNrShards;
    uint32_t rn0 = rec(i), rn1 = rec(i + nw);
    {
        const __amdgpu_buffer_rsrc_t none = uniform_rsrc(s.agg, 0);
#pragma unroll
        for (int j = 0; j < kNrSumTail; ++j)   // (1 KiB apart: separate instructions, not one merged store)
            __builtin_amdgcn_raw_buffer_store_b32(0u, none, 1024 * j, 0, 0);
    }
    for (; i < n; i += 2 * nw) {
        Rec A = open(rn0), B = open(rn1);
        rn0 = rec(i + 2 * nw);
        rn1 = rec(i + 3 * nw);
        const Rows LA = take(A), LB = take(B);
        add(A, LA);
        close(A);
        add(B, LB);
        close(B);
    }
}

// ---------------------------------------------------------------------------
// Egress (nts.c:365-372 / :447-453 broadcast, :353-356 / :435-438 replay;
// frames per util.c:331-442): every output frame of input frame f, rows
// f * fan_in + c -- all fan_in children on COMPLETED, the sender's child on
// REPLAY -- from the slot's aggregate and RETH keeper as ingress left them.
//
// Persistent 16-wave blocks, two per CU: each block loads the CRC tables into
// LDS and builds the 2 fan_in header images and their ICRC terms H_c once.  A
// wave then takes egress_chunk(fan_in) consecutive input frames at a time (a chunk),
// lane l frame l: their claim results and header words in four vector loads,
// the row lengths of all its frames' fan_in rows lane-parallel, and then
// only the frames that emit, one after another, each frame's aggregate and
// keeper in flight while the frame before it is built, and the wave's next
// chunk's claim results in flight while this chunk is built.  (A wave per input
// frame spent as long on the absorbed half of the frames, which emit nothing,
// as on the rest: 58-60 against 56-57 us per 131 072-frame batch.  Chunks of
// 16 / 8 / 4 / 2 frames with the next chunk read ahead: 49.9 / 47.1-47.6 /
// 45.4-45.6 / 50.8 us, profiles/r04/switch/egress_chunk_sweep.txt.)
//
// Loads and stores retire in order on one counter (vmcnt).  So that the
// compiler can wait for the prefetched aggregate without also waiting for the
// stores issued after it, every emitted frame issues the same memory
// instructions: the children loop unrolled for a fixed fan-in (2, 3, 4, 8),
// every load and store unconditional -- a frame that emits nothing, or a child
// that gets no frame, is given a zero-size buffer (its loads return 0, its
// stores are dropped, neither reaches memory) -- and all CRC work in branches
// without memory instructions.  Two register sets take alternate frames (a
// copy between them would wait for the load in flight).
//
// The payload goes from registers to the rows: lane l holds payload bytes
// [16 l, 16 l + 16) (htonl of the aggregate, util.c:403-405 / :419-421), frame
// bytes doff + 16 l ..; doff (54, or 70 with a RETH) is 6 mod 16, so 16-byte
// output chunk doff / 16 + 1 + l is lane l's bytes 10-15 then lane l + 1's
// bytes 0-9: built once per input frame, stored once per child.  Lane 63's
// chunk ends the frame: payload bytes 1018-1023, the ICRC (host order), two
// bytes of zero padding.  The header chunks are the child's template image
// (LDS) ORed with one patch per input frame (opcode, PSN, the payload's first
// 10 bytes) and, with a RETH, the child's 16 RETH bytes.  The ICRC is
// ~(P ^ V_op,psn ^ H_c ^ V_reth,c) (above): one payload reduction per input
// frame, one RETH reduction per RETH child.
// ---------------------------------------------------------------------------
constexpr int kEgressWaves = 16;
// input frames per wave at a time: 4 up to fan-in 8; 16 above, where most
// chunks of 4 would hold no completing frame (fan-in 16: 48.3 us with 4, 43.0
// with 16; fan-in 5: 29.2 with 4, 32.3 with 16)
__host__ __device__ constexpr uint32_t egress_chunk(int fan)
{
    return fan <= 8 ? 4u : 16u;
}
constexpr int kEgressAhead = 1;    // emitting frames whose aggregate is in flight ahead of the one emitted

__device__ uint32_t g_segb[16][256];   // [byte j of a 16-byte segment][value] = Z_{15-j}(T[value])

struct EgressLds {
    uint32_t segb[16][256];
    uint32_t lane16[8][16][kWave];
    uint32_t var[kVarRows][2][16];
    uint32_t z1024[8][16];
    uint32_t ackvar[kAckVar][2][16];
    uint32_t hcrc[3 * 32];                                  // H_c: [2 c + RETH flag] data, [2 dests + c] ACK
    __attribute__((aligned(16))) uint8_t img[3 * 32][kHdrImg];
};

// The raw CRC of 16 bytes (a[]: memory order, little-endian words) as 16 byte
// lookups, shifted past the (63 - sh_lane) 16-byte segments after it
// (Z_{16 (63 - sh_lane)}) as 8 nibble lookups.
__device__ __forceinline__ uint32_t seg16(const EgressLds& t, const uint32_t (&a)[4], int sh_lane)
{
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t v0 = t.segb[4 * j][a[j] & 0xFFu], v1 = t.segb[4 * j + 1][(a[j] >> 8) & 0xFFu];
        const uint32_t v2 = t.segb[4 * j + 2][(a[j] >> 16) & 0xFFu], v3 = t.segb[4 * j + 3][a[j] >> 24];
        c = xor3(c, v0, v1) ^ xor3(v2, v3, 0u);
        c = opaque_u32(c);   // four lookups in flight at a time: registers for the occupancy
    }
    const uint32_t clo = opaque_u32(c & 0x0F0F0F0Fu), chi = opaque_u32((c >> 4) & 0x0F0F0F0Fu);
    uint32_t s[8];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        s[2 * b] = t.lane16[2 * b][(uint8_t)(clo >> (8 * b))][sh_lane];
        s[2 * b + 1] = t.lane16[2 * b + 1][(uint8_t)(chi >> (8 * b))][sh_lane];
    }
    return xor3(xor3(s[0], s[1], s[2]), xor3(s[3], s[4], s[5]), s[6]) ^ s[7];
}

// The tables, the 3 `fan` header images (fan: the destinations, fan_in
// children and a non-root's parent) and their ICRC terms H_c into the
// block's LDS (ends with a block barrier).  H_c: quad i of the block takes
// image i; the header part of the ICRC message (doff - 10 bytes: 44, or 60
// with a RETH; an ACK's whole 48-byte message) is right-aligned in a 64-byte
// window (leading zeros do not change a raw CRC), lane q of the quad takes
// window bytes 16 q .. 16 q + 15, and the quad's XOR of a data image is
// shifted past the 1024-byte payload.
__device__ void egress_setup(EgressLds& t, const InccFrameTemplate* __restrict__ tmpl, int fan)
{
    // the tables as 16-byte words, every thread's loads issued before its
    // stores (one round trip, not one per word); blocks of kEgressWaves waves
    static_assert(kWave * kEgressWaves == 1024, "the copy below assumes 1024-thread blocks");
    const int x = threadIdx.x;
    const u4* gs = reinterpret_cast<const u4*>(&g_segb[0][0]);       // 1024 words
    const u4* gl = reinterpret_cast<const u4*>(&g_lane16[0][0][0]);  // 2048
    const u4* gv = reinterpret_cast<const u4*>(&g_var[0][0][0]);     // kVarRows * 8
    const u4* gz = reinterpret_cast<const u4*>(&g_z1024[0][0]);      // 32
    const u4 s0 = gs[x], l0 = gl[x], l1 = gl[x + 1024];
    const u4* ga = reinterpret_cast<const u4*>(&g_ackvar[0][0][0]);  // kAckVar * 8
    const u4 v0 = x < kVarRows * 8 ? gv[x] : u4{}, z0 = x < 32 ? gz[x] : u4{};
    const u4 av = x < kAckVar * 8 ? ga[x] : u4{};
    uint32_t img[kHdrImg / 4];
    if (x < 3 * fan) build_header_image(img, tmpl[x < 2 * fan ? x >> 1 : x - 2 * fan], x < 2 * fan ? (x & 1) : kImgAck);
    reinterpret_cast<u4*>(&t.segb[0][0])[x] = s0;
    reinterpret_cast<u4*>(&t.lane16[0][0][0])[x] = l0;
    reinterpret_cast<u4*>(&t.lane16[0][0][0])[x + 1024] = l1;
    if (x < kVarRows * 8) reinterpret_cast<u4*>(&t.var[0][0][0])[x] = v0;
    if (x < 32) reinterpret_cast<u4*>(&t.z1024[0][0])[x] = z0;
    if (x < kAckVar * 8) reinterpret_cast<u4*>(&t.ackvar[0][0][0])[x] = av;
    if (x < 3 * fan) {
#pragma unroll
        for (int k = 0; k < kHdrImg / 16; ++k)
            reinterpret_cast<u4*>(t.img[x])[k] = u4{img[4 * k], img[4 * k + 1], img[4 * k + 2], img[4 * k + 3]};
    }
    __syncthreads();
    const int i = threadIdx.x >> 2, q = threadIdx.x & 3;
    uint32_t c = 0;
    if (i < 3 * fan) {
        const int hdr = i >= 2 * fan ? kAckMsg : (i & 1) ? 60 : 44;
        uint32_t a[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int p = 16 * q + 4 * k + b - (64 - hdr);   // header byte; frame byte p + 10
                uint32_t byte = 0;
                if (p >= 0) {
                    const int fo = p + 10;
                    bool ff = fo < 14;                             // the 4 x 0xFF CRC prefix (util.c:262)
#pragma unroll
                    for (int m = 4; m < kNumMasked; ++m) ff = ff || fo == masked_pos(m);   // util.c:266-270
                    byte = ff ? 0xFFu : t.img[i][fo];
                }
                v |= byte << (8 * b);
            }
            a[k] = v;
        }
        c = seg16(t, a, kWave - 4 + q);
    }
    c ^= (uint32_t)__shfl_xor((int)c, 1, kWave);
    c ^= (uint32_t)__shfl_xor((int)c, 2, kWave);
    uint32_t r = 0;
#pragma unroll
    for (int n = 0; n < 8; ++n) r ^= t.z1024[n][(c >> (4 * n)) & 15u];
    if (i >= 2 * fan) r = c;   // an ACK has no payload after its header
    if (i < 3 * fan && q == 0) t.hcrc[i] = r;
    __syncthreads();
}

// What egress reads and writes (the kernel argument; 32-bit frame indices:
// count < 2^31).
struct EgressArgs {
    const int32_t* agg;
    const int32_t* res;   // a non-root's parent results (the DOWN / REPLAY payloads)
    const uint32_t* reth;
    const uint8_t* frames;
    const int32_t* ports;
    const int32_t* action;
    const uint32_t* psns;
    const InccFrameTemplate* tmpl;
    uint8_t* out;
    int32_t* out_len;
    uint32_t stride, out_stride, count, smask;
    int fan;
    int dests;            // rows per input frame: fan, and a non-root's parent row fan
};

// One input frame as an egress wave knows it: three wave-uniform words
struct EgressF {
    uint32_t f, psn;
    uint32_t bits;   // opcode | WRITE_FIRST << 8 | in << 9 | all << 10 | one << 11 | res << 14 | port << 16
    __device__ uint32_t op() const { return bits & 0xFFu; }
    __device__ uint32_t wf() const { return (bits >> 8) & 1u; }
    __device__ bool in() const { return (bits >> 9) & 1u; }     // f < count
    __device__ bool all() const { return (bits >> 10) & 1u; }   // COMPLETED: every child
    __device__ bool one() const { return (bits >> 11) & 1u; }   // REPLAY: child port(); FORWARD: port() = fan_in
    __device__ bool res() const { return (bits >> 14) & 1u; }   // the payload from res (a non-root's DOWN, REPLAY)
    __device__ uint32_t port() const { return bits >> 16; }
};

// the slot's aggregate (this lane's four words) and RETH keeper (lane 4 c + j:
// word j of child c's, c < 16); nothing for a frame that emits nothing
__device__ __forceinline__ void egress_load(const EgressArgs& A, const EgressF& e, int lane, u4& acc, uint32_t& keep)
{
    const bool em = e.all() || e.one();
    const uint32_t slot = e.psn & A.smask;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int32_t*>(e.res() ? A.res : A.agg) + (size_t)slot * kLanes, 0, em ? kLanes * 4 : 0, 0x00020000);
    acc = __builtin_amdgcn_raw_buffer_load_b128(ra, 16 * lane, 0, 0);
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t*>(A.reth) + (size_t)slot * A.fan * 4, 0, em && e.wf() ? 16 * A.fan : 0, 0x00020000);
    keep = __builtin_amdgcn_raw_buffer_load_b32(rk, 4 * lane, 0, 0);
}

// Frame e's output rows (their lengths are stored per chunk, k_egress).
template <int kFan, bool kOut16, bool kNR>
__device__ __forceinline__ void egress_emit(const EgressLds& t, const EgressArgs& A, const EgressF& e, const u4& acc,
                                            uint32_t keep, int lane)
{
    const int fan = kFan ? kFan : A.fan, dests = fan + (kNR ? 1 : 0);
    const uint32_t wf = e.wf(), op = e.op(), port = e.port();
    const bool all = e.all(), one = e.one();
    const bool em_any = all || one;
    const bool last = lane == kWave - 1;
    // (a frame that emits nothing stores nowhere: its values are left undefined)
    uint32_t pc = unset(), p0 = unset(), p1 = unset(), p2 = unset(), p3 = unset();
    u4 patch = unset4();
    if (em_any) {
        uint32_t a[4];   // this lane's 16 payload bytes, big-endian (util.c:403-405), memory order
        a[0] = __builtin_bswap32(acc.x);
        a[1] = __builtin_bswap32(acc.y);
        a[2] = __builtin_bswap32(acc.z);
        a[3] = __builtin_bswap32(acc.w);
        const uint32_t pw = e.psn | 0x80000000u;   // ack-request bit + PSN (util.c:386)
        // P ^ V_op,psn: the payload segment's term, and on lanes 0-4 the opcode's
        // and the PSN bytes' (util.c:378, :386)
        const uint32_t vb = lane == 0 ? op : (pw >> (8 * (4 - lane))) & 0xFFu;
        const uint32_t var = lane < 5 ? var_crc(t, (int)wf, lane, vb) : 0u;
        pc = wave_xor(seg16(t, a, lane) ^ var);
        const int next4 = ((lane + 1) & (kWave - 1)) * 4;
        const uint32_t n0 = from_next(a[0], next4), n1 = from_next(a[1], next4), n2 = from_next(a[2], next4);
        p0 = __builtin_amdgcn_alignbyte(a[3], a[2], 2);
        p1 = last ? a[3] >> 16 : __builtin_amdgcn_alignbyte(n0, a[3], 2);
        p2 = last ? 0u : __builtin_amdgcn_alignbyte(n1, n0, 2);
        p3 = last ? 0u : __builtin_amdgcn_alignbyte(n2, n1, 2);
        // the header chunks' patch over the template images (zeros there):
        // opcode (byte 42), PSN (50-53), and the payload's first 10 bytes after
        // the BTH (no RETH) or after the RETH (lane 4's chunk)
        const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)a[0], 0);
        const uint32_t a1 = (uint32_t)__builtin_amdgcn_readlane((int)a[1], 0);
        const uint32_t a2 = (uint32_t)__builtin_amdgcn_readlane((int)a[2], 0);
        const uint32_t psn_hi = (pw >> 24) | (((pw >> 16) & 0xFFu) << 8);    // frame bytes 50, 51
        const uint32_t psn_lo = ((pw >> 8) & 0xFFu) | ((pw & 0xFFu) << 8);   // bytes 52, 53
        const uint32_t q1 = a0 << 16, q2 = __builtin_amdgcn_alignbyte(a1, a0, 2);
        const uint32_t q3 = __builtin_amdgcn_alignbyte(a2, a1, 2);
        const int pl = wf ? 4 : 3;   // the lane whose chunk ends with the payload's first 10 bytes
        patch.x = lane == 3 ? psn_hi << 16 : 0u;
        patch.y = (lane == 3 ? psn_lo : 0u) | (lane == pl ? q1 : 0u);
        patch.z = lane == pl ? q2 : (lane == 2 ? op << 16 : 0u);
        patch.w = lane == pl ? q3 : 0u;
    }
    const int hchunks = 4 + (int)wf;   // header + the payload's first 10 bytes
    const int ho = lane < hchunks ? 16 * lane : kOobOffset, po = 16 * (hchunks + lane);
    // 16-byte rows: a row is two stores, chunks 0-63 (lane l: chunk l) and
    // 64-67 or 64-68 (lanes 0-3 or 0-4), so that every 64-byte write request
    // but the row's last is whole (header and payload as separate stores split
    // the request at the header's end: 19 requests per row against 17).  Lane
    // l then carries payload chunk l - hchunks (mod 64), the payload rotated
    // by hchunks lanes, once per input frame; the chunk that ends the frame
    // (the ICRC's) lands on lane hchunks - 1 of the second store.
    u4 pr = unset4();
    if (kOut16 && em_any) {
        const int from = ((lane - hchunks) & (kWave - 1)) * 4;
        pr.x = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)p0);
        pr.y = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)p1);
        pr.z = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)p2);
        pr.w = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)p3);
    }
    const bool tail = lane == hchunks - 1;   // the frame's last chunk, in the second store
    // fan row slots per frame: "all" fills them with rows 0 .. fan-1, "one" puts
    // its single row (port; a non-root's parent row fan_in included) in the
    // first and drops the rest.  So a non-root issues fan rows' stores, not
    // fan + 1, and the count stays fixed (k_egress's waits are counts)
    uint8_t* const row0 = A.out + (size_t)e.f * dests * A.out_stride;
    constexpr int kUnroll = kFan ? kFan : 1;
#pragma unroll kUnroll
    for (int i = 0; i < fan; ++i) {
        const int c = one ? (int)port : i;
        const bool em = all || (one && i == 0);
        u4 h = unset4(), v = unset4();
        if (em) {
            h = reinterpret_cast<const u4*>(t.img[2 * c + wf])[lane < 5 ? lane : 0];
            h.x |= patch.x;
            h.y |= patch.y;
            h.z |= patch.z;
            h.w |= patch.w;
            uint32_t crc = pc ^ t.hcrc[2 * c + wf];
            if (wf) {
                // child c's RETH (reth_keeper[slot][c], nts.c:442; util.c:409-417):
                // bytes 54-69, lane 3's chunk from byte 6 on and lane 4's first 6
                // bytes; its ICRC term on lanes 0-15.  A non-root's parent gets a
                // zeroed RETH (send_roce_data_with_reth(FAN_IN, NULL), :464, :478):
                // keep's lanes past the children's 4 fan_in words read as zero
                uint32_t R[4];
                if (kFan || c < kWave / 4) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) R[j] = (uint32_t)__builtin_amdgcn_readlane((int)keep, 4 * c + j);
                } else if (kNR && c == fan) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) R[j] = 0u;
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j) R[j] = A.reth[((size_t)(e.psn & A.smask) * fan + c) * 4 + j];
                }
                if (lane == 3) {
                    h.y |= R[0] << 16;
                    h.z = __builtin_amdgcn_alignbyte(R[1], R[0], 2);
                    h.w = __builtin_amdgcn_alignbyte(R[2], R[1], 2);
                }
                if (lane == 4) {
                    h.x = __builtin_amdgcn_alignbyte(R[3], R[2], 2);
                    h.y |= R[3] >> 16;
                }
                const uint32_t rk = (lane & 8) ? ((lane & 4) ? R[3] : R[2]) : ((lane & 4) ? R[1] : R[0]);
                crc ^= wave_xor(lane < 16 ? var_crc(t, 1, 5 + lane, (rk >> (8 * (lane & 3))) & 0xFFu) : 0u);
            }
            crc = ~crc;   // util.c:424-426
            if (kOut16) {
                v = u4{pr.x, tail ? pr.y | (crc << 16) : pr.y, tail ? crc >> 16 : pr.z, pr.w};
                h = lane < hchunks ? h : pr;
            } else {
                v = u4{p0, last ? p1 | (crc << 16) : p1, last ? crc >> 16 : p2, p3};
            }
        }
        const __amdgpu_buffer_rsrc_t orow =
            __builtin_amdgcn_make_buffer_rsrc(row0 + (size_t)c * A.out_stride, 0, em ? (int)A.out_stride : 0, 0x00020000);
        if (kOut16) {
            __builtin_amdgcn_raw_buffer_store_b128(h, orow, 16 * lane, 0, kAuxNt);
            __builtin_amdgcn_raw_buffer_store_b128(v, orow, lane < hchunks ? 16 * (kWave + lane) : kOobOffset, 0,
                                                   kAuxNt);
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(h.x, orow, ho, 0, kAuxNt);
            __builtin_amdgcn_raw_buffer_store_b32(h.y, orow, ho + 4, 0, kAuxNt);
            __builtin_amdgcn_raw_buffer_store_b32(h.z, orow, ho + 8, 0, kAuxNt);
            __builtin_amdgcn_raw_buffer_store_b32(h.w, orow, ho + 12, 0, kAuxNt);
            __builtin_amdgcn_raw_buffer_store_b32(v.x, orow, po, 0, kAuxNt);
            __builtin_amdgcn_raw_buffer_store_b32(v.y, orow, po + 4, 0, kAuxNt);
            __builtin_amdgcn_raw_buffer_store_b32(v.z, orow, po + 8, 0, kAuxNt);
            // lane 63 stops at the frame's 4-byte-rounded end
            __builtin_amdgcn_raw_buffer_store_b32(v.w, orow, last ? kOobOffset : po + 12, 0, kAuxNt);
        }
    }
}

// ACK reflection (nts.c:403-406; send_roce_ack :284-298, a PACKET_TYPE_ACK
// frame per util.c:331-442): every ACK input frame j of a chunk (its claim
// result INCCL_SW_ACK, bit 12 of its lane's `bits`) sends one 62-B frame back
// to its own port, row (f0 + j) fan_in + port: the port's ACK image (opcode
// 0x11) with the PSN (bytes 51-53, no ack-request bit) and the AETH
// htonl((psn + 1) | 0x1f000000) (54-57) patched in, and the ICRC ~(H_ack,c ^
// the 7 variable bytes' terms).  Lane 4 j + q writes the frame's 16-byte chunk
// q (bytes 62-63 are written as zero).  Per-lane rows: plain global stores
// under the ACK lanes' mask, issued before the chunk's data frames.
template <bool kOut16>
__device__ __forceinline__ void egress_acks(const EgressLds& t, const EgressArgs& A, uint32_t f0, bool ack,
                                            uint32_t bits, uint32_t psn, int fan, int dests, int lane)
{
    if (!__ballot(ack)) return;   // (lane l: frame f0 + l; most chunks hold no ACK)
    const int j = lane >> 2, q = lane & 3;
    const uint32_t bj = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * j, (int)bits);
    const uint32_t pj = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * j, (int)psn) & 0x00FFFFFFu;
    const bool ak = j < (int)egress_chunk(fan) && ((bj >> 12) & 1u);
    if (!ak) return;
    const uint32_t c = bj >> 16, msn = pj + 1u;
    const uint32_t aeth = msn | 0x1f000000u;
    // the variable bytes (frame 51 .. 57): PSN bytes 2..0, AETH bytes 3..0 (big-endian)
    uint32_t crc = t.hcrc[2 * dests + c];
#pragma unroll
    for (int k = 0; k < kAckVar; ++k) {
        const uint32_t b = k < 3 ? (pj >> (8 * (2 - k))) & 0xFFu : (aeth >> (8 * (6 - k))) & 0xFFu;
        crc ^= t.ackvar[k][0][b & 15u] ^ t.ackvar[k][1][b >> 4];
    }
    crc = ~crc;   // util.c:424-426
    u4 v = reinterpret_cast<const u4*>(t.img[2 * dests + c])[q];
    if (q == 3) {   // bytes 48-63: QPN low bytes (image), 0, PSN, AETH, ICRC (host order), 2 zero bytes
        v.x |= ((pj >> 16) & 0xFFu) << 24;
        v.y = ((pj >> 8) & 0xFFu) | ((pj & 0xFFu) << 8) | ((aeth >> 24) << 16) | (((aeth >> 16) & 0xFFu) << 24);
        v.z = ((aeth >> 8) & 0xFFu) | ((aeth & 0xFFu) << 8) | (crc << 16);
        v.w = crc >> 16;
    }
    uint8_t* row = A.out + ((size_t)(f0 + (uint32_t)j) * dests + c) * A.out_stride + 16 * q;
    if (kOut16) {
        *reinterpret_cast<u4*>(row) = v;
    } else {
        uint32_t* w = reinterpret_cast<uint32_t*>(row);
        w[0] = v.x;
        w[1] = v.y;
        w[2] = v.z;
        w[3] = v.w;
    }
}

// kFan: 2, 3, 4 or 8 (the children loop unrolled), or 0 (A.fan, a loop).
// kOut16: 16-byte aligned output rows.  kNR: a non-root switch -- row fan_in
// of each input frame is the parent's; FORWARD sends the aggregate there,
// DOWN sends the parent's result (res) to every child, REPLAY res to one.
template <int kFan, bool kOut16, bool kNR>
__global__ __launch_bounds__(kWave* kEgressWaves) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_egress(
    EgressArgs A)
{
    __shared__ EgressLds t;
    const int fan = kFan ? kFan : A.fan, dests = fan + (kNR ? 1 : 0);
    const uint32_t kEgressChunk = egress_chunk(fan);   // (a constant for the unrolled fan-ins)
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane0 = threadIdx.x % kWave;
    const uint32_t count = A.count, chunks = (count + kEgressChunk - 1) / kEgressChunk;
    const uint32_t nw = gridDim.x * kEgressWaves;
    auto ln = [&]() { return (int)opaque_u32((uint32_t)lane0); };
    // a chunk's claim results and header words (lane l: frame f0 + l; past the
    // end or past count: zero-size reads)
    struct ChunkIn {
        uint32_t act, port, psn, w10;
    };
    auto chunk_in = [&](uint32_t ch) {
        const int lane = ln();
        const uint32_t f0 = ch * kEgressChunk, nf = ch < chunks ? min((uint32_t)kEgressChunk, count - f0) : 0u;
        const int off = lane < (int)nf ? 4 * lane : kOobOffset;
        const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<int32_t*>(A.action) + (ch < chunks ? f0 : 0), 0, 4 * kEgressChunk, 0x00020000);
        const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<int32_t*>(A.ports) + (ch < chunks ? f0 : 0), 0, 4 * kEgressChunk, 0x00020000);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t*>(A.psns) + (ch < chunks ? f0 : 0), 0, 4 * kEgressChunk, 0x00020000);
        const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(A.frames) + (size_t)(ch < chunks ? f0 : 0) * A.stride, 0,
            (int)(kEgressChunk * A.stride), 0x00020000);
        ChunkIn c;
        c.act = __builtin_amdgcn_raw_buffer_load_b32(ra, off, 0, 0);
        c.port = __builtin_amdgcn_raw_buffer_load_b32(rp, off, 0, 0);
        c.psn = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
        c.w10 = __builtin_amdgcn_raw_buffer_load_b32(rf, lane < (int)nf ? lane * (int)A.stride + 40 : kOobOffset, 0, 0);
        return c;
    };
    // the wave's first chunk is read while the block sets up its tables
    uint32_t ch = blockIdx.x * kEgressWaves + w;
    ChunkIn cin = chunk_in(ch);
    egress_setup(t, A.tmpl, dests);
    for (; ch < chunks; ch += nw) {
        const ChunkIn cur = cin;
        cin = chunk_in(ch + nw);   // the wave's next chunk, read while this one is built (past the end: nothing)
        const int lane = ln();
        const uint32_t f0 = ch * kEgressChunk, nf = min((uint32_t)kEgressChunk, count - f0);
        const int act = (int)cur.act;
        const uint32_t port = cur.port, psn = cur.psn;
        const uint32_t op = (cur.w10 >> 16) & 0xFFu;
        const bool in = lane < (int)nf;
        const bool fwd = kNR && in && act == INCCL_SW_FORWARD;
        const bool all = in && act == (kNR ? INCCL_SW_DOWN : INCCL_SW_COMPLETED);
        const bool one = (in && act == INCCL_SW_REPLAY && port < (uint32_t)fan) || fwd;
        const bool ack = in && act == INCCL_SW_ACK && port < (uint32_t)fan;
        const bool res = kNR && in && (act == INCCL_SW_DOWN || act == INCCL_SW_REPLAY);
        const uint32_t bits = op | (is_write_first((uint8_t)op) ? 1u << 8 : 0u) | (in ? 1u << 9 : 0u) |
                              (all ? 1u << 10 : 0u) | (one ? 1u << 11 : 0u) | (ack ? 1u << 12 : 0u) |
                              (res ? 1u << 14 : 0u) | (((fwd ? (uint32_t)fan : port) & 0xFFFFu) << 16);
        {   // the chunk's row lengths: entry e = f dests + c, lane-parallel (util.c:341-345)
            const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
                A.out_len + (size_t)f0 * dests, 0, (int)(4 * nf * dests), 0x00020000);
            for (int k = 0; k < (kEgressChunk * dests + kWave - 1) / kWave; ++k) {
                const int e = lane + kWave * k, fr = e / dests, c = e - fr * dests;
                const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (fr & (kWave - 1)), (int)bits);
                const bool mine = (b >> 16) == (uint32_t)c;
                const bool on = (((b >> 10) & 1u) && c < fan) || (((b >> 11) & 1u) && mine);
                const uint32_t total = 54 + 16 * ((b >> 8) & 1u) + kLanes * 4 + 4;
                const uint32_t len = on ? total : (((b >> 12) & 1u) && mine ? (uint32_t)kAckLen : 0u);
                __builtin_amdgcn_raw_buffer_store_b32(len, rl, 4 * e, 0, 0);
            }
        }
        egress_acks<kOut16>(t, A, f0, ack, bits, psn, fan, dests, lane);
        uint64_t m = __ballot(all || one);
        if (!m) continue;
        // a frame of the ring is its lane in the chunk (-1: none); its words
        // are read from the chunk's registers where used
        auto take = [&]() {
            int b = -1;
            if (m) {
                b = __builtin_ctzll(m);
                m &= m - 1;
            }
            return b;
        };
        auto frame = [&](int b) {
            EgressF e;
            e.f = f0 + (uint32_t)max(b, 0);
            e.psn = b >= 0 ? (uint32_t)__builtin_amdgcn_readlane((int)psn, b) : 0u;
            e.bits = b >= 0 ? (uint32_t)__builtin_amdgcn_readlane((int)bits, b) : 0u;
            return e;
        };
        // a ring of kEgressAhead + 1 frames: a frame's aggregate and keeper are
        // loaded kEgressAhead emitting frames before it is built (deeper rings,
        // 2 and 3, measured no faster: the stores bound this loop)
        constexpr int kR = kEgressAhead + 1;
        int B[kR];
        u4 acc[kR];
        uint32_t keep[kR];
#pragma unroll
        for (int r = 0; r < kEgressAhead; ++r) {
            B[r] = take();
            egress_load(A, frame(B[r]), ln(), acc[r], keep[r]);
        }
        if (kFan) {
            // as many dropped stores as the frames ahead will issue: the loop is
            // entered with its back edge's memory history, so its waits are counts
            const __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(A.out_len, 0, 0, 0x00020000);
#pragma unroll
            for (int k = 0; k < kEgressAhead * kFan * (kOut16 ? 2 : 8); ++k)
                __builtin_amdgcn_raw_buffer_store_b32(0u, none, 16 * k, 0, 0);
        }
        for (;;) {
            bool more = true;
#pragma unroll
            for (int r = 0; r < kR; ++r) {
                const int ld = (r + kEgressAhead) % kR;
                B[ld] = take();
                egress_load(A, frame(B[ld]), ln(), acc[ld], keep[ld]);
                egress_emit<kFan, kOut16, kNR>(t, A, frame(B[r]), acc[r], keep[r], ln());
                more = B[(r + 1) % kR] >= 0;
                if (!more) break;
            }
            if (!more) break;
        }
    }
}

// ---------------------------------------------------------------------------
// host: CRC tables (util.c:141-159) and the zero-append operators
// ---------------------------------------------------------------------------
uint32_t host_tab[256];
uint32_t host_lane16[8][16][kWave];
uint32_t host_seg34[kSeg2][2][16];
uint32_t host_lane_shift32[8][16][32];
uint32_t host_var[5 + kVarBytes][2][16];
uint32_t host_z1024[8][16];
uint32_t host_ackvar[kAckVar][2][16];
uint32_t host_segb[16][256];
bool g_tables_ready[64];
std::mutex g_tables_mu;

uint32_t zeros_append(uint32_t c, int nbytes)
{
    for (int i = 0; i < nbytes; ++i) c = (c >> 8) ^ host_tab[c & 0xFF];
    return c;
}

int ensure_tables()
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return (int)e;
    std::lock_guard<std::mutex> lk(g_tables_mu);
    if (dev >= 0 && dev < 64 && g_tables_ready[dev]) return 0;
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int j = 0; j < 8; ++j) c = (c >> 1) ^ ((c & 1u) ? 0xEDB88320u : 0u);
        host_tab[i] = c;
    }
    // the standalone ICRC (k_icrc): 34-byte segments, Z_{34 (31 - lane')}; Z_n is
    // linear, Z_{n+34}(x) = Z_34(Z_n(x)), so lanes are filled from 31 down
    for (int j = 0; j < kSeg2; ++j)
        for (int h = 0; h < 2; ++h)
            for (uint32_t v = 0; v < 16; ++v) host_seg34[j][h][v] = zeros_append(host_tab[v << (4 * h)], kSeg2 - 1 - j);
    for (int n = 0; n < 8; ++n)
        for (uint32_t v = 0; v < 16; ++v) {
            uint32_t x = v << (4 * n);
            for (int l = 31; l >= 0; --l) {
                host_lane_shift32[n][v][l] = x;
                x = zeros_append(x, kSeg2);
            }
        }
    // egress by linearity: Z_{16 (63 - lane)}, each variable header byte's
    // contribution shifted to the message end, and Z_1024
    for (int n = 0; n < 8; ++n)
        for (uint32_t v = 0; v < 16; ++v) {
            uint32_t x = v << (4 * n);
            host_z1024[n][v] = zeros_append(x, 1024);
            for (int lane = kWave - 1; lane >= 0; --lane) {
                host_lane16[n][v][lane] = x;
                x = zeros_append(x, 16);
            }
        }
    // egress: byte j of a 16-byte segment -> Z_{15-j}(T[value])
    for (int j = 0; j < 16; ++j)
        for (uint32_t v = 0; v < 256; ++v) host_segb[j][v] = zeros_append(host_tab[v], 15 - j);
    for (int wf = 0; wf < 2; ++wf) {
        const int hdr = wf ? 60 : 44;   // ICRC message bytes before the payload (frame 10 .. doff - 1)
        for (int k = 0; k < kVarBytes; ++k) {
            const int p = k == 0 ? 32 : 39 + k;   // message position: opcode (frame 42), PSN (50-53), RETH (54-69)
            for (int h = 0; h < 2; ++h)
                for (uint32_t v = 0; v < 16; ++v)
                    if (wf || k < 5) host_var[wf ? 5 + k : k][h][v] = p < hdr ? zeros_append(host_tab[v << (4 * h)], hdr - 1 - p + 1024) : 0u;
        }
    }
    // the ACK: byte 51 + k of the frame is message byte 41 + k of 48
    for (int k = 0; k < kAckVar; ++k)
        for (int h = 0; h < 2; ++h)
            for (uint32_t v = 0; v < 16; ++v) host_ackvar[k][h][v] = zeros_append(host_tab[v << (4 * h)], kAckMsg - 1 - (41 + k));
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_lane16), host_lane16, sizeof(host_lane16));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_ackvar), host_ackvar, sizeof(host_ackvar));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_var), host_var, sizeof(host_var));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_z1024), host_z1024, sizeof(host_z1024));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_seg34), host_seg34, sizeof(host_seg34));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_lane_shift32), host_lane_shift32, sizeof(host_lane_shift32));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_segb), host_segb, sizeof(host_segb));
    if (e != hipSuccess) return (int)e;
    if (dev >= 0 && dev < 64) g_tables_ready[dev] = true;
    return 0;
}

int num_cus()
{
    static int cus = 0;
    if (cus == 0) {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            cus = v;
        else
            cus = 256;
    }
    return cus;
}

// classify (a lane per frame), then sum (a wave per pair of frames, short-lived blocks)
int launch_apply(const ApplyArgs& a, hipStream_t st)
{
    const dim3 lanes((unsigned)((a.count + kClassifyBlock - 1) / kClassifyBlock));
    hipLaunchKernelGGL(k_ingress_classify, lanes, dim3(kClassifyBlock), 0, st, a.s, a.frames, a.stride, a.count, a.ports,
                       a.action, a.psns);
    const int64_t groups = (a.count + kSumGroup - 1) / kSumGroup, blocks = (groups + kApplyWaves - 1) / kApplyWaves;
    hipLaunchKernelGGL(k_ingress_sum, dim3((unsigned)(blocks < 1 ? 1 : blocks)), dim3(kWave * kApplyWaves), 0, st, a,
                       (const int32_t*)a.action, a.ports, a.psns);
    return (int)hipGetLastError();
}

// persistent egress: a wave per chunk of egress_chunk(fan_in) frames, as many blocks as
// fit beside each other (two per CU)
template <int kFan, bool kOut16, bool kNR>
int launch_egress_t(const EgressArgs& a, hipStream_t st)
{
    static const int per_cu = [] {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_egress<kFan, kOut16, kNR>, kWave * kEgressWaves, 0) !=
                hipSuccess || n < 1)
            n = 1;
        return n;
    }();
    const int64_t chunks = ((int64_t)a.count + egress_chunk(a.fan) - 1) / egress_chunk(a.fan);
    const int64_t need = (chunks + kEgressWaves - 1) / kEgressWaves, cap = (int64_t)num_cus() * per_cu;
    hipLaunchKernelGGL((k_egress<kFan, kOut16, kNR>), dim3((unsigned)(need < cap ? (need < 1 ? 1 : need) : cap)),
                       dim3(kWave * kEgressWaves), 0, st, a);
    return (int)hipGetLastError();
}

template <bool kOut16, bool kNR>
int launch_egress_o(const EgressArgs& a, hipStream_t st)
{
    switch (a.fan) {   // fan-in 2, 3, 4, 8: the children loop unrolled; others a loop
    case 2: return launch_egress_t<2, kOut16, kNR>(a, st);
    case 3: return launch_egress_t<3, kOut16, kNR>(a, st);
    case 4: return launch_egress_t<4, kOut16, kNR>(a, st);
    case 8: return launch_egress_t<8, kOut16, kNR>(a, st);
    default: return launch_egress_t<0, kOut16, kNR>(a, st);
    }
}

int launch_egress(const InccSwitchState* s, const uint8_t* frames, size_t stride, size_t count, const int32_t* ports,
                  const int32_t* action, const uint32_t* psns, const InccFrameTemplate* tmpl, uint8_t* out,
                  size_t out_stride, int32_t* out_len, hipStream_t st)
{
    EgressArgs a{};
    a.agg = s->agg;
    a.res = s->res;
    a.reth = s->reth;
    a.frames = frames;
    a.ports = ports;
    a.action = action;
    a.psns = psns;
    a.tmpl = tmpl;
    a.out = out;
    a.out_len = out_len;
    a.stride = (uint32_t)stride;
    a.out_stride = (uint32_t)out_stride;
    a.count = (uint32_t)count;
    a.smask = s->slots - 1;
    a.fan = s->fan_in;
    a.dests = s->fan_in + (s->nonroot ? 1 : 0);
    const bool o16 = ((out_stride & 15) == 0) && (((uintptr_t)out & 15) == 0);
    if (s->nonroot) return o16 ? launch_egress_o<true, true>(a, st) : launch_egress_o<false, true>(a, st);
    return o16 ? launch_egress_o<true, false>(a, st) : launch_egress_o<false, false>(a, st);
}

int check_batch_args(const InccSwitchState* s, const uint8_t* frames, size_t stride, size_t count, const int32_t* ports,
                     const int32_t* action, const uint32_t* psn_out)
{
    if (!s || !frames || !ports || !action || !psn_out || (stride & 3) || stride < INCCL_FRAME_MIN_STRIDE ||
        ((uintptr_t)frames & 3) || count >= 0x7FFFFFFFull || stride > (1u << 20))
        return INCCL_ERR_ARG;
    return 0;
}

ApplyArgs apply_args(const InccSwitchState* s, const uint8_t* frames, size_t stride, size_t count,
                     const int32_t* ports, int32_t* action, const uint32_t* psn_out)
{
    ApplyArgs a{};
    a.s = *s;
    a.frames = frames;
    a.stride = (int64_t)stride;
    a.count = (int64_t)count;
    a.ports = ports;
    a.action = action;
    a.psns = psn_out;
    // 16-byte aligned rows: payloads as one dwordx4 per lane, loaded speculatively
    a.wide = ((uintptr_t)frames & 15) == 0 && (stride & 15) == 0;
    return a;
}

void launch_claim(const InccSwitchState* s, const uint8_t* frames, size_t stride, size_t count, const int32_t* ports,
                  int32_t* action, uint32_t* psn_out, hipStream_t st)
{
    const dim3 lanes((unsigned)(((int64_t)count + kClaimBlock - 1) / kClaimBlock));
    hipLaunchKernelGGL(k_ingress_claim, lanes, dim3(kClaimBlock), 0, st, *s, frames, (int64_t)stride, (int64_t)count,
                       ports, action, psn_out);
}

// the non-root ingress: claim, classify (a lane per frame, owners only), sum
// (waves over the work list; at most one item per frame)
int launch_nr_ingress(const InccSwitchState* s, const uint8_t* frames, size_t stride, size_t count,
                      const int32_t* ports, int32_t* action, uint32_t* psn_out, hipStream_t st)
{
    const int64_t n = (int64_t)count;
    hipLaunchKernelGGL(k_nr_claim, dim3((unsigned)((n + kClaimBlock - 1) / kClaimBlock)), dim3(kClaimBlock), 0, st, *s,
                       frames, (int64_t)stride, n, ports, action, psn_out);
    hipLaunchKernelGGL(k_nr_classify, dim3((unsigned)((n + kClassifyBlock - 1) / kClassifyBlock)), dim3(kClassifyBlock),
                       0, st, *s, frames, (int64_t)stride, n, action, (const uint32_t*)psn_out);
    const bool wide = ((uintptr_t)frames & 15) == 0 && (stride & 15) == 0;
    // whole groups of kNrShards waves (every region gets the same number of waves)
    constexpr int64_t group = kNrShards / kNrSumWaves;
    const int64_t need = (n + kNrSumWaves - 1) / kNrSumWaves, cap = (int64_t)num_cus() * 8;
    const int64_t blocks = ((need < cap ? need : cap) + group - 1) / group * group;
    if (wide)
        hipLaunchKernelGGL(k_nr_sum<true>, dim3((unsigned)blocks), dim3(kWave * kNrSumWaves), 0, st, *s, frames,
                           (int64_t)stride, n);
    else
        hipLaunchKernelGGL(k_nr_sum<false>, dim3((unsigned)blocks), dim3(kWave * kNrSumWaves), 0, st, *s, frames,
                           (int64_t)stride, n);
    return (int)hipGetLastError();
}

int egress_args_ok(const InccSwitchState* s, const uint8_t* frames, const int32_t* ports, const int32_t* action,
                   const uint32_t* psns, const InccFrameTemplate* tmpl, const uint8_t* out, size_t out_stride,
                   const int32_t* out_len)
{
    return s && frames && ports && action && psns && tmpl && out && out_len && !(out_stride & 3) &&
           out_stride >= 1100 && out_stride <= (1u << 20) && !((uintptr_t)out & 3);
}

}  // namespace

extern "C" {

int inccl_k_frames_init(void) { return ensure_tables(); }

size_t inccl_k_nr_work_words(size_t count, int fan_in)
{
    return kNrShards + (size_t)kNrShards * nr_region_cap((int64_t)count) * (size_t)(fan_in + 2);
}

int inccl_k_icrc(const uint8_t* frames, size_t stride, size_t count, uint32_t* out, void* stream)
{
    if ((frames == nullptr || out == nullptr) && count) return INCCL_ERR_ARG;
    if (count == 0) return 0;
    if ((stride & 3) || stride < INCCL_FRAME_MIN_STRIDE || stride > (1u << 20) || ((uintptr_t)frames & 3))
        return INCCL_ERR_ARG;
    int rc = ensure_tables();
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    // 8-wave blocks, four per CU (20.7 KiB of tables each); the output buffer's
    // byte size is a 32-bit field, so very large counts go in pieces
    const int64_t piece = (int64_t)1 << 28, cap = (int64_t)num_cus() * 4;
    for (int64_t f = 0; f < (int64_t)count; f += piece) {
        const int64_t n = (int64_t)count - f < piece ? (int64_t)count - f : piece;
        const int64_t need = ((n + 1) / 2 + 7) / 8;
        hipLaunchKernelGGL(k_icrc<8>, dim3((unsigned)(need < cap ? need : cap)), dim3(kWave * 8), 0, st,
                           frames + f * (int64_t)stride, (int64_t)stride, n, out + f);
    }
    return (int)hipGetLastError();
}

int inccl_k_switch_ingress(const InccSwitchState* s, const uint8_t* frames, size_t stride, size_t count,
                           const int32_t* ports, int32_t* action, uint32_t* psn_out, void* stream)
{
    if (count == 0) return 0;
    if (check_batch_args(s, frames, stride, count, ports, action, psn_out)) return INCCL_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (s->nonroot) return launch_nr_ingress(s, frames, stride, count, ports, action, psn_out, st);
    launch_claim(s, frames, stride, count, ports, action, psn_out, st);
    return launch_apply(apply_args(s, frames, stride, count, ports, action, psn_out), st);
}

// ingress then egress of one batch: claim, classify, sum, egress on one stream
int inccl_k_switch_batch(const InccSwitchState* s, const uint8_t* frames, size_t stride, size_t count,
                         const int32_t* ports, int32_t* action, uint32_t* psn_out, const InccFrameTemplate* tmpl,
                         uint8_t* out, size_t out_stride, int32_t* out_len, void* stream)
{
    if (count == 0) return 0;
    if (check_batch_args(s, frames, stride, count, ports, action, psn_out) ||
        !egress_args_ok(s, frames, ports, action, psn_out, tmpl, out, out_stride, out_len))
        return INCCL_ERR_ARG;
    int rc = ensure_tables();
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    if (s->nonroot) {
        rc = launch_nr_ingress(s, frames, stride, count, ports, action, psn_out, st);
    } else {
        launch_claim(s, frames, stride, count, ports, action, psn_out, st);
        rc = launch_apply(apply_args(s, frames, stride, count, ports, action, psn_out), st);
    }
    if (rc) return rc;
    return launch_egress(s, frames, stride, count, ports, action, psn_out, tmpl, out, out_stride, out_len, st);
}

int inccl_k_switch_egress(const InccSwitchState* s, const uint8_t* in_frames, size_t in_stride, size_t count,
                          const int32_t* ports, const int32_t* action, const uint32_t* psns,
                          const InccFrameTemplate* tmpl, uint8_t* out, size_t out_stride, int32_t* out_len,
                          void* stream)
{
    if (count == 0) return 0;
    if (!egress_args_ok(s, in_frames, ports, action, psns, tmpl, out, out_stride, out_len) || (in_stride & 3) ||
        in_stride < INCCL_FRAME_MIN_STRIDE || in_stride > (1u << 20) || ((uintptr_t)in_frames & 3) ||
        count >= 0x7FFFFFFFull)
        return INCCL_ERR_ARG;
    int rc = ensure_tables();
    if (rc) return rc;
    return launch_egress(s, in_frames, in_stride, count, ports, action, psns, tmpl, out, out_stride, out_len,
                         (hipStream_t)stream);
}

}  // extern "C"
