// inccl_frames.hip -- the reference's switch dataplane on the GPU (gfx950):
// RoCEv2 frame parse, per-PSN idempotent aggregation, egress frame build and
// the RoCE ICRC (CRC-32).  Reference: repository/src/non_termination_switch.c
// (nts.c) :303-501 for the pipeline and :55-60 / :231-250 for its state;
// repository/src/util.c:331-442 (build_eth_packet), :250-286 (compute_icrc),
// :141-195 (crc32), :106-127 (ipv4_checksum).
//
// A batch of frames (frame index = arrival order) goes through
//   k_ingress_claim   a lane per frame: parse + validate, degree, and the
//                     first copy of every (slot, port) by a batch-tagged atomicMin
//   k_ingress_apply   persistent, a wave per two consecutive frames: classify
//                     in the reference's serial order (nts.c:353-372), sum each
//                     slot's counted arrivals into its aggregate (:361-363), the
//                     arrival bitmap, the RETH keeper (:442), the recycle
//                     (:235-242, :367) -- and in the batch call
//                     (inccl_switch_batch) the broadcast frames of every PSN that
//                     completes (:447-453, util.c:331-442) straight from the
//                     aggregate in registers
//   k_egress_fixed<F> / k_egress   (inccl_switch_egress) every output frame of a
//                     batch from the state ingress left: COMPLETED broadcasts and
//                     REPLAY resends (:353-356)
//   k_replay          (inccl_switch_batch) the REPLAY resends, after apply
// The ICRC is linear over GF(2), so every CRC here is a XOR of table lookups
// (nibble planes, one SDWA byte select per lookup, three-way XORs) reduced over
// the wave with DPP -- no serial byte loop.
//
// State on the GPU (slots = PSN ring size, power of two; the reference uses 16):
//   agg[slots][256] int32        aggregator        (nts.c:55)
//   arrival[slots][2] uint64     port bitmap + bit fan_in = "result known" (nts.c:59, :366),
//                                tagged with the batch that wrote it, double-buffered by
//                                batch parity (k_ingress_apply)
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
constexpr int kSeg = 17;              // egress segment table rows (row j: Z_{16-j})
constexpr int kEgressWaves = 8;       // 512-lane blocks, three per CU, persistent grid
constexpr int kLanes = 256;           // int32 lanes per packet (nts.c:55)
constexpr int kAuxNt = 2;   // buffer instruction cache policy: nt (streaming, not re-read)
constexpr int kOobOffset = 0x7FFFFFF0;   // past any row: a buffer store there is dropped, a load returns 0

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

__device__ uint32_t g_seg[kSeg][2][16];       // [byte j][nibble][value] = Z_{16-j}(T[value << 4 nibble]), T = util.c:141-150

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

// The 16 RETH bytes of the frame at `fr` (bytes 54-69, util.c:409-417) as four
// little-endian words, wave-uniform (2-byte loads: the RETH is 2-byte aligned).
__device__ __forceinline__ void reth_words(const uint8_t* fr, int lane, uint32_t (&r)[4])
{
    const uint16_t* h = reinterpret_cast<const uint16_t*>(fr + 54);
    const uint32_t v = lane < 4 ? ((uint32_t)h[2 * lane] | ((uint32_t)h[2 * lane + 1] << 16)) : 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (uint32_t)__builtin_amdgcn_readlane((int)v, i);
}

__device__ __forceinline__ void put16(uint8_t* p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

// Header image of child c's egress frames (util.c:348-388) with opcode and PSN
// left zero: identical for every frame of that child and RETH flag, so each
// block builds the 2*fan_in images once into LDS and frames copy them word-wise.
constexpr int kHdrImg = 80;   // 70 header bytes (with RETH slot), rows 16-byte aligned (read as 16-byte chunks)

__device__ void build_header_image(uint8_t* fr, const InccFrameTemplate& h, bool wf)
{
    const int total = 14 + 20 + 8 + 12 + (wf ? 16 : 0) + kLanes * 4 + 4;   // util.c:341-345
    for (int i = 0; i < kHdrImg; ++i) fr[i] = 0;
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
    for (int i = 0; i < 4; ++i) {
        ip[12 + i] = (uint8_t)(h.src_ip >> (8 * i));                 // stored as-is (network order value)
        ip[16 + i] = (uint8_t)(h.dst_ip >> (8 * i));
    }
    uint32_t sum = 0;                                                // util.c:106-127
    for (int i = 0; i < 20; i += 2) sum += ((uint32_t)ip[i] << 8) | ip[i + 1];
    while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
    put16(ip + 10, (~sum) & 0xFFFF);
    uint8_t* udp = ip + 20;                                          // util.c:367-372
    put16(udp + 0, h.src_port);
    put16(udp + 2, h.dst_port);
    put16(udp + 4, (uint32_t)(total - 14 - 20));
    uint8_t* bth = udp + 8;                                          // util.c:376-388
    bth[2] = 0xFF; bth[3] = 0xFF;
    const uint32_t q = h.qp & 0x00FFFFFFu;
    bth[4] = (uint8_t)(q >> 24); bth[5] = (uint8_t)(q >> 16); bth[6] = (uint8_t)(q >> 8); bth[7] = (uint8_t)q;
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

// variable-byte rows: a RETH-less frame's 5 (opcode, PSN) at rows 0-4, a RETH
// frame's 21 (opcode, PSN, RETH) at rows 5-25
constexpr int kVarRows = 5 + kVarBytes;
__device__ __forceinline__ constexpr int var_row(int wf, int k) { return wf ? 5 + k : k; }

template <int kImgs>
struct EgressLdsT {
    uint32_t seg[kSeg][2][16];      // g_seg: rows 1..16 are a 16-byte segment's Z_{15-j}
    uint32_t lane16[8][16][kWave];
    uint32_t var[kVarRows][2][16];
    uint32_t z1024[8][16];
    uint32_t hcrc[kImgs];           // H_c for (child, RETH flag)
};
using EgressLds = EgressLdsT<2 * 31>;

// What one egress wave needs from global memory for input frame f: loaded one
// frame ahead of its use (k_egress), so these dependent loads overlap the
// previous frame's build instead of stalling the wave.
struct EgressIn {
    int act, port;
    uint32_t psn, slot;
    uint32_t op;        // bytes 40-43 of the input frame across lanes (opcode: lane 2)
    uint32_t reth;      // lane 4c+i: word i of child c's RETH (c < 16)
    int32_t agg[4];     // words 4 lane .. 4 lane + 3 of the slot's aggregate: this lane's 16 payload bytes
};

// Branch-free, so that no wait is needed until egress_emit uses the values: the
// RETH and aggregate words are loaded whatever the action (the slot index is in
// range for any PSN).
__device__ __forceinline__ EgressIn egress_fetch(const InccSwitchState& s, const uint8_t* __restrict__ in_frames,
                                                 int64_t in_stride, const int32_t* __restrict__ ports,
                                                 const int32_t* __restrict__ action,
                                                 const uint32_t* __restrict__ psns, int64_t f, int lane)
{
    EgressIn e;
    const int fan = s.fan_in;
    e.act = action[f];
    e.port = ports[f];
    e.psn = psns[f];
    // a lane-varying load stays in a VGPR, where a uniform one would be read into
    // an SGPR at once -- and that wait would also drain the previous frame's stores
    e.op = in_frames[f * in_stride + 40 + (lane & 3)];
    e.slot = e.psn & (s.slots - 1);
    e.reth = lane < 4 * fan ? s.reth[(size_t)e.slot * fan * 4 + lane] : 0u;
    typedef int32_t i4 __attribute__((ext_vector_type(4)));
    const i4 v = reinterpret_cast<const i4*>(s.agg + (size_t)e.slot * kLanes)[lane];   // one dwordx4 per lane
    e.agg[0] = v.x; e.agg[1] = v.y; e.agg[2] = v.z; e.agg[3] = v.w;
    return e;
}

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

// A 16-byte segment's raw CRC (bytes in memory order in a[0..3], little-endian
// words) shifted by Z_{16 (63 - sh_lane)}.
template <class L>
__device__ __forceinline__ uint32_t seg16_crc(const L& t, const uint32_t (&a)[4], int sh_lane)
{
    // nibble planes, one SDWA byte select per lookup, XORs three at a time (icrc_wave)
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t lo = opaque_u32(a[k] & 0x0F0F0F0Fu), hi = opaque_u32((a[k] >> 4) & 0x0F0F0F0Fu);
        uint32_t v[8];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            v[2 * b] = t.seg[4 * k + b + 1][0][(uint8_t)(lo >> (8 * b))];
            v[2 * b + 1] = t.seg[4 * k + b + 1][1][(uint8_t)(hi >> (8 * b))];
        }
        c = xor3(xor3(xor3(c, v[0], v[1]), v[2], v[3]), xor3(v[4], v[5], v[6]), v[7]);
    }
    const uint32_t clo = opaque_u32(c & 0x0F0F0F0Fu), chi = opaque_u32((c >> 4) & 0x0F0F0F0Fu);
    uint32_t v[8];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        v[2 * b] = t.lane16[2 * b][(uint8_t)(clo >> (8 * b))][sh_lane];
        v[2 * b + 1] = t.lane16[2 * b + 1][(uint8_t)(chi >> (8 * b))][sh_lane];
    }
    return xor3(xor3(v[0], v[1], v[2]), xor3(v[3], v[4], v[5]), v[6]) ^ v[7];
}

template <class L>
__device__ __forceinline__ uint32_t var_crc(const L& t, int wf, int k, uint32_t b)
{
    return t.var[var_row(wf, k)][0][b & 15u] ^ t.var[var_row(wf, k)][1][(b >> 4) & 15u];
}

// H_c for every (child, RETH flag) of the block's templates: quad q of wave w
// takes pair i = 16 w + q.  The header part of the message (doff - 10 bytes:
// 44, or 60 with RETH) is right-aligned in a 64-byte window (leading zeros do
// not change a raw CRC); lane s of the quad takes window bytes 16 s .. 16 s + 15.
template <class L>
__device__ void header_crcs(L& t, const uint8_t (*himg)[kHdrImg], int fan, int w, int lane)
{
    const int i = w * 16 + (lane >> 2), s = lane & 3;
    uint32_t c = 0;
    if (i < 2 * fan) {
        const int wf = i & 1;
        const int hdr = wf ? 60 : 44;
        uint32_t a[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int p = 16 * s + 4 * k + b - (64 - hdr);   // header byte; frame byte p + 10
                uint32_t byte = 0;
                if (p >= 0) {
                    const int fo = p + 10;
                    bool ff = fo < 14;
#pragma unroll
                    for (int m = 4; m < kNumMasked; ++m) ff = ff || fo == masked_pos(m);
                    byte = ff ? 0xFFu : himg[i][fo];
                }
                v |= byte << (8 * b);
            }
            a[k] = v;
        }
        c = seg16_crc(t, a, 60 + s);
    }
    c ^= (uint32_t)__shfl_xor((int)c, 1, kWave);
    c ^= (uint32_t)__shfl_xor((int)c, 2, kWave);
    uint32_t r = 0;
#pragma unroll
    for (int n = 0; n < 8; ++n) r ^= t.z1024[n][(c >> (4 * n)) & 15u];   // past the 1024-byte payload
    if (i < 2 * fan && s == 0) t.hcrc[i] = r;
}

// The CRC tables, the 2 * fan_in header images and their constant ICRC terms
// into the block's LDS (ends with a block barrier).  Blocks of 8 waves: quad
// q of wave w computes header term 16 w + q (2 * 31 at most).
template <class L>
__device__ void egress_setup(L& t, uint8_t (*himg)[kHdrImg], const InccFrameTemplate* __restrict__ tmpl, int fan, int w,
                             int lane)
{
    for (int i = threadIdx.x; i < kSeg * 2 * 16; i += blockDim.x) (&t.seg[0][0][0])[i] = (&g_seg[0][0][0])[i];
    for (int i = threadIdx.x; i < 8 * 16 * kWave; i += blockDim.x) (&t.lane16[0][0][0])[i] = (&g_lane16[0][0][0])[i];
    for (int i = threadIdx.x; i < kVarRows * 2 * 16; i += blockDim.x) (&t.var[0][0][0])[i] = (&g_var[0][0][0])[i];
    for (int i = threadIdx.x; i < 8 * 16; i += blockDim.x) (&t.z1024[0][0])[i] = (&g_z1024[0][0])[i];
    for (int i = threadIdx.x; i < 2 * fan; i += blockDim.x) build_header_image(himg[i], tmpl[i >> 1], (i & 1) != 0);
    __syncthreads();
    header_crcs(t, himg, fan, w, lane);
    __syncthreads();
}

// Every output frame of input frame f (rows f * fan_in + c): all fan_in children
// on COMPLETED (the broadcast, nts.c:368-371), the sender's child on REPLAY
// (nts.c:353-356).
//
// The payload (htonl of the aggregate, util.c:403-405 / :419-421) goes from
// registers straight to the output rows.  Lane l holds payload bytes
// [16 l, 16 l + 16), i.e. frame bytes doff + 16 l ..; doff (54, or 70 with a
// RETH) is 6 mod 16, so 16-byte output chunk doff/16 + 1 + l is lane l's bytes
// 10..15 followed by lane l+1's bytes 0..9: one funnel shift with the next
// lane's words, built once per input frame and stored once per child.  The
// chunks before it (the header, with the payload's first 10 bytes) are staged
// in a 80-byte LDS buffer per wave; lane 63 stores the last chunk: payload
// bytes 1018-1023 and the ICRC.  No per-child pass over the payload touches LDS.
__device__ void egress_emit(const InccSwitchState& s, const EgressIn& e, const uint8_t (*himg)[kHdrImg],
                            uint8_t* __restrict__ out, int64_t out_stride, bool out16, int32_t* __restrict__ out_len,
                            const EgressLds& t, uint8_t* hbuf, int64_t f, int lane)
{
    const int fan = s.fan_in;
    const bool all = e.act == INCCL_SW_COMPLETED;
    const bool one = e.act == INCCL_SW_REPLAY && e.port >= 0 && e.port < fan;
    const uint32_t op = (uint32_t)__shfl((int)e.op, 2, kWave) & 0xFFu;
    const int wf = is_write_first((uint8_t)op) ? 1 : 0;
    const int doff = 54 + 16 * wf;
    const int hchunks = doff / 16 + 1;         // 4 (or 5) chunks: header + payload bytes 0-9
    const int total = doff + kLanes * 4 + 4;   // util.c:341-345
    if (lane < fan) out_len[f * fan + lane] = (all || (one && lane == e.port)) ? total : 0;
    if (!all && !one) return;
    // this lane's 16 payload bytes (big-endian words, util.c:403-405), memory order
    uint32_t a[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = __builtin_bswap32((uint32_t)e.agg[k]);
    uint32_t nx[3];                            // lane l+1's first 12 bytes
#pragma unroll
    for (int k = 0; k < 3; ++k) nx[k] = (uint32_t)__shfl_down((int)a[k], 1, kWave);
    // output chunk hchunks + lane (lanes 0-62): bytes 10-15 of mine, 0-9 of the next lane's
    const uint32_t pc0 = __builtin_amdgcn_alignbyte(a[3], a[2], 2);
    const uint32_t pc1 = __builtin_amdgcn_alignbyte(nx[0], a[3], 2);
    const uint32_t pc2 = __builtin_amdgcn_alignbyte(nx[1], nx[0], 2);
    const uint32_t pc3 = __builtin_amdgcn_alignbyte(nx[2], nx[1], 2);
    // the payload's first 10 bytes into the header buffer (doff = 2 mod 4), once
    {
        const uint32_t a0 = (uint32_t)__shfl((int)a[0], 0, kWave), a1 = (uint32_t)__shfl((int)a[1], 0, kWave);
        const uint32_t a2 = (uint32_t)__shfl((int)a[2], 0, kWave);
        if (lane == 0) *reinterpret_cast<uint16_t*>(hbuf + doff) = (uint16_t)a0;
        if (lane == 1) *reinterpret_cast<uint32_t*>(hbuf + doff + 2) = __builtin_amdgcn_alignbyte(a1, a0, 2);
        if (lane == 2) *reinterpret_cast<uint32_t*>(hbuf + doff + 6) = __builtin_amdgcn_alignbyte(a2, a1, 2);
    }
    // P ^ V_op,psn: the payload's contribution (this lane's segment) and, on
    // lanes 0-4, the opcode and the four PSN bytes (util.c:378, :386)
    const uint32_t pw = e.psn | 0x80000000u;
    uint32_t pv = seg16_crc(t, a, lane);
    if (lane < 5) {
        const uint32_t b = lane == 0 ? op : (pw >> (8 * (4 - lane))) & 0xFFu;
        pv ^= var_crc(t, wf, lane, b);
    }
    const uint32_t pc = wave_xor(pv);
    const int c0 = all ? 0 : e.port, c1 = all ? fan : e.port + 1;
    for (int c = c0; c < c1; ++c) {
        // child c's RETH words (reth_keeper[slot][c], nts.c:442): lane 4c+i of
        // e.reth for c < 16, else from memory
        uint32_t r = 0, rk = 0;
        if (wf) {
            const int src = (4 * c + (lane & 3)) & (kWave - 1);
            r = (uint32_t)__shfl((int)e.reth, src, kWave);
            if (c >= kWave / 4) r = s.reth[((size_t)e.slot * fan + c) * 4 + (lane & 3)];
            // lane k < 16: RETH byte k = byte k & 3 of word k >> 2
            rk = (uint32_t)__shfl((int)r, lane >> 2, kWave);
        }
        uint32_t vr = 0;
        if (wf) vr = wave_xor(lane < 16 ? var_crc(t, 1, 5 + lane, (rk >> (8 * (lane & 3))) & 0xFFu) : 0u);
        const uint32_t crc = ~(pc ^ t.hcrc[2 * c + wf] ^ vr);   // util.c:424-426
        // header words 0-12 (bytes 0-51) from the image, opcode and PSN patched in
        if (lane < 13) {
            uint32_t hw = reinterpret_cast<const uint32_t*>(himg[2 * c + wf])[lane];
            if (lane == 10) hw = (hw & 0xFF00FFFFu) | (op << 16);                            // byte 42
            if (lane == 12) hw = (hw & 0x0000FFFFu) | ((pw >> 24) << 16) | (((pw >> 16) & 0xFFu) << 24);   // 50-51
            reinterpret_cast<uint32_t*>(hbuf)[lane] = hw;
        } else if (lane == 13) {                                                               // 52-53
            *reinterpret_cast<uint16_t*>(hbuf + 52) = (uint16_t)(((pw >> 8) & 0xFFu) | ((pw & 0xFFu) << 8));
        }
        if (wf) {                                                   // util.c:409-417: bytes 54-69
            const int k = lane - 14;                                // lanes 14..18
            const uint32_t rlo = (uint32_t)__shfl((int)r, (k - 1) & 3, kWave);
            const uint32_t rhi = (uint32_t)__shfl((int)r, k & 3, kWave);
            if (k == 0) *reinterpret_cast<uint16_t*>(hbuf + 54) = (uint16_t)rhi;
            else if (k >= 1 && k <= 3) *reinterpret_cast<uint32_t*>(hbuf + 52 + 4 * k) = __builtin_amdgcn_alignbyte(rhi, rlo, 2);
            else if (k == 4) *reinterpret_cast<uint16_t*>(hbuf + 68) = (uint16_t)(rlo >> 16);
        }
        __builtin_amdgcn_wave_barrier();
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        uint8_t* o = out + (f * fan + c) * out_stride;
        // header chunks (lanes 0 .. hchunks-1) from LDS
        if (lane < hchunks) {
            const u4 h = reinterpret_cast<const u4*>(hbuf)[lane];
            if (out16) reinterpret_cast<u4*>(o)[lane] = h;
            else {
                uint32_t* o32 = reinterpret_cast<uint32_t*>(o) + 4 * lane;
                o32[0] = h.x; o32[1] = h.y; o32[2] = h.z; o32[3] = h.w;
            }
        }
        // payload chunks (lanes 0-62) and the last chunk (lane 63: payload bytes
        // 1018-1023, the ICRC stored host order (LE), two bytes of zero padding)
        const u4 v = lane < kWave - 1 ? u4{pc0, pc1, pc2, pc3}
                                      : u4{pc0, (a[3] >> 16) | ((crc & 0xFFFFu) << 16), crc >> 16, 0u};
        if (out16) reinterpret_cast<u4*>(o)[hchunks + lane] = v;
        else {
            uint32_t* o32 = reinterpret_cast<uint32_t*>(o) + 4 * (hchunks + lane);
            o32[0] = v.x; o32[1] = v.y; o32[2] = v.z;
            if (lane < kWave - 1) o32[3] = v.w;   // lane 63: stop at the frame's 4-byte-rounded end
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Egress (nts.c:365-372 / :447-453 broadcast, :353-356 / :435-438 replay;
// frames per util.c:331-442): wave f builds input frame f's output frames.
// Persistent: each wave walks its input frames with the next one's inputs in
// flight.
__global__ __launch_bounds__(kWave* kEgressWaves) void k_egress(InccSwitchState s, const uint8_t* __restrict__ in_frames,
                                                               int64_t in_stride, int64_t count,
                                                               const int32_t* __restrict__ ports,
                                                               const int32_t* __restrict__ action,
                                                               const uint32_t* __restrict__ psns,
                                                               const InccFrameTemplate* __restrict__ tmpl,
                                                               uint8_t* __restrict__ out, int64_t out_stride,
                                                               int32_t* __restrict__ out_len)
{
    __shared__ EgressLds t;
    __shared__ __attribute__((aligned(16))) uint8_t buf[kEgressWaves][80];   // per wave: header chunks
    __shared__ __attribute__((aligned(16))) uint8_t himg[2 * 31][kHdrImg];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    egress_setup(t, himg, tmpl, s.fan_in, w, lane);
    const bool out16 = ((out_stride & 15) == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
    // Round r covers frames [r * step, (r + 1) * step); in round r this wave
    // takes frame r * step + (wave + r) mod step.  Rotating the offset by one per
    // round balances the waves: only every fan_in-th input frame of a PSN
    // completes it and emits, and with a fixed offset (step is even) the waves of
    // the other residues would idle while the rest built every output frame.
    // Once a round's frame is past count, every later round's is too.
    const int64_t step = (int64_t)gridDim.x * kEgressWaves;
    int64_t rot = (int64_t)blockIdx.x * kEgressWaves + w, base = 0;
    int64_t f = rot;
    if (f >= count) return;
    auto next = [&]() {
        base += step;
        rot = rot + 1 == step ? 0 : rot + 1;
        return base + rot;
    };
    // two register sets used alternately (no copy between them: a copy would
    // wait on every outstanding store of the previous frame too)
    EgressIn a = egress_fetch(s, in_frames, in_stride, ports, action, psns, f, lane), b;
    for (;;) {
        int64_t fn = next();
        if (fn < count) b = egress_fetch(s, in_frames, in_stride, ports, action, psns, fn, lane);
        egress_emit(s, a, himg, out, out_stride, out16, out_len, t, buf[w], f, lane);
        f = fn;
        if (f >= count) break;
        fn = next();
        if (fn < count) a = egress_fetch(s, in_frames, in_stride, ports, action, psns, fn, lane);
        egress_emit(s, b, himg, out, out_stride, out16, out_len, t, buf[w], f, lane);
        f = fn;
        if (f >= count) break;
    }
}

// ---------------------------------------------------------------------------
// Egress with a fixed fan-in (2, 3, 4 or 8): the same frames as k_egress, with
// every frame issuing the same global-memory instructions.
//
// gfx9 counts loads and stores on one counter (vmcnt), retired in issue order.
// The compiler waits for a loaded value with "vmcnt <= number of memory
// instructions issued after it" -- and where paths that issue different numbers
// of stores join (an absorbed frame returns early, a REPLAY emits one child, a
// COMPLETED fan_in), it can only wait conservatively.  k_egress's ISA shows
// vmcnt(0) at the top of every frame: it waits for the previous frame's stores
// AND for the next frame's prefetch, which then hides nothing.  Here the
// children loop is unrolled, the loads are unconditional (the last frame is
// re-read past the end), all CRC work sits in branches without memory
// instructions, and every store is predicated on the lane (exec mask), not
// branched around.
// ---------------------------------------------------------------------------

// egress_fetch with the RETH words through a buffer resource (lanes past
// 4 fan_in read out of range and get 0): no predicated load
template <int kFan>
__device__ __forceinline__ EgressIn egress_fetch_fixed(const InccSwitchState& s, const uint8_t* __restrict__ in_frames,
                                                       int64_t in_stride, const int32_t* __restrict__ ports,
                                                       const int32_t* __restrict__ action,
                                                       const uint32_t* __restrict__ psns, int64_t f, int lane)
{
    EgressIn e;
    e.act = action[f];
    e.port = ports[f];
    e.psn = psns[f];
    e.op = in_frames[f * in_stride + 40 + (lane & 3)];
    e.slot = e.psn & (s.slots - 1);
    const __amdgpu_buffer_rsrc_t rr =
        __builtin_amdgcn_make_buffer_rsrc(s.reth + (size_t)e.slot * kFan * 4, 0, 16 * kFan, 0x00020000);
    e.reth = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rr, lane < 4 * kFan ? 4 * lane : kOobOffset, 0, 0);
    // the slot's aggregate only for a frame that emits (COMPLETED / REPLAY): an
    // absorbed frame's load goes past the buffer (no memory traffic)
    typedef int32_t i4 __attribute__((ext_vector_type(4)));
    const bool emits = e.act == INCCL_SW_COMPLETED || e.act == INCCL_SW_REPLAY;
    const i4 v = (i4)__builtin_amdgcn_raw_buffer_load_b128(
        __builtin_amdgcn_make_buffer_rsrc(s.agg + (size_t)e.slot * kLanes, 0, 1024, 0x00020000),
        emits ? 16 * lane : kOobOffset, 0, 0);
    e.agg[0] = v.x; e.agg[1] = v.y; e.agg[2] = v.z; e.agg[3] = v.w;
    return e;
}

template <int kFan, bool kOut16, int kAux, class L>
__device__ __forceinline__ void egress_emit_fixed(const EgressIn& e, const uint8_t (*himg)[kHdrImg],
                                                  uint8_t* __restrict__ out, int64_t out_stride,
                                                  int32_t* __restrict__ out_len, const L& t, int64_t f, int lane)
{
    const bool all = e.act == INCCL_SW_COMPLETED;
    const bool one = e.act == INCCL_SW_REPLAY && e.port >= 0 && e.port < kFan;
    const uint32_t op = (uint32_t)__shfl((int)e.op, 2, kWave) & 0xFFu;
    const int wf = is_write_first((uint8_t)op) ? 1 : 0;
    const int doff = 54 + 16 * wf;
    const int hchunks = doff / 16 + 1;
    const int total = doff + kLanes * 4 + 4;   // util.c:341-345
    {
        const __amdgpu_buffer_rsrc_t lr = __builtin_amdgcn_make_buffer_rsrc(out_len + f * kFan, 0, 4 * kFan, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32((all || (one && lane == e.port)) ? total : 0, lr,
                                              lane < kFan ? 4 * lane : kOobOffset, 0, 0);
    }
    uint32_t a[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = __builtin_bswap32((uint32_t)e.agg[k]);
    uint32_t nx[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) nx[k] = (uint32_t)__shfl_down((int)a[k], 1, kWave);
    const uint32_t pc0 = __builtin_amdgcn_alignbyte(a[3], a[2], 2);
    const uint32_t pc1 = __builtin_amdgcn_alignbyte(nx[0], a[3], 2);
    const uint32_t pc2 = __builtin_amdgcn_alignbyte(nx[1], nx[0], 2);
    const uint32_t pc3 = __builtin_amdgcn_alignbyte(nx[2], nx[1], 2);
    const uint32_t pw = e.psn | 0x80000000u;
    // the payload's first 10 bytes (words 0-2 of lane 0, memory order): they
    // end the header chunks
    const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)a[0], 0);
    const uint32_t a1 = (uint32_t)__builtin_amdgcn_readlane((int)a[1], 0);
    const uint32_t a2 = (uint32_t)__builtin_amdgcn_readlane((int)a[2], 0);
    uint32_t pc = 0;
    if (all || one) {
        uint32_t pv = seg16_crc(t, a, lane);
        if (lane < 5) {
            const uint32_t b = lane == 0 ? op : (pw >> (8 * (4 - lane))) & 0xFFu;
            pv ^= var_crc(t, wf, lane, b);
        }
        pc = wave_xor(pv);
    }
    const uint32_t psn_hi = (pw >> 24) | (((pw >> 16) & 0xFFu) << 8);    // frame bytes 50, 51 (util.c:386)
    const uint32_t psn_lo = ((pw >> 8) & 0xFFu) | ((pw & 0xFFu) << 8);   // bytes 52, 53
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int c = 0; c < kFan; ++c) {
        const bool act_c = all || (one && c == e.port);
        uint32_t crc = 0;
        // child c's RETH words (reth_keeper[slot][c], nts.c:442), wave-uniform
        const uint32_t R0 = (uint32_t)__builtin_amdgcn_readlane((int)e.reth, 4 * c);
        const uint32_t R1 = (uint32_t)__builtin_amdgcn_readlane((int)e.reth, 4 * c + 1);
        const uint32_t R2 = (uint32_t)__builtin_amdgcn_readlane((int)e.reth, 4 * c + 2);
        const uint32_t R3 = (uint32_t)__builtin_amdgcn_readlane((int)e.reth, 4 * c + 3);
        if (act_c) {
            uint32_t vr = 0;
            if (wf) {
                // lane k < 16: RETH byte k = byte k & 3 of word k >> 2
                const uint32_t rk = (lane & 8) ? ((lane & 4) ? R3 : R2) : ((lane & 4) ? R1 : R0);
                vr = wave_xor(lane < 16 ? var_crc(t, 1, 5 + lane, (rk >> (8 * (lane & 3))) & 0xFFu) : 0u);
            }
            crc = ~(pc ^ t.hcrc[2 * c + wf] ^ vr);   // util.c:424-426
        }
        // header chunk `lane` (< hchunks) built in registers: the template image's
        // 16 bytes (util.c:348-388) with the opcode (byte 42), the PSN (50-53), the
        // RETH (54-69, util.c:409-417) and the payload's first 10 bytes patched in
        const u4 img = reinterpret_cast<const u4*>(himg[2 * c + wf])[lane < 5 ? lane : 0];
        uint32_t h0 = img.x, h1 = img.y, h2 = img.z, h3 = img.w;
        if (lane == 2) h2 = (h2 & 0xFF00FFFFu) | (op << 16);
        if (lane == 3) {
            const uint32_t b0 = wf ? R0 : a0, b1 = wf ? R1 : a1, b2 = wf ? R2 : a2;   // bytes 54-63
            h0 = (h0 & 0xFFFFu) | (psn_hi << 16);
            h1 = psn_lo | (b0 << 16);
            h2 = __builtin_amdgcn_alignbyte(b1, b0, 2);
            h3 = __builtin_amdgcn_alignbyte(b2, b1, 2);
        }
        if (lane == 4) {                                                // RETH frames only: bytes 64-79
            h0 = __builtin_amdgcn_alignbyte(R3, R2, 2);
            h1 = (R3 >> 16) | (a0 << 16);
            h2 = __builtin_amdgcn_alignbyte(a1, a0, 2);
            h3 = __builtin_amdgcn_alignbyte(a2, a1, 2);
        }
        const u4 h = {h0, h1, h2, h3};
        const __amdgpu_buffer_rsrc_t orow =
            __builtin_amdgcn_make_buffer_rsrc(out + (f * kFan + c) * out_stride, 0, (int)out_stride, 0x00020000);
        const bool sh = act_c && lane < hchunks;
        const u4 v = lane < kWave - 1 ? u4{pc0, pc1, pc2, pc3}
                                      : u4{pc0, (a[3] >> 16) | ((crc & 0xFFFFu) << 16), crc >> 16, 0u};
        const int ho = sh ? 16 * lane : kOobOffset, po = act_c ? 16 * (hchunks + lane) : kOobOffset;
        if (kOut16) {
            __builtin_amdgcn_raw_buffer_store_b128(h, orow, ho, 0, kAux);
            __builtin_amdgcn_raw_buffer_store_b128(v, orow, po, 0, kAux);
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(h.x, orow, ho, 0, kAux);
            __builtin_amdgcn_raw_buffer_store_b32(h.y, orow, ho + 4, 0, kAux);
            __builtin_amdgcn_raw_buffer_store_b32(h.z, orow, ho + 8, 0, kAux);
            __builtin_amdgcn_raw_buffer_store_b32(h.w, orow, ho + 12, 0, kAux);
            __builtin_amdgcn_raw_buffer_store_b32(v.x, orow, po, 0, kAux);
            __builtin_amdgcn_raw_buffer_store_b32(v.y, orow, po + 4, 0, kAux);
            __builtin_amdgcn_raw_buffer_store_b32(v.z, orow, po + 8, 0, kAux);
            // lane 63 stops at the frame's 4-byte-rounded end
            __builtin_amdgcn_raw_buffer_store_b32(v.w, orow, lane < kWave - 1 ? po + 12 : kOobOffset, 0, kAux);
        }
    }
}

template <int kFan, bool kOut16, int kEgW, int kAux>
__device__ __forceinline__ void egress_fixed_body(InccSwitchState s,
                                                                      const uint8_t* __restrict__ in_frames,
                                                                      int64_t in_stride, int64_t count,
                                                                      const int32_t* __restrict__ ports,
                                                                      const int32_t* __restrict__ action,
                                                                      const uint32_t* __restrict__ psns,
                                                                      const InccFrameTemplate* __restrict__ tmpl,
                                                                      uint8_t* __restrict__ out, int64_t out_stride,
                                                                      int32_t* __restrict__ out_len)
{
    __shared__ EgressLdsT<2 * kFan> t;   // header terms and images for this fan-in only
    __shared__ __attribute__((aligned(16))) uint8_t himg[2 * kFan][kHdrImg];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    egress_setup(t, himg, tmpl, kFan, w, lane);
    // the rotation of k_egress; frames past the end re-read the last one (a fixed
    // instruction stream) and are never emitted
    const int64_t step = (int64_t)gridDim.x * kEgW;
    int64_t rot = (int64_t)blockIdx.x * kEgW + w, base = 0;
    int64_t f = rot;
    if (f >= count) return;
    auto next = [&]() {
        base += step;
        rot = rot + 1 == step ? 0 : rot + 1;
        return base + rot;
    };
    auto clamp = [&](int64_t x) { return x < count ? x : count - 1; };
    EgressIn a = egress_fetch_fixed<kFan>(s, in_frames, in_stride, ports, action, psns, f, lane), b;
    {
        // as many stores as one frame emits, all dropped (a zero-size buffer): the
        // loop is entered with the same memory-instruction history as from its
        // back edge, so its first half's waits are not shortened by the merge
        const __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(out_len, 0, 0, 0x00020000);
#pragma unroll
        for (int i = 0; i < (kOut16 ? 2 * kFan + 1 : 8 * kFan + 1); ++i)
            __builtin_amdgcn_raw_buffer_store_b32(0, none, 4 * i, 0, 0);   // distinct offsets: kept
    }
    // two register sets used alternately, the fetch one frame ahead (two ahead,
    // with three sets, measured the same: 73.9 vs 73.6-74.4 us)
    for (;;) {
        int64_t fn = next();
        b = egress_fetch_fixed<kFan>(s, in_frames, in_stride, ports, action, psns, clamp(fn), lane);
        egress_emit_fixed<kFan, kOut16, kAux>(a, himg, out, out_stride, out_len, t, f, lane);
        f = fn;
        if (f >= count) break;
        fn = next();
        a = egress_fetch_fixed<kFan>(s, in_frames, in_stride, ports, action, psns, clamp(fn), lane);
        egress_emit_fixed<kFan, kOut16, kAux>(b, himg, out, out_stride, out_len, t, f, lane);
        f = fn;
        if (f >= count) break;
    }
}

#define INCCL_EGRESS_FIXED_ARGS                                                                                      \
    InccSwitchState s, const uint8_t *__restrict__ in_frames, int64_t in_stride, int64_t count,                      \
        const int32_t *__restrict__ ports, const int32_t *__restrict__ action, const uint32_t *__restrict__ psns,    \
        const InccFrameTemplate *__restrict__ tmpl, uint8_t *__restrict__ out, int64_t out_stride,                   \
        int32_t *__restrict__ out_len
// 8-wave blocks, three per CU = 24 waves: the measured optimum (profiles/r03/egress_waves/: 8 / 16 / 24 / 28
// waves per CU = 95.5 / 74.8 / 71.0 / 82-83 us)
template <int kFan, bool kOut16, int kAux = 0>
__global__ __launch_bounds__(kWave * 8) void k_egress_fixed(INCCL_EGRESS_FIXED_ARGS)
{
    egress_fixed_body<kFan, kOut16, 8, kAux>(s, in_frames, in_stride, count, ports, action, psns, tmpl, out, out_stride,
                                       out_len);
}
#undef INCCL_EGRESS_FIXED_ARGS


// ---------------------------------------------------------------------------
// Ingress (nts.c:303-483, root branch) reproduces the reference's one-frame-at-
// a-time order: frame index within the batch = arrival order.  What a serial
// switch decides for frame f depends on which copies of its (psn, port) and of
// its PSN's other ports came BEFORE f, so:
//   claim   (a lane per frame) parse + validate; per (slot, port) an atomicMin
//           of a batch-tagged frame index finds the first copy in the batch
//   apply   the first copy of a pair whose port bit was not set before the
//           batch is the arrival that counts: it adds its payload (nts.c:359-
//           363) and keeps its RETH (:442).  The PSN completes at the LAST of
//           its ports' counted arrivals (the max over ports of the first index;
//           ports already in before the batch count as earlier than every
//           frame): that frame is COMPLETED (:365-372), the others ABSORBED.
//           Every other copy is a retransmit (:353): REPLAY if the slot completed
//           before the batch or at an earlier frame of it (:354-356), else
//           DROPPED.
// Batch generation: claim tags its first-copy keys with g = gen[0] + 1 and
// publishes g in gen[1]; apply reads g from gen[1] and stores it to gen[0] for
// the next batch.  Each word is written while no kernel of the batch reads it,
// and nothing changes on the host per batch, so a captured batch (hipGraph)
// tags every replay anew.
// ---------------------------------------------------------------------------
// claim -> apply: a data frame still to classify: kActPending | WRITE_FIRST << 9 | opcode
// (the final actions are all below 0x100)
constexpr int kActPending = 0x100;
constexpr int kClaimBlock = 256;

// (~gen << 32) | (frame << 1) | wf: the minimum over a (slot, port)'s keys is the
// newest batch's earliest copy (the frame index dominates bit 0), and bit 0 tells
// apply where that copy's payload starts (byte 54, or 70 after a RETH) without
// another dependent load.  Frame indices stay below 2^31.
__device__ __forceinline__ uint64_t first_key(uint32_t gen, int64_t f, bool wf)
{
    return ((uint64_t)(~gen) << 32) | ((uint64_t)(uint32_t)f << 1) | (wf ? 1u : 0u);
}

// The batch call's per-child header terms, once per batch (claim's first wave):
// lane i < 2 fan_in builds child i/2's header image with RETH flag i&1
// (util.c:348-388; opcode, PSN and RETH left zero) and its ICRC term H =
// Z_1024(raw CRC of frame bytes 10 .. doff-1 with the CRC init and the masks as
// 0xFF) (util.c:250-286), into s.hdr: 2 * 31 images of 80 bytes, then the terms.
__device__ uint32_t g_tab[256];   // util.c:141-150

__device__ void header_terms(const InccSwitchState& s, const InccFrameTemplate* __restrict__ tmpl, int lane,
                             uint8_t (*img)[kHdrImg], uint32_t* tab)
{
    for (int i = lane; i < 256; i += kWave) tab[i] = g_tab[i];
    const int fan = s.fan_in;
    if (lane < 2 * fan) build_header_image(img[lane], tmpl[lane >> 1], (lane & 1) != 0);
    __builtin_amdgcn_wave_barrier();
    if (lane >= 2 * fan) return;
    const int wf = lane & 1, hdr = wf ? 60 : 44;
    uint32_t c = 0;
    for (int p = 0; p < hdr; ++p) {
        const int fo = p + 10;
        bool ff = fo < 14;
#pragma unroll
        for (int m = 4; m < kNumMasked; ++m) ff = ff || fo == masked_pos(m);
        const uint32_t b = ff ? 0xFFu : img[lane][fo];
        c = (c >> 8) ^ tab[(c ^ b) & 0xFFu];
    }
    uint32_t r = 0;
#pragma unroll
    for (int n = 0; n < 8; ++n) r ^= g_z1024[n][(c >> (4 * n)) & 15u];   // past the 1024-byte payload
    uint32_t* out = s.hdr + lane * (kHdrImg / 4);
    const uint32_t* im = reinterpret_cast<const uint32_t*>(img[lane]);
#pragma unroll
    for (int i = 0; i < kHdrImg / 4; ++i) out[i] = im[i];
    s.hdr[2 * 31 * (kHdrImg / 4) + lane] = r;
}

__global__ __launch_bounds__(kClaimBlock) void k_ingress_claim(InccSwitchState s, const uint8_t* __restrict__ frames,
                                                               int64_t stride, int64_t count,
                                                               const int32_t* __restrict__ ports,
                                                               int32_t* __restrict__ action,
                                                               uint32_t* __restrict__ psn_out,
                                                               const InccFrameTemplate* __restrict__ tmpl)
{
    const uint32_t g = *s.gen + 1u;   // this batch's generation
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) s.gen[1] = g;
        if (tmpl && threadIdx.x < kWave) {
            __shared__ __attribute__((aligned(16))) uint8_t img[2 * 31][kHdrImg];
            __shared__ uint32_t tab[256];
            header_terms(s, tmpl, threadIdx.x, img, tab);
        }
    }
    const int64_t f = (int64_t)blockIdx.x * kClaimBlock + threadIdx.x;
    if (f >= count) return;
    // rows are 4-byte aligned and at least 64 bytes: the header fields from four
    // dword loads (bytes 36-43 and 48-55 of the row) instead of byte loads
    const uint32_t* fw = reinterpret_cast<const uint32_t*>(frames + f * stride);
    const uint32_t w9 = fw[9], w10 = fw[10], w12 = fw[12], w13 = fw[13];
    const int port = ports[f];
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
            atomicAdd(&s.degree[slot], 1);                       // nts.c:351 / :431
            atomicMin(reinterpret_cast<unsigned long long*>(&s.first[(size_t)slot * s.fan_in + port]),
                      (unsigned long long)first_key(g, f, wf));
            act = kActPending | (wf ? 0x200 : 0) | op;
        }
    }
    action[f] = act;
    psn_out[f] = psn;
}

// ---------------------------------------------------------------------------
// Apply (after claim): one wave per two consecutive frames.
//
// A wave's work on its pair is three dependent memory round trips at most, and
// in the common case -- every port of a PSN arriving as consecutive frames,
// the reference's hosts posting one message each (api.c:293-327) -- two:
//   1. the claim results (action | WRITE_FIRST | opcode, port, PSN) and, on
//      16-byte aligned rows, both rows' payload chunks, loaded before anything
//      is known about the frames (lane l the 16-byte chunk 3 + l of each row,
//      lanes 0 and 1 also chunks 67 and 68: the payload starts 6 bytes into
//      chunk 3 or 4, whichever the opcode says, so both placements are covered);
//   2. the slot state, lane-parallel: lanes 32 k + p hold frame k's port p
//      (first-copy key), lanes 32 k and 32 k + 1 its two tagged arrival words;
//      in the batch call also the RETH keeper;
//   3. only when needed: the slot's partial from earlier batches (its bitmap
//      was not empty), the payload of a counted copy another wave holds.
// The slot's counted arrivals of this batch are summed by ONE wave -- the one
// holding the lowest counted port's first copy -- into the slot's partial with
// plain loads and stores: the same wrap-around sum as one atomic add per
// arrival (nts.c:361-363 / :443-445; integer addition commutes).  That wave
// also writes the slot's new arrival bitmap, recycles slot psn + slots/2 when
// the PSN completes (nts.c:235-242, :367: bitmap, degree and RETH keeper; the
// 1 KiB of aggregator words are left, since a slot whose bitmap is empty is
// summed from zero without reading them and nothing else reads a slot before
// its next counted arrival rewrites them), and in the batch call builds the
// completed PSN's fan_in broadcast frames (nts.c:447-453, util.c:331-442) from
// the aggregate in its registers.
//
// The split call's apply runs one pair per wave in short-lived blocks (a wave
// leaves once its stores are issued and the next starts).  The batch call's
// runs persistent blocks that load the egress tables (57 KiB) once; its waves
// walk the pairs.  The counters (profiles/r04/) put these kernels' VALU issue
// near the limit, so the code spends instructions sparingly: lane-rotation
// addresses are computed once, the WRITE_FIRST flag travels in the claim
// result, the payload CRC takes byte lookups, and the header chunks are the
// template image ORed with one patch per PSN.
//
// Arrival bitmap: every frame classifies against the bitmap as it was before
// the batch, while the summing wave writes the new one in the same launch.  A
// slot holds two 64-bit words {bits, tag = the batch that wrote them}; batch g
// writes word g & 1 only, and reads the newer of the words whose tag is not g.
// Whether a reader sees a word before or after batch g's store, it gets the
// pre-batch bitmap (64-bit accesses are single-copy atomic).  The recycle
// writes both words (no frame of the batch reads that slot).
// ---------------------------------------------------------------------------
constexpr int kApplyWaves = 8;    // split call: one pair per wave, 8-wave blocks
constexpr int kEmitWaves = 16;    // batch call: persistent 16-wave blocks

struct ApplyArgs {
    InccSwitchState s;
    const uint8_t* frames;
    int64_t stride, count;
    const int32_t* ports;
    int32_t* action;
    const uint32_t* psns;
    uint8_t* out;                    // batch call: the output rows and lengths
    int64_t out_stride;
    int32_t* out_len;
    int wide;                        // 16-byte aligned rows
};

// the arrival bitmap as it was before batch g: the newer of the two tagged
// words that batch g did not write (nts.c:59)
__device__ __forceinline__ uint32_t arrival_before(uint64_t w0, uint64_t w1, uint32_t g)
{
    const uint32_t t0 = (uint32_t)(w0 >> 32), t1 = (uint32_t)(w1 >> 32);
    const uint32_t d0 = t0 == g ? 0xFFFFFFFFu : g - t0, d1 = t1 == g ? 0xFFFFFFFFu : g - t1;
    return d0 <= d1 ? (uint32_t)w0 : (uint32_t)w1;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l)
{
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32);
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

// lane l + 1's value (lane 63 gets lane 0's), through a precomputed address
__device__ __forceinline__ uint32_t from_next(uint32_t v, int next4)
{
    return (uint32_t)__builtin_amdgcn_ds_bpermute(next4, (int)v);
}

// The batch call's egress tables in LDS, once per persistent block.
__device__ uint32_t g_segb[16][256];   // [byte j of a 16-byte segment][value] = Z_{15-j}(T[value])

struct EmitLds {
    uint32_t segb[16][256];
    uint32_t lane16[8][16][kWave];
    uint32_t var[kVarRows][2][16];
    uint32_t hcrc[2 * 31];
    __attribute__((aligned(16))) uint8_t img[2 * 31][kHdrImg];
};

// P ^ V_op,psn, in every lane: the payload's contribution to the ICRC (lane l's
// 16 bytes a[] -- memory order, little-endian words -- as 16 byte lookups, then
// shifted past the segments after it, Z_{16 (63 - l)}, as 8 nibble lookups)
// plus the opcode and PSN bytes' (lanes 0-4, already shifted to the message
// end), XORed over the wave.
__device__ __forceinline__ uint32_t payload_term(const EmitLds& t, const uint32_t (&a)[4], uint32_t var, int lane)
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
        s[2 * b] = t.lane16[2 * b][(uint8_t)(clo >> (8 * b))][lane];
        s[2 * b + 1] = t.lane16[2 * b + 1][(uint8_t)(chi >> (8 * b))][lane];
    }
    return wave_xor(xor3(xor3(s[0], s[1], s[2]), xor3(s[3], s[4], s[5]), xor3(s[6], s[7], var)));
}

// per-lane constants of a wave
struct LaneK {
    int lane, next4;   // lane, 4 * (lane + 1 mod 64): ds_bpermute address of the next lane
};

// What apply knows about one frame of its pair.
struct FrameK {
    int act, port;
    uint32_t psn, slot, op, wf;
    bool live;
};

// The batch call's broadcast of one completed PSN: fan_in frames into rows
// fd * fan_in + c, from the aggregate acc (this lane's four words).
template <bool kOut16, class RethOf>
__device__ __forceinline__ void emit_broadcast(const ApplyArgs& A, const EmitLds& t, const LaneK& L, const u4& acc,
                                               int64_t fd, uint32_t opd, uint32_t wfd, uint32_t psn, int fan,
                                               RethOf reth_of)
{
    const int lane = L.lane;
    uint32_t a[4];   // this lane's 16 payload bytes, big-endian (util.c:403-405), memory order
    a[0] = __builtin_bswap32(acc.x);
    a[1] = __builtin_bswap32(acc.y);
    a[2] = __builtin_bswap32(acc.z);
    a[3] = __builtin_bswap32(acc.w);
    const uint32_t pw = psn | 0x80000000u;
    // the opcode and PSN bytes' terms (util.c:378, :386), lanes 0-4
    const uint32_t vb = lane == 0 ? opd : (pw >> (8 * (4 - lane))) & 0xFFu;
    const uint32_t var = lane < 5 ? var_crc(t, (int)wfd, lane, vb) : 0u;
    const uint32_t pc = payload_term(t, a, var, lane);
    // payload chunk hchunks + l: bytes 10-15 of lane l, 0-9 of lane l + 1; the
    // last one (lane 63): bytes 1018-1023, the ICRC (host order), zero padding
    const uint32_t n0 = from_next(a[0], L.next4), n1 = from_next(a[1], L.next4), n2 = from_next(a[2], L.next4);
    const bool last = lane == kWave - 1;
    const uint32_t p0 = __builtin_amdgcn_alignbyte(a[3], a[2], 2);
    const uint32_t p1 = __builtin_amdgcn_alignbyte(n0, a[3], 2);
    const uint32_t p2 = __builtin_amdgcn_alignbyte(n1, n0, 2);
    const uint32_t p3 = last ? 0u : __builtin_amdgcn_alignbyte(n2, n1, 2);
    const uint32_t t63 = a[3] >> 16;
    // the header chunks' PSN-wide patch over the template images (which hold
    // zeros there): opcode (byte 42), PSN (50-53), and the payload's first 10
    // bytes after the BTH (no RETH) or after the RETH (lane 4's chunk)
    const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)a[0], 0);
    const uint32_t a1 = (uint32_t)__builtin_amdgcn_readlane((int)a[1], 0);
    const uint32_t a2 = (uint32_t)__builtin_amdgcn_readlane((int)a[2], 0);
    const uint32_t psn_hi = (pw >> 24) | (((pw >> 16) & 0xFFu) << 8);    // frame bytes 50, 51
    const uint32_t psn_lo = ((pw >> 8) & 0xFFu) | ((pw & 0xFFu) << 8);   // bytes 52, 53
    const uint32_t q1 = a0 << 16, q2 = __builtin_amdgcn_alignbyte(a1, a0, 2), q3 = __builtin_amdgcn_alignbyte(a2, a1, 2);
    const int pl = wfd ? 4 : 3;   // the lane whose chunk ends with the payload's first 10 bytes
    u4 patch;
    patch.x = lane == 3 ? psn_hi << 16 : 0u;
    patch.y = lane == 3 ? psn_lo : 0u;
    patch.y |= lane == pl ? q1 : 0u;
    patch.z = lane == pl ? q2 : (lane == 2 ? opd << 16 : 0u);
    patch.w = lane == pl ? q3 : 0u;
    const int hchunks = 4 + (int)wfd;
    const int ho = lane < hchunks ? 16 * lane : kOobOffset, po = 16 * (hchunks + lane);
    for (int c = 0; c < fan; ++c) {
        u4 h = reinterpret_cast<const u4*>(t.img[2 * c + wfd])[lane < 5 ? lane : 0];
        h.x |= patch.x;
        h.y |= patch.y;
        h.z |= patch.z;
        h.w |= patch.w;
        uint32_t crc = pc ^ t.hcrc[2 * c + wfd];
        if (wfd) {
            // child c's RETH (util.c:409-417): bytes 54-69, lane 3's chunk from
            // byte 6 on and lane 4's first 6 bytes; its ICRC term, lanes 0-15
            uint32_t R[4];
            reth_of(c, R);
            const uint32_t R0 = R[0], R1 = R[1], R2 = R[2], R3 = R[3];
            if (lane == 3) {
                h.y |= R0 << 16;
                h.z = __builtin_amdgcn_alignbyte(R1, R0, 2);
                h.w = __builtin_amdgcn_alignbyte(R2, R1, 2);
            }
            if (lane == 4) {
                h.x = __builtin_amdgcn_alignbyte(R3, R2, 2);
                h.y |= R3 >> 16;
            }
            const uint32_t rk = (lane & 8) ? ((lane & 4) ? R3 : R2) : ((lane & 4) ? R1 : R0);
            crc ^= wave_xor(lane < 16 ? var_crc(t, 1, 5 + lane, (rk >> (8 * (lane & 3))) & 0xFFu) : 0u);
        }
        crc = ~crc;   // util.c:424-426
        const u4 v = {p0, last ? t63 | (crc << 16) : p1, last ? crc >> 16 : p2, p3};
        const __amdgpu_buffer_rsrc_t orow = uniform_rsrc(A.out + (fd * fan + c) * A.out_stride, A.out_stride);
        if (kOut16) {
            __builtin_amdgcn_raw_buffer_store_b128(h, orow, ho, 0, kAuxNt);
            __builtin_amdgcn_raw_buffer_store_b128(v, orow, po, 0, kAuxNt);
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

// One pair of frames (2 pidx, 2 pidx + 1): classify, sum, and (batch call)
// broadcast.  g = the batch generation.
template <bool kEmit, bool kOut16>
__device__ __forceinline__ void apply_pair(const ApplyArgs& A, const int32_t* __restrict__ act_in,
                                           const int32_t* __restrict__ ports_in, const uint32_t* __restrict__ psns_in,
                                           int64_t pidx, uint32_t g, const EmitLds* tp, const LaneK& L)
{
    const InccSwitchState& s = A.s;
    // the lane number through an opaque copy: what the pair derives from it is
    // computed per pair, not hoisted out of the persistent loop into registers
    // held for the whole kernel (the occupancy is what hides this kernel's latency)
    const int lane = (int)opaque_u32((uint32_t)L.lane), fan = s.fan_in;
    const int64_t count = A.count, stride = A.stride;
    const bool have = 2 * pidx < count;
    const int64_t f0 = have ? 2 * pidx : 0;
    const bool in1 = have && f0 + 1 < count;
    const int64_t f1 = in1 ? f0 + 1 : f0;
    // round trip 1: the payload chunks of both rows, and the claim results
    u4 x[2] = {}, e[2] = {};
    if (A.wide) {
        const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(A.frames + f0 * stride, have ? (in1 ? 2 : 1) * stride : 0);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int rb = k * (int)stride;
            x[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, rb + 48 + 16 * lane, 0, 0);
            e[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane < 2 ? rb + 1072 + 16 * lane : kOobOffset, 0, 0);
        }
    }
    // the claim results, as scalar loads (the kernel's read-only views of
    // action / ports / PSNs, so that they arrive apart from the payloads and
    // round trip 2 can be issued before those land)
    FrameK F[2];
    F[0].act = have ? act_in[f0] : INCCL_SW_IGNORED;
    F[1].act = in1 ? act_in[f1] : INCCL_SW_IGNORED;
    F[0].port = ports_in[f0];
    F[1].port = ports_in[f1];
    F[0].psn = psns_in[f0];
    F[1].psn = psns_in[f1];
    const uint32_t tag = ~g, result_bit = 1u << fan, smask = s.slots - 1;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        FrameK& f = F[k];
        f.live = (f.act & kActPending) != 0;
        f.op = (uint32_t)f.act & 0xFFu;
        f.wf = ((uint32_t)f.act >> 9) & 1u;
        f.slot = f.psn & smask;
    }
    // round trip 2, lane-parallel over the two frames: half h = lane / 32 is
    // frame h; lane 32 h + p < 32 h + fan_in loads port p's first-copy key,
    // lanes 32 h and 32 h + 1 the two tagged arrival words
    const int hf = lane >> 5, pl = lane & 31;
    const bool live_h = hf ? F[1].live : F[0].live;
    const uint32_t slot_h = hf ? F[1].slot : F[0].slot;
    const uint64_t key = live_h && pl < fan ? s.first[(size_t)slot_h * fan + pl] : 0ull;
    const uint64_t av = live_h && pl < 2 ? s.arrival[2 * (size_t)slot_h + pl] : 0ull;
    uint32_t keep[2] = {0u, 0u};   // the batch call: the RETH keeper of each frame's slot
    if (kEmit) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (F[k].live) keep[k] = s.reth[(size_t)F[k].slot * fan * 4 + (lane < 4 * fan ? lane : 0)];
    }
    // each frame's payload words (this lane's four) and RETH words (uniform),
    // from the chunks of round trip 1 while round trip 2 is in flight
    uint32_t P[2][4], R[2][4];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const FrameK& f = F[k];
#pragma unroll
        for (int j = 0; j < 4; ++j) P[k][j] = R[k][j] = 0u;
        if (!f.live) continue;
        if (A.wide) {
            // chunk 4 + lane (lane 63: chunk 67) and 5 + lane (lane 62: 67, lane 63: 68)
            const bool last = lane == kWave - 1;
            uint32_t y0 = from_next(x[k].x, L.next4), y1 = from_next(x[k].y, L.next4);
            y0 = last ? (uint32_t)__builtin_amdgcn_readlane((int)e[k].x, 0) : y0;
            y1 = last ? (uint32_t)__builtin_amdgcn_readlane((int)e[k].y, 0) : y1;
            if (f.wf) {
                uint32_t y2 = from_next(x[k].z, L.next4), y3 = from_next(x[k].w, L.next4);
                uint32_t z0 = from_next(y0, L.next4), z1 = from_next(y1, L.next4);
                y2 = last ? (uint32_t)__builtin_amdgcn_readlane((int)e[k].z, 0) : y2;
                y3 = last ? (uint32_t)__builtin_amdgcn_readlane((int)e[k].w, 0) : y3;
                z0 = last ? (uint32_t)__builtin_amdgcn_readlane((int)e[k].x, 1) : z0;
                z1 = last ? (uint32_t)__builtin_amdgcn_readlane((int)e[k].y, 1) : z1;
                payload_from_chunks(u4{y0, y1, y2, y3}, z0, z1, P[k]);
                // the RETH, bytes 54-69: bytes 6-15 of chunk 3 (lane 0), 0-5 of chunk 4 (lane 1)
                const uint32_t c3y = (uint32_t)__builtin_amdgcn_readlane((int)x[k].y, 0);
                const uint32_t c3z = (uint32_t)__builtin_amdgcn_readlane((int)x[k].z, 0);
                const uint32_t c3w = (uint32_t)__builtin_amdgcn_readlane((int)x[k].w, 0);
                const uint32_t c4x = (uint32_t)__builtin_amdgcn_readlane((int)x[k].x, 1);
                const uint32_t c4y = (uint32_t)__builtin_amdgcn_readlane((int)x[k].y, 1);
                R[k][0] = __builtin_amdgcn_alignbyte(c3z, c3y, 2);
                R[k][1] = __builtin_amdgcn_alignbyte(c3w, c3z, 2);
                R[k][2] = __builtin_amdgcn_alignbyte(c4x, c3w, 2);
                R[k][3] = __builtin_amdgcn_alignbyte(c4y, c4x, 2);
            } else {
                payload_from_chunks(x[k], y0, y1, P[k]);
            }
        } else {
            const uint8_t* fr = A.frames + (f0 + k) * stride;
            payload16(fr, f.wf, lane, false, P[k]);
            if (f.wf) reth_words(fr, lane, R[k]);
        }
    }
    uint32_t pre[2];
#pragma unroll
    for (int k = 0; k < 2; ++k)
        pre[k] = F[k].live ? arrival_before(readlane64(av, 32 * k), readlane64(av, 32 * k + 1), g) : 0u;
    // classify (nts.c:353-372): lane 32 h + p < fan_in says when frame h's port
    // p counts, as 1 + frame index; 0 = before the batch, ~0 = not in this batch
    const uint32_t pre_h = hf ? pre[1] : pre[0];
    uint32_t at = 0, mine = 0xFFFFFFFFu, fo = 0xFFFFFFFFu;
    bool counted = false;
    if (live_h && pl < fan) {
        const bool in_batch = (uint32_t)(key >> 32) == tag;
        const uint32_t ef = ((uint32_t)key) >> 1;
        const bool before = (pre_h >> pl) & 1u;
        at = before ? 0u : (in_batch ? ef + 1u : 0xFFFFFFFFu);
        mine = in_batch ? ef : 0xFFFFFFFFu;
        fo = (uint32_t)key;                                 // frame << 1 | wf
        counted = in_batch && !before;
    }
    const uint64_t bal = __ballot(counted);
    uint32_t d = at;                                        // max over each half: the completing arrival
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) d = max(d, (uint32_t)__shfl_xor((int)d, o, kWave));
    int out_act[2];
    bool lead[2], counted_me[2];
    uint32_t cports[2], done_at[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const FrameK& f = F[k];
        out_act[k] = f.act;
        cports[k] = (uint32_t)(bal >> (32 * k));
        done_at[k] = (uint32_t)__builtin_amdgcn_readlane((int)d, 32 * k);
        lead[k] = counted_me[k] = false;
        if (!f.live) continue;
        const uint32_t fi = (uint32_t)(f0 + k);
        const uint32_t mk = (uint32_t)__builtin_amdgcn_readlane((int)mine, 32 * k + f.port);
        const uint32_t dk = done_at[k];
        const bool arrival = !((pre[k] >> f.port) & 1u) && mk == fi;   // the counted arrival: nts.c:359-363
        counted_me[k] = arrival;
        if (arrival) {
            out_act[k] = (dk == fi + 1u) ? INCCL_SW_COMPLETED : INCCL_SW_ABSORBED;   // nts.c:365
        } else {                                                 // retransmit: nts.c:353-357
            const bool done_before = (pre[k] & result_bit) != 0;
            const bool done_earlier = dk != 0u && dk != 0xFFFFFFFFu && dk - 1u < fi;
            out_act[k] = (done_before || done_earlier) ? INCCL_SW_REPLAY : INCCL_SW_DROPPED;
        }
        lead[k] = arrival && f.port == __builtin_ctz(cports[k]);
    }
    // the leaders: sum, store, bitmap, recycle, broadcast
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (!lead[k]) continue;
        const FrameK& f = F[k];
        u4 acc = {0u, 0u, 0u, 0u};
        // a slot whose bitmap was empty before the batch holds zeros (reset,
        // or recycled since its last use), so its partial is not read
        if (pre[k] != 0u) acc = reinterpret_cast<const u4*>(s.agg + (size_t)f.slot * kLanes)[lane];
        for (uint32_t m = cports[k]; m; m &= m - 1) {
            const uint32_t ek = (uint32_t)__builtin_amdgcn_readlane((int)fo, 32 * k + __builtin_ctz(m));
            const int64_t fe = (int64_t)(ek >> 1);
            uint32_t q[4];
            if (fe == f0) {
#pragma unroll
                for (int j = 0; j < 4; ++j) q[j] = P[0][j];
            } else if (in1 && fe == f1) {
#pragma unroll
                for (int j = 0; j < 4; ++j) q[j] = P[1][j];
            } else {
                payload16(A.frames + fe * stride, ek & 1u, lane, A.wide != 0, q);
            }
            acc.x += q[0];
            acc.y += q[1];
            acc.z += q[2];
            acc.w += q[3];
        }
        __builtin_nontemporal_store(acc, reinterpret_cast<u4*>(s.agg + (size_t)f.slot * kLanes) + lane);
        const bool complete = done_at[k] != 0xFFFFFFFFu;
        if (lane == 0)
            s.arrival[2 * (size_t)f.slot + (g & 1u)] =
                ((uint64_t)g << 32) | (pre[k] | cports[k] | (complete ? result_bit : 0u));   // nts.c:359, :366
        if (!complete) continue;
        {   // clear_state_data(psn + WINDOW), nts.c:235-242, :367
            const uint32_t rs = (f.psn + (s.slots >> 1)) & smask;
            for (int i = lane; i < fan * 4; i += kWave) s.reth[(size_t)rs * fan * 4 + i] = 0u;
            if (lane < 2) s.arrival[2 * (size_t)rs + lane] = (uint64_t)g << 32;
            if (lane == 0) s.degree[rs] = 0;
        }
        if constexpr (kEmit) {
            // the broadcast of the completing frame fd (nts.c:447-453): its
            // opcode, this PSN, each child's RETH as the keeper now holds it
            const int64_t fd = (int64_t)done_at[k] - 1;
            uint32_t opd, wfd;
            if (fd == f0) {
                opd = F[0].op;
                wfd = F[0].wf;
            } else if (in1 && fd == f1) {
                opd = F[1].op;
                wfd = F[1].wf;
            } else {
                const uint32_t w10 = reinterpret_cast<const uint32_t*>(A.frames + fd * stride)[10 + (lane & 1)];
                opd = ((uint32_t)__builtin_amdgcn_readlane((int)w10, 0) >> 16) & 0xFFu;
                wfd = is_write_first((uint8_t)opd) ? 1u : 0u;
            }
            // child c's RETH as the keeper holds it after this batch
            auto reth_of = [&](int c, uint32_t (&r)[4]) {
                const uint32_t ec = (uint32_t)__builtin_amdgcn_readlane((int)fo, 32 * k + c);
                if (((cports[k] >> c) & 1u) && (ec & 1u)) {   // counted in this batch from a WRITE_FIRST copy
                    const int64_t fe = (int64_t)(ec >> 1);
                    if (fe == f0) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) r[j] = R[0][j];
                    } else if (in1 && fe == f1) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) r[j] = R[1][j];
                    } else {
                        reth_words(A.frames + fe * stride, lane, r);
                    }
                } else if (c < kWave / 4) {                 // the keeper, as loaded
#pragma unroll
                    for (int j = 0; j < 4; ++j) r[j] = (uint32_t)__builtin_amdgcn_readlane((int)keep[k], 4 * c + j);
                } else {
                    const uint32_t v = s.reth[((size_t)f.slot * fan + c) * 4 + (lane & 3)];
#pragma unroll
                    for (int j = 0; j < 4; ++j) r[j] = (uint32_t)__builtin_amdgcn_readlane((int)v, j);
                }
            };
            emit_broadcast<kOut16>(A, *tp, L, acc, fd, opd, wfd, f.psn, fan, reth_of);
        }
    }
    // every frame: its action, its RETH into the keeper if it is a counted
    // WRITE_FIRST (nts.c:442), and (batch call) its rows' lengths
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (k == 0 ? !have : !in1) continue;
        const FrameK& f = F[k];
        const int64_t fi = f0 + k;
        if (f.live && lane == 0) A.action[fi] = out_act[k];
        if (counted_me[k] && f.wf && lane < 4)
            s.reth[((size_t)f.slot * fan + f.port) * 4 + lane] =
                lane == 0 ? R[k][0] : lane == 1 ? R[k][1] : lane == 2 ? R[k][2] : R[k][3];
        if (kEmit && lane < fan) {
            const int fin = out_act[k];
            const int total = 54 + 16 * (int)f.wf + kLanes * 4 + 4;   // util.c:341-345
            A.out_len[fi * fan + lane] =
                (f.live && (fin == INCCL_SW_COMPLETED || (fin == INCCL_SW_REPLAY && lane == f.port))) ? total : 0;
        }
    }
}

// The claim results are read through separate restrict views of the same
// arrays (act_in == A.action): every entry is read by one wave before that wave
// writes it, so the reads are of claim's values.
#define INCCL_APPLY_ARGS                                                                                        \
    ApplyArgs A, const int32_t *__restrict__ act_in, const int32_t *__restrict__ ports_in,                     \
        const uint32_t *__restrict__ psns_in

// the split call: one pair per wave, short-lived blocks
__global__ __launch_bounds__(kWave* kApplyWaves) void k_ingress_apply(INCCL_APPLY_ARGS)
{
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    const LaneK L{lane, ((lane + 1) & (kWave - 1)) * 4};
    const uint32_t g = A.s.gen[1];   // this batch's generation (claim's)
    apply_pair<false, true>(A, act_in, ports_in, psns_in, (int64_t)blockIdx.x * kApplyWaves + w, g, nullptr, L);
    // the next batch's claim adds one (stored last: a store before the claim
    // results' loads would keep the compiler from reading them as scalars)
    if (blockIdx.x == 0 && threadIdx.x == 0) A.s.gen[0] = g;
}

// the batch call: persistent blocks, the egress tables loaded once per block
template <bool kOut16>
__global__ __launch_bounds__(kWave* kEmitWaves) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_ingress_apply_emit(
    INCCL_APPLY_ARGS)
{
    __shared__ EmitLds t;
    const InccSwitchState& s = A.s;
    const int fan = s.fan_in;
    {
        constexpr int kFixed = (int)(sizeof(t.segb) + sizeof(t.lane16) + sizeof(t.var)) / 16;
        constexpr int n0 = (int)sizeof(t.segb) / 16, n1 = n0 + (int)sizeof(t.lane16) / 16;
        u4* dst = reinterpret_cast<u4*>(&t.segb[0][0]);
        for (int i = threadIdx.x; i < kFixed; i += blockDim.x)
            dst[i] = i < n0 ? reinterpret_cast<const u4*>(&g_segb[0][0])[i]
                   : i < n1 ? reinterpret_cast<const u4*>(&g_lane16[0][0][0])[i - n0]
                            : reinterpret_cast<const u4*>(&g_var[0][0][0])[i - n1];
        // this fan-in's header images and ICRC terms (claim's first wave wrote them)
        const int nh = 2 * fan * (kHdrImg / 4);
        for (int i = threadIdx.x; i < nh; i += blockDim.x) reinterpret_cast<uint32_t*>(&t.img[0][0])[i] = s.hdr[i];
        for (int i = threadIdx.x; i < 2 * fan; i += blockDim.x) t.hcrc[i] = s.hdr[2 * 31 * (kHdrImg / 4) + i];
    }
    __syncthreads();
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    const LaneK L{lane, ((lane + 1) & (kWave - 1)) * 4};
    const uint32_t g = s.gen[1];
    const int64_t pairs = (A.count + 1) >> 1, step = (int64_t)gridDim.x * kEmitWaves;
    for (int64_t p = (int64_t)blockIdx.x * kEmitWaves + w; p < pairs; p += step)
        apply_pair<true, kOut16>(A, act_in, ports_in, psns_in, p, g, &t, L);
    if (blockIdx.x == 0 && threadIdx.x == 0) s.gen[0] = g;
}

// The batch call's REPLAY resends (nts.c:353-356 / :435-438), after apply: a
// slot that completed earlier in the same batch has its aggregate only now.
// Each block scans its share of the actions; a block with no REPLAY leaves
// before loading any table (the common case: no retransmits).
__global__ __launch_bounds__(kWave* kEgressWaves) void k_replay(InccSwitchState s, const uint8_t* __restrict__ in_frames,
                                                                int64_t in_stride, int64_t count,
                                                                const int32_t* __restrict__ ports,
                                                                const int32_t* __restrict__ action,
                                                                const uint32_t* __restrict__ psns,
                                                                const InccFrameTemplate* __restrict__ tmpl,
                                                                uint8_t* __restrict__ out, int64_t out_stride,
                                                                int32_t* __restrict__ out_len)
{
    __shared__ EgressLds t;
    __shared__ __attribute__((aligned(16))) uint8_t buf[kEgressWaves][80];
    __shared__ __attribute__((aligned(16))) uint8_t himg[2 * 31][kHdrImg];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    const int64_t per = ((count + gridDim.x - 1) / gridDim.x + kWave - 1) / kWave * kWave;
    const int64_t b0 = (int64_t)blockIdx.x * per, b1 = b0 + per < count ? b0 + per : count;
    int any = 0;
    for (int64_t f = b0 + threadIdx.x; f < b1; f += blockDim.x) any |= action[f] == INCCL_SW_REPLAY;
    if (!__syncthreads_or(any)) return;
    egress_setup(t, himg, tmpl, s.fan_in, w, lane);
    const bool out16 = ((out_stride & 15) == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
    for (int64_t base = b0 + (int64_t)w * kWave; base < b1; base += (int64_t)kEgressWaves * kWave) {
        const int64_t f = base + lane;
        uint64_t m = __ballot(f < b1 && action[f] == INCCL_SW_REPLAY);
        while (m) {
            const int64_t fr = base + __builtin_ctzll(m);
            m &= m - 1;
            const EgressIn e = egress_fetch(s, in_frames, in_stride, ports, action, psns, fr, lane);
            egress_emit(s, e, himg, out, out_stride, out16, out_len, t, buf[w], fr, lane);
        }
    }
}


// ---------------------------------------------------------------------------
// host: CRC tables (util.c:141-159) and the zero-append operators
// ---------------------------------------------------------------------------
uint32_t host_tab[256];
uint32_t host_seg[kSeg][2][16];
uint32_t host_lane16[8][16][kWave];
uint32_t host_seg34[kSeg2][2][16];
uint32_t host_lane_shift32[8][16][32];
uint32_t host_var[5 + kVarBytes][2][16];
uint32_t host_z1024[8][16];
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
    for (int j = 0; j < kSeg; ++j)
        for (int h = 0; h < 2; ++h)
            for (uint32_t v = 0; v < 16; ++v) host_seg[j][h][v] = zeros_append(host_tab[v << (4 * h)], kSeg - 1 - j);
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
    // the batch call's payload segments: byte j of 16 -> Z_{15-j}(T[value])
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
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_seg), host_seg, sizeof(host_seg));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_lane16), host_lane16, sizeof(host_lane16));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_var), host_var, sizeof(host_var));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_z1024), host_z1024, sizeof(host_z1024));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_seg34), host_seg34, sizeof(host_seg34));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_lane_shift32), host_lane_shift32, sizeof(host_lane_shift32));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_segb), host_segb, sizeof(host_segb));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_tab), host_tab, sizeof(host_tab));
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

// split call: one wave per pair of frames, short-lived blocks
int launch_apply(const ApplyArgs& a, hipStream_t st)
{
    const int64_t pairs = (a.count + 1) / 2, blocks = (pairs + kApplyWaves - 1) / kApplyWaves;
    hipLaunchKernelGGL(k_ingress_apply, dim3((unsigned)(blocks < 1 ? 1 : blocks)), dim3(kWave * kApplyWaves), 0, st, a,
                       (const int32_t*)a.action, a.ports, a.psns);
    return (int)hipGetLastError();
}

// batch call: persistent blocks, as many as fit beside each other
template <bool kOut16>
int launch_apply_emit(const ApplyArgs& a, hipStream_t st)
{
    static const int per_cu = [] {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_ingress_apply_emit<kOut16>, kWave * kEmitWaves, 0) !=
                hipSuccess || n < 1)
            n = 1;
        return n;
    }();
    const int64_t pairs = (a.count + 1) / 2, need = (pairs + kEmitWaves - 1) / kEmitWaves;
    const int64_t cap = (int64_t)num_cus() * per_cu;
    hipLaunchKernelGGL(k_ingress_apply_emit<kOut16>, dim3((unsigned)(need < cap ? (need < 1 ? 1 : need) : cap)),
                       dim3(kWave * kEmitWaves), 0, st, a, (const int32_t*)a.action, a.ports, a.psns);
    return (int)hipGetLastError();
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
                  int32_t* action, uint32_t* psn_out, const InccFrameTemplate* tmpl, hipStream_t st)
{
    const dim3 lanes((unsigned)(((int64_t)count + kClaimBlock - 1) / kClaimBlock));
    hipLaunchKernelGGL(k_ingress_claim, lanes, dim3(kClaimBlock), 0, st, *s, frames, (int64_t)stride, (int64_t)count,
                       ports, action, psn_out, tmpl);
}

}  // namespace

extern "C" {

int inccl_k_frames_init(void) { return ensure_tables(); }

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
    launch_claim(s, frames, stride, count, ports, action, psn_out, nullptr, st);
    return launch_apply(apply_args(s, frames, stride, count, ports, action, psn_out), st);
}

int inccl_k_switch_batch(const InccSwitchState* s, const uint8_t* frames, size_t stride, size_t count,
                         const int32_t* ports, int32_t* action, uint32_t* psn_out, const InccFrameTemplate* tmpl,
                         uint8_t* out, size_t out_stride, int32_t* out_len, void* stream)
{
    if (count == 0) return 0;
    if (check_batch_args(s, frames, stride, count, ports, action, psn_out) || !tmpl || !out || !out_len ||
        (out_stride & 3) || out_stride < 1100 || out_stride > (1u << 20) || ((uintptr_t)out & 3))
        return INCCL_ERR_ARG;
    int rc = ensure_tables();
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    launch_claim(s, frames, stride, count, ports, action, psn_out, tmpl, st);
    ApplyArgs a = apply_args(s, frames, stride, count, ports, action, psn_out);
    a.out = out;
    a.out_stride = (int64_t)out_stride;
    a.out_len = out_len;
    const bool o16 = ((out_stride & 15) == 0) && (((uintptr_t)out & 15) == 0);
    rc = o16 ? launch_apply_emit<true>(a, st) : launch_apply_emit<false>(a, st);
    if (rc) return rc;
    const int64_t need = ((int64_t)count + kWave * kEgressWaves - 1) / (kWave * kEgressWaves);
    const int64_t cap = num_cus();
    hipLaunchKernelGGL(k_replay, dim3((unsigned)(need < cap ? need : cap)), dim3(kWave * kEgressWaves), 0, st, *s, frames,
                       (int64_t)stride, (int64_t)count, ports, (const int32_t*)action, (const uint32_t*)psn_out, tmpl, out,
                       (int64_t)out_stride, out_len);
    return (int)hipGetLastError();
}

int inccl_k_switch_egress(const InccSwitchState* s, const uint8_t* in_frames, size_t in_stride, size_t count,
                          const int32_t* ports, const int32_t* action, const uint32_t* psns,
                          const InccFrameTemplate* tmpl, uint8_t* out, size_t out_stride, int32_t* out_len,
                          void* stream)
{
    if (count == 0) return 0;
    if (!s || !in_frames || !ports || !action || !psns || !tmpl || !out || !out_len || (out_stride & 3) ||
        out_stride < 1100 || ((uintptr_t)out & 3))
        return INCCL_ERR_ARG;
    int rc = ensure_tables();
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    // persistent grid (the CRC tables are loaded once per block), three 8-wave
    // blocks per CU: 24 waves, the measured optimum (profiles/r03/egress_waves/)
    const int64_t need = ((int64_t)count + kEgressWaves - 1) / kEgressWaves;
    const int64_t cap = (int64_t)num_cus() * 3;
    const int eg = (int)(need < cap ? (need < 1 ? 1 : need) : cap);
    const bool o16 = ((out_stride & 15) == 0) && (((uintptr_t)out & 15) == 0);
    // non-temporal frame stores (the frames are not re-read here): egress 65.3 vs
    // 71.0 us, and the next batch's apply no longer starts behind 144 MB of dirty
    // lines (profiles/r03/store_policy/)
    const dim3 g(eg), b(kWave * kEgressWaves);
    const int64_t is = (int64_t)in_stride, os = (int64_t)out_stride, n = (int64_t)count;
#define INCCL_EGRESS_FIXED(F)                                                                                   \
    case F:                                                                                                     \
        if (o16)                                                                                                \
            hipLaunchKernelGGL((k_egress_fixed<F, true, kAuxNt>), g, b, 0, st, *s, in_frames, is, n, ports,     \
                               action, psns, tmpl, out, os, out_len);                                           \
        else                                                                                                    \
            hipLaunchKernelGGL((k_egress_fixed<F, false, kAuxNt>), g, b, 0, st, *s, in_frames, is, n, ports,    \
                               action, psns, tmpl, out, os, out_len);                                           \
        return (int)hipGetLastError();
    // fan-in 2, 3, 4, 8: the straight-line kernel; others the generic one
    switch (s->fan_in) {
        INCCL_EGRESS_FIXED(2)
        INCCL_EGRESS_FIXED(3)
        INCCL_EGRESS_FIXED(4)
        INCCL_EGRESS_FIXED(8)
    default: break;
    }
#undef INCCL_EGRESS_FIXED
    hipLaunchKernelGGL(k_egress, g, b, 0, st, *s, in_frames, is, n, ports, action, psns, tmpl, out, os, out_len);
    return (int)hipGetLastError();
}

}  // extern "C"
