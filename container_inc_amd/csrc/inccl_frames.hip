// inccl_frames.hip -- the reference's switch dataplane on the GPU (gfx950):
// RoCEv2 frame parse, per-PSN idempotent aggregation, egress frame build and
// the RoCE ICRC (CRC-32).  Reference: repository/src/non_termination_switch.c
// (nts.c) :303-501 for the pipeline and :55-60 / :231-250 for its state;
// repository/src/util.c:331-442 (build_eth_packet), :250-286 (compute_icrc),
// :141-195 (crc32), :106-127 (ipv4_checksum).
//
// One wave64 per frame.  A frame is staged in LDS; the ICRC input (4 x 0xFF --
// the CRC init folded into the message -- then the masked IP .. payload bytes)
// is the frame from byte 10 on, with bytes 10-13 and the masked fields set to
// 0xFF in LDS while the CRC runs.  It is right-aligned in a 1088-byte window
// (64 lanes x 17 B), so leading zeros do not change the raw CRC.  CRC-32 is
// linear over GF(2): the window's raw CRC is the XOR over lanes of
// Z_{17 (63 - lane)}(crc(segment)), Z_n = "append n zero bytes".  Each lane
// (1) reads its 17 bytes as 6 dwords + byte-aligns them, (2) computes the
// segment's CRC as 34 independent nibble lookups (byte j's contribution is
// Z_{16-j}(T[b_j]); a 2.2 KiB table whose 16 entries per lookup sit in 16
// distinct banks, so no dependency chain and no bank conflicts), (3) applies
// its own fixed Z as 8 nibble lookups in a lane-major table (bank = lane), and
// (4) the wave XOR-reduces.  34 KiB of tables per block.
//
// State on the GPU (slots = PSN ring size, power of two; the reference uses 16):
//   agg[slots][256] int32        aggregator        (nts.c:55)
//   arrival[slots] uint32        port bitmap + bit fan_in = "result known" (nts.c:59, :366)
//   degree[slots] int32          arrivals incl. retransmits (nts.c:60, :351)
//   reth[slots][fan_in][16 B]    RETH of each child's WRITE_FIRST (nts.c:57, :442)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <mutex>

#include "inccl_frames.h"

namespace {

constexpr int kWave = 64;
constexpr int kWin = 1088;            // 64 lanes x 17 bytes
constexpr int kSeg = 17;
constexpr int kFrameMax = 1152;       // staged frame bytes (>= 1098)
constexpr int kWavesPerBlock = 4;
constexpr int kEgressWaves = 8;       // 512-lane blocks, two per CU, persistent grid
constexpr int kLanes = 256;           // int32 lanes per packet (nts.c:55)
constexpr int kAuxNt = 2;   // buffer instruction cache policy: nt (streaming, not re-read)
constexpr int kOobOffset = 0x7FFFFFF0;   // past any row: a buffer store there is dropped

__device__ uint32_t g_seg[kSeg][2][16];       // [byte j][nibble][value] = Z_{16-j}(T[value << 4 nibble]), T = util.c:141-150
__device__ uint32_t g_segb[kSeg][256];        // [byte j][value] = Z_{16-j}(T[value])
__device__ uint32_t g_lane_shift[8][16][kWave];   // [nibble][value][lane] = Z_{17 (63 - lane)}(value << 4 nibble)

// kByte = false: a lane's segment CRC as 34 independent nibble lookups in a
// 2.2 KiB table (no bank conflicts, two VALU ops of index math per lookup).
// kByte = true: 17 byte lookups in a 17 KiB table (half the index math; the
// lanes' random entries conflict in the banks, and 59 KiB of LDS per block
// leaves two blocks per CU).  Measured 64.5 vs 62.7 us per 131 072 frames, so
// the nibble form stays the product; $INCCL_ICRC_BYTE_TABLES=1 selects the
// byte form (profiles/r03/icrc_byte_vs_nibble.txt).
template <bool kByte>
struct CrcLds {
    uint32_t seg[kByte ? kSeg * 256 : kSeg * 2 * 16];
    uint32_t lane_sh[8][16][kWave]; // per-lane zero-append operator, nibble-sliced
};

template <bool kByte>
__device__ __forceinline__ void load_tables(CrcLds<kByte>& t)
{
    const uint32_t* seg = kByte ? &g_segb[0][0] : &g_seg[0][0][0];
    for (int i = threadIdx.x; i < (kByte ? kSeg * 256 : kSeg * 2 * 16); i += blockDim.x) t.seg[i] = seg[i];
    uint32_t* dst = &t.lane_sh[0][0][0];
    const uint32_t* src = &g_lane_shift[0][0][0];
    for (int i = threadIdx.x; i < 8 * 16 * kWave; i += blockDim.x) dst[i] = src[i];
}

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

// ICRC of the frame staged at `fr` (LDS, at least 1152 B, 4-B aligned), whose
// masked bytes are already 0xFF; result valid in every lane.
template <bool kByte>
__device__ uint32_t icrc_wave(const uint8_t* fr, const CrcLds<kByte>& t, int lane)
{
    const int ip_total = ((int)fr[16] << 8) | fr[17];   // message = 4 (init) + ip_total - 4 (no ICRC) bytes
    const int lead = kWin - ip_total;                   // zero bytes before the message
    const int o = 10 + lane * kSeg - lead;              // frame offset of this lane's first byte
    uint32_t c = 0;
    if (o + kSeg > 10) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(fr);
        const int d0 = o >> 2;   // floor division (o may be negative)
        uint32_t dw[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) dw[k] = d0 + k >= 0 ? w[d0 + k] : 0u;
        const uint32_t sh = (uint32_t)o & 3u;
        uint32_t a[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) a[k] = __builtin_amdgcn_alignbyte(dw[k + 1], dw[k], sh);
        const int nz = 10 - o;   // leading bytes of this lane before the message: zero
        if (nz > 0) {
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const int z = nz - 4 * k;
                a[k] = z >= 4 ? 0u : (z > 0 ? a[k] & (0xFFFFFFFFu << (8 * z)) : a[k]);
            }
        }
        // the segment's CRC register (util.c:190-192 run from 0) is linear in its
        // bytes: XOR over byte j of Z_{16-j}(T[b_j]), each split into two nibble
        // lookups.  No lookup depends on another, and the 16 entries one
        // ds_read_b32 can touch sit in 16 distinct banks (no conflicts).
        if (kByte) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
#pragma unroll
                for (int b = 0; b < 4; ++b) c ^= t.seg[(4 * k + b) * 256 + ((a[k] >> (8 * b)) & 0xFFu)];
            }
            c ^= t.seg[16 * 256 + (a[4] & 0xFFu)];
        } else {
            // nibble planes: byte b of lo / hi is the low / high nibble of byte b,
            // so each lookup's index is one SDWA byte select; XOR three at a time
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t lo = opaque_u32(a[k] & 0x0F0F0F0Fu), hi = opaque_u32((a[k] >> 4) & 0x0F0F0F0Fu);
                uint32_t v[8];
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    v[2 * b] = t.seg[((4 * k + b) * 2) * 16 + (uint8_t)(lo >> (8 * b))];
                    v[2 * b + 1] = t.seg[((4 * k + b) * 2 + 1) * 16 + (uint8_t)(hi >> (8 * b))];
                }
                c = xor3(xor3(xor3(c, v[0], v[1]), v[2], v[3]), xor3(v[4], v[5], v[6]), v[7]);
            }
            c = xor3(c, t.seg[(16 * 2) * 16 + (a[4] & 15u)], t.seg[(16 * 2 + 1) * 16 + ((a[4] >> 4) & 15u)]);
        }
        // shift to the window's end: Z_{17 (63 - lane)}(c)
        const uint32_t clo = opaque_u32(c & 0x0F0F0F0Fu), chi = opaque_u32((c >> 4) & 0x0F0F0F0Fu);
        uint32_t v[8];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            v[2 * b] = t.lane_sh[2 * b][(uint8_t)(clo >> (8 * b))][lane];
            v[2 * b + 1] = t.lane_sh[2 * b + 1][(uint8_t)(chi >> (8 * b))][lane];
        }
        c = xor3(xor3(v[0], v[1], v[2]), xor3(v[3], v[4], v[5]), v[6]) ^ v[7];
    }
    // XOR-reduce the 64 lane contributions with DPP (one VALU op per step, no
    // LDS): quads, half-rows, rows, then the row broadcasts; lane 63 ends with
    // the whole window
    c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x141, 0xF, 0xF, false);   // row_half_mirror
    c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x140, 0xF, 0xF, false);   // row_mirror
    c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x142, 0xA, 0xF, false);   // row_bcast15 -> rows 1, 3
    c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x143, 0xC, 0xF, false);   // row_bcast31 -> rows 2, 3
    return ~(uint32_t)__builtin_amdgcn_readlane((int)c, 63);
}

// Header word of a frame (bytes 16-19), loaded lane-varying so that it stays a
// vector load: a uniform one would go through the scalar cache, and the LDS
// waits of the running CRC (lgkmcnt) would then wait for it too.
__device__ __forceinline__ uint32_t icrc_hdr_load(const uint8_t* g, int lane)
{
    return reinterpret_cast<const uint32_t*>(g)[4 + (lane & 1)];
}

__device__ __forceinline__ int icrc_ip_total(uint32_t hdr_lane)
{
    const uint32_t h = (uint32_t)__builtin_amdgcn_readlane((int)hdr_lane, 0);
    return (int)(((h & 0xFFu) << 8) | ((h >> 8) & 0xFFu));
}

// an ICRC is computed only for an IP length the window holds and whose frame
// lies inside its row: a header claiming more bytes than the row has reads as
// malformed (ICRC 0), never as the next row's bytes
__device__ __forceinline__ bool icrc_len_ok(int ipt, int64_t stride)
{
    return ipt >= 28 && ipt <= kWin && 14 + ipt <= kFrameMax && 14 + ipt <= stride;
}

// Persistent: each wave walks its frames with the next frame's words (5 dwords
// a lane, coalesced) and the one after's header in flight while the current
// frame's CRC runs from LDS.
template <bool kByte, int kIcrcWaves>
__global__ __launch_bounds__(kWave* kIcrcWaves) void k_icrc(const uint8_t* __restrict__ frames, int64_t stride,
                                                                int64_t count, uint32_t* __restrict__ out)
{
    __shared__ CrcLds<kByte> t;
    __shared__ __attribute__((aligned(16))) uint8_t buf[kIcrcWaves][kFrameMax];
    load_tables(t);
    __syncthreads();
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    constexpr int kWords = (kFrameMax / 4 + kWave - 1) / kWave;   // 5
    const int64_t step = (int64_t)gridDim.x * kIcrcWaves;
    int64_t f = (int64_t)blockIdx.x * kIcrcWaves + w;
    if (f >= count) return;
    uint32_t* lds = reinterpret_cast<uint32_t*>(buf[w]);
    auto fetch = [&](int64_t fr, int ipt, uint32_t (&v)[kWords]) {
        const uint32_t* g = reinterpret_cast<const uint32_t*>(frames + fr * stride);
        const int words = icrc_len_ok(ipt, stride) ? (14 + ipt + 3) >> 2 : 0;
#pragma unroll
        for (int k = 0; k < kWords; ++k) {
            const int i = lane + k * kWave;
            v[k] = i < words ? g[i] : 0u;
        }
    };
    int ip = icrc_ip_total(icrc_hdr_load(frames + f * stride, lane));
    uint32_t cur[kWords];
    fetch(f, ip, cur);
    uint32_t hdrN = f + step < count ? icrc_hdr_load(frames + (f + step) * stride, lane) : 0u;
    for (;;) {
#pragma unroll
        for (int k = 0; k < kWords; ++k)
            if (lane + k * kWave < kFrameMax / 4) lds[lane + k * kWave] = cur[k];
        __builtin_amdgcn_wave_barrier();
        if (lane < kNumMasked) buf[w][masked_pos(lane)] = 0xFF;
        __builtin_amdgcn_wave_barrier();
        const int64_t fn = f + step;
        int ipn = 0;
        if (fn < count) {
            ipn = icrc_ip_total(hdrN);
            fetch(fn, ipn, cur);
            hdrN = fn + step < count ? icrc_hdr_load(frames + (fn + step) * stride, lane) : 0u;
        }
        const uint32_t crc = icrc_len_ok(ip, stride) ? icrc_wave<kByte>(buf[w], t, lane) : 0u;
        if (lane == 0) out[f] = crc;
        __builtin_amdgcn_wave_barrier();
        f = fn;
        ip = ipn;
        if (f >= count) break;
    }
}

// ---------------------------------------------------------------------------
// ICRC, two frames per wave ($INCCL_ICRC_DIRECT=0; $INCCL_ICRC_PAIR=0: k_icrc): lanes 0-31 take frame 2p,
// lanes 32-63 frame 2p+1, each lane 34 bytes of the 1088-byte window (32 x 34).
// Per frame: 34 x 2 nibble lookups over 32 lanes (38 lookup instructions per
// frame, against 42), a 16 KiB lane-shift table (Z_{34 (31 - lane')}), and one
// 5-step DPP reduction for both frames.  Same right-aligned window, masks and
// results as icrc_wave.
// ---------------------------------------------------------------------------
constexpr int kSeg2 = 34;
__device__ uint32_t g_seg34[kSeg2][2][16];          // [byte j][nibble][value] = Z_{33-j}(T[value << 4 nibble])
__device__ uint32_t g_lane_shift32[8][16][32];      // [nibble][value][lane'] = Z_{34 (31 - lane')}(value << 4 nibble)

struct CrcLdsPair {
    uint32_t seg[kSeg2][2][16];
    uint32_t lane_sh[8][16][32];
    uint32_t spread[16];   // k_icrc_direct<.., 1>: nibble -> byte mask (bit i -> byte i)
    uint32_t andor[32][2];   // k_icrc_direct<.., 2>: [nibble | 16 (frame dword <= 2)] -> (AND, OR)
};

// ICRC of the frame of this lane's half (staged at `fr`, masked bytes 0xFF);
// returns the raw (pre-reduction) contribution of this lane
// The segment's contribution from its frame dwords dw[k] = frame dword (o >> 2) + k
// (o = the segment's first frame byte; masked bytes already 0xFF)
// kZeroed: dw already holds 0 for every frame byte below 10 (icrc_mask_regs_zero),
// so neither the zeroing nor the skip of an all-zero segment is needed
template <bool kZeroed = false>
__device__ __forceinline__ uint32_t icrc_half_regs(const uint32_t (&dw)[10], int o, const CrcLdsPair& t, int l)
{
    uint32_t c = 0;
    if (kZeroed || o + kSeg2 > 10) {
        const uint32_t sh = (uint32_t)o & 3u;
        uint32_t a[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) a[k] = __builtin_amdgcn_alignbyte(dw[k + 1], dw[k], sh);
        const int nz = 10 - o;
        if (!kZeroed && nz > 0) {
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const int z = nz - 4 * k;
                a[k] = z >= 4 ? 0u : (z > 0 ? a[k] & (0xFFFFFFFFu << (8 * z)) : a[k]);
            }
        }
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
        c = xor3(xor3(v[0], v[1], v[2]), xor3(v[3], v[4], v[5]), v[6]) ^ v[7];
    }
    return c;
}

__device__ __forceinline__ uint32_t icrc_half_lane(const uint8_t* fr, const CrcLdsPair& t, int l)
{
    const int ip_total = ((int)fr[16] << 8) | fr[17];
    const int lead = kWin - ip_total;
    const int o = 10 + l * kSeg2 - lead;                 // frame offset of this lane's first byte
    const uint32_t* w = reinterpret_cast<const uint32_t*>(fr);
    const int d0 = o >> 2;
    uint32_t dw[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) dw[k] = d0 + k >= 0 && o + kSeg2 > 10 ? w[d0 + k] : 0u;
    return icrc_half_regs(dw, o, t, l);
}

template <int kW>
__global__ __launch_bounds__(kWave* kW) void k_icrc_pair(const uint8_t* __restrict__ frames, int64_t stride,
                                                         int64_t count, uint32_t* __restrict__ out)
{
    __shared__ CrcLdsPair t;
    __shared__ __attribute__((aligned(16))) uint8_t buf[kW][2][kFrameMax];
    for (int i = threadIdx.x; i < kSeg2 * 2 * 16; i += blockDim.x) (&t.seg[0][0][0])[i] = (&g_seg34[0][0][0])[i];
    for (int i = threadIdx.x; i < 8 * 16 * 32; i += blockDim.x) (&t.lane_sh[0][0][0])[i] = (&g_lane_shift32[0][0][0])[i];
    __syncthreads();
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    const int half = lane >> 5, l = lane & 31;
    constexpr int kWords = kFrameMax / 4 / 32;   // 9 dwords per lane and frame
    const int64_t pairs = (count + 1) >> 1, step = (int64_t)gridDim.x * kW;
    int64_t p = (int64_t)blockIdx.x * kW + w;
    if (p >= pairs) return;
    uint8_t* mine = buf[w][half];
    uint32_t* lds = reinterpret_cast<uint32_t*>(mine);
    auto fetch = [&](int64_t pp, uint32_t (&v)[kWords]) {
        const int64_t f = 2 * pp + half;
        const bool in = f < count;
        const uint8_t* g8 = frames + (in ? f : 0) * stride;
        const uint32_t* g = reinterpret_cast<const uint32_t*>(g8);
        // the half's IP length (its lanes all read the same dword) bounds the words read
        const uint32_t hw = g[4];
        const int ipt = (int)(((hw & 0xFFu) << 8) | ((hw >> 8) & 0xFFu));
        const int words = in && icrc_len_ok(ipt, stride) ? (14 + ipt + 3) >> 2 : 0;
#pragma unroll
        for (int k = 0; k < kWords; ++k) {
            const int i = l + k * 32;
            v[k] = i < words ? g[i] : 0u;
        }
    };
    uint32_t cur[kWords];
    fetch(p, cur);
    for (;;) {
#pragma unroll
        for (int k = 0; k < kWords; ++k) lds[l + k * 32] = cur[k];
        __builtin_amdgcn_wave_barrier();
        if (l < kNumMasked) mine[masked_pos(l)] = 0xFF;
        __builtin_amdgcn_wave_barrier();
        const int64_t pn = p + step;
        if (pn < pairs) fetch(pn, cur);
        const int ipt = ((int)mine[16] << 8) | mine[17];
        const int64_t f = 2 * p + half;
        uint32_t c = icrc_half_lane(mine, t, l);
        if (!icrc_len_ok(ipt, stride)) c = 0u;
        // XOR-reduce each 32-lane half: quads, half-rows, rows, then row 0 into
        // row 1 and row 2 into row 3 (lanes 31 and 63 end with the two frames)
        c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0xB1, 0xF, 0xF, false);
        c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x4E, 0xF, 0xF, false);
        c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x141, 0xF, 0xF, false);
        c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x140, 0xF, 0xF, false);
        c ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x142, 0xA, 0xF, false);
        const uint32_t ca = ~(uint32_t)__builtin_amdgcn_readlane((int)c, 31);
        const uint32_t cb = ~(uint32_t)__builtin_amdgcn_readlane((int)c, 63);
        if (lane == 0) out[2 * p] = icrc_len_ok(((int)buf[w][0][16] << 8) | buf[w][0][17], stride) ? ca : 0u;
        if (lane == 32 && f < count) out[f] = icrc_len_ok(ipt, stride) ? cb : 0u;
        __builtin_amdgcn_wave_barrier();
        p = pn;
        if (p >= pairs) break;
    }
}

// masked_pos() as a bitmap of frame byte positions (10-13, 15, 22, 24, 25, 40, 41, 46)
constexpr uint64_t kIcrcMaskBits = (1ull << 10) | (1ull << 11) | (1ull << 12) | (1ull << 13) | (1ull << 15) |
                                   (1ull << 22) | (1ull << 24) | (1ull << 25) | (1ull << 40) | (1ull << 41) |
                                   (1ull << 46);

// OR the mask bytes into dw[k] = frame dword d0 + k, straight-line: the bitmap
// shifted to byte 4 d0, and each nibble spread to four byte masks (bit i -> byte i)
__device__ __forceinline__ void icrc_mask_regs(uint32_t (&dw)[10], int d0)
{
    // -28 .. 44 where any mask byte is in reach; a shift of 64 or more (a segment far
    // before the frame) is clamped to no bits, not left to the hardware's 6-bit shift
    const int s4 = 4 * d0;
    const uint64_t x = (d0 >= 12 || d0 <= -16) ? 0ull : (s4 >= 0 ? kIcrcMaskBits >> s4 : kIcrcMaskBits << (-s4));
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const uint32_t b = __builtin_amdgcn_ubfe(k < 8 ? lo : hi, 4 * (k & 7), 4);
        const uint32_t m = (b * 0x00204081u) & 0x01010101u;
        dw[k] |= (m << 8) - m;
    }
}

// icrc_mask_regs with the nibble -> byte-mask spread from a 16-entry LDS table
// (323 instead of 343 VALU per pair, 10 more LDS reads; $INCCL_ICRC_MASK_LDS=1)
__device__ __forceinline__ void icrc_mask_regs_lds(uint32_t (&dw)[10], int d0, const CrcLdsPair& t)
{
    const int s4 = 4 * d0;
    const uint64_t x = (d0 >= 12 || d0 <= -16) ? 0ull : (s4 >= 0 ? kIcrcMaskBits >> s4 : kIcrcMaskBits << (-s4));
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
#pragma unroll
    for (int k = 0; k < 10; ++k) dw[k] |= t.spread[__builtin_amdgcn_ubfe(k < 8 ? lo : hi, 4 * (k & 7), 4)];
}

// icrc_mask_regs_lds that also clears frame bytes 0-9 (dwords 0-2; bytes 10-11 of
// dword 2 are then set by its OR mask): dw = (dw & AND) | OR from a 32-entry table
// indexed by the dword's mask nibble and a "dword <= 2" bit, so that the CRC needs
// no per-byte zeroing of the leading bytes: 295 VALU per pair (the default)
__device__ __forceinline__ void icrc_mask_regs_zero(uint32_t (&dw)[10], int d0, const CrcLdsPair& t)
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

// ICRC, two frames per wave without LDS staging (the default): each lane loads its own 34-byte
// segment straight from the frame (two dwordx4 + two dword buffer loads at the
// segment's dword offset), the mask bytes are ORed in registers, and LDS holds
// only the tables.  Every memory instruction runs on every pass (a frame past
// the end, or malformed, gets a zero-size buffer: its loads return 0 and its
// store is dropped), so the waits stay one pass deep.  39 VGPRs and 20.7 KiB of
// LDS (k_icrc_pair: 50 and 39 KiB).  Same window, masks and
// results as k_icrc_pair.  Out-of-range segment words: a load partly before
// the frame covers only bytes below 10 (zeroed or masked), and the segment's
// last byte o + 33 <= 14 + ip_total - 5 keeps both dwordx4 inside the frame.
template <int kW, int kPP, int kMaskLds = 0>
__global__ __launch_bounds__(kWave* kW) void k_icrc_direct(const uint8_t* __restrict__ frames, int64_t stride,
                                                           int64_t count, uint32_t* __restrict__ out)
{
    __shared__ CrcLdsPair t;
    for (int i = threadIdx.x; i < kSeg2 * 2 * 16; i += blockDim.x) (&t.seg[0][0][0])[i] = (&g_seg34[0][0][0])[i];
    for (int i = threadIdx.x; i < 8 * 16 * 32; i += blockDim.x) (&t.lane_sh[0][0][0])[i] = (&g_lane_shift32[0][0][0])[i];
    if (threadIdx.x < 32) {
        const uint32_t m = ((threadIdx.x & 15u) * 0x00204081u) & 0x01010101u;
        if (threadIdx.x < 16) t.spread[threadIdx.x] = (m << 8) - m;
        t.andor[threadIdx.x][0] = threadIdx.x & 16u ? 0u : 0xFFFFFFFFu;
        t.andor[threadIdx.x][1] = (m << 8) - m;
    }
    __syncthreads();
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    const int half = lane >> 5, l = lane & 31;
    // a wave takes kPP consecutive pairs per pass (group q = pairs kPP q .. kPP q + kPP - 1),
    // all fetched one pass ahead: kPP pairs of loads in flight while a group's CRCs run
    const int64_t pairs = (count + 1) >> 1, groups = (pairs + kPP - 1) / kPP, step = (int64_t)gridDim.x * kW;
    int64_t q = (int64_t)blockIdx.x * kW + w;
    if (q >= groups) return;
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
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    auto fetch = [&](int64_t pp, uint32_t h, uint32_t (&dw)[10], int& o, bool& ok) {
        const int64_t f = 2 * pp + half;
        const int ipt = (int)(((h & 0xFFu) << 8) | ((h >> 8) & 0xFFu));
        ok = f < count && icrc_len_ok(ipt, stride);
        o = 10 + l * kSeg2 - (kWin - ipt);
        // the segment's dwords, inside this frame's row: a dword before the row (a
        // lane whose segment starts before byte 10) or past the frame's last dword
        // reads 0; the two dwordx4 never reach past the frame (header comment)
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
    uint32_t cur[kPP][10], hn[kPP];
    int o[kPP];
    bool ok[kPP];
#pragma unroll
    for (int j = 0; j < kPP; ++j) fetch(kPP * q + j, hdr(kPP * q + j), cur[j], o[j], ok[j]);
#pragma unroll
    for (int j = 0; j < kPP; ++j) hn[j] = hdr(kPP * (q + step) + j);
    // dropped stores: the loop is entered with its back edge's memory history
#pragma unroll
    for (int j = 0; j < kPP; ++j) __builtin_amdgcn_raw_buffer_store_b32(0u, ors, kOobOffset, 0, 0);
    for (;;) {
        const int64_t qn = q + step;
        uint32_t nxt[kPP][10];
        int on[kPP];
        bool okn[kPP];
#pragma unroll
        for (int j = 0; j < kPP; ++j) fetch(kPP * qn + j, hn[j], nxt[j], on[j], okn[j]);
#pragma unroll
        for (int j = 0; j < kPP; ++j) hn[j] = hdr(kPP * (qn + step) + j);
        uint32_t c[kPP];
#pragma unroll
        for (int j = 0; j < kPP; ++j) {
            if (kMaskLds == 2)
                icrc_mask_regs_zero(cur[j], o[j] >> 2, t);
            else if (kMaskLds == 1)
                icrc_mask_regs_lds(cur[j], o[j] >> 2, t);
            else
                icrc_mask_regs(cur[j], o[j] >> 2);
            c[j] = ok[j] ? icrc_half_regs<kMaskLds == 2>(cur[j], o[j], t, l) : 0u;
        }
#pragma unroll
        for (int j = 0; j < kPP; ++j) {
            uint32_t x = c[j];
            x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);
            x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);
            x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);
            x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false);
            x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
            const uint32_t ca = ~(uint32_t)__builtin_amdgcn_readlane((int)x, 31);
            const uint32_t cb = ~(uint32_t)__builtin_amdgcn_readlane((int)x, 63);
            // lane 0 writes frame 2 pp, lane 32 frame 2 pp + 1 (past the end: dropped)
            const int64_t pp = kPP * q + j;
            __builtin_amdgcn_raw_buffer_store_b32(ok[j] ? (half ? cb : ca) : 0u, ors,
                                                  l == 0 && pp < pairs ? (int)(4 * (2 * pp + half)) : kOobOffset, 0, 0);
        }
        q = qn;
        if (q >= groups) break;
#pragma unroll
        for (int j = 0; j < kPP; ++j) {
#pragma unroll
            for (int k = 0; k < 10; ++k) cur[j][k] = nxt[j][k];
            o[j] = on[j];
            ok[j] = okn[j];
        }
    }
}

__device__ __forceinline__ bool is_data_opcode(uint8_t op)
{
    return op == 0x00 || op == 0x01 || op == 0x02 || op == 0x04 || op == 0x07 || op == 0x08;   // nts.c:314-319
}
__device__ __forceinline__ bool is_write_first(uint8_t op) { return op == 0x06 || op == 0x0A; }   // nts.c:327-328

// Ingress (nts.c:303-483, root branch) in three passes that reproduce the
// reference's one-frame-at-a-time order: frame index within the batch = arrival
// order.  What a serial switch decides for frame f depends on which copies of
// its (psn, port) and of its PSN's other ports came BEFORE f, so:
//   claim   (a lane per frame) parse + validate; per (slot, port) an atomicMin
//           of a batch-tagged frame index finds the first copy in the batch
//   apply   (a wave per frame) the first copy of a pair whose port bit was not
//           set before the batch is the arrival that counts: it adds its payload
//           (nts.c:359-363) and keeps its RETH (:442).  The PSN completes at the
//           LAST of its ports' counted arrivals (the max over ports of the first
//           index; ports already in before the batch count as earlier than
//           every frame): that frame is COMPLETED (:365-372), the others
//           ABSORBED.  Every other copy is a retransmit (:353): REPLAY if the
//           slot completed before the batch or at an earlier frame of it
//           (:354-356), else DROPPED.
//   commit  (a lane per frame) the arrival bitmap: port bits of the counted
//           arrivals, and the result bit (:366) of the completing ones.
// The arrival bitmap is read (apply) and written (commit) in different
// launches, so every frame sees the state from before the batch.
constexpr int kActPending = 100;   // claim -> apply: a data frame still to classify
constexpr int kClaimBlock = 256;

// (~gen << 32) | (frame << 1) | wf: the minimum over a (slot, port)'s keys is the
// newest batch's earliest copy (the frame index dominates bit 0), and bit 0 tells
// apply where that copy's payload starts (byte 54, or 70 after a RETH) without
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
                      (unsigned long long)first_key(*s.gen + 1u, f, wf));
            act = kActPending;
        }
    }
    action[f] = act;
    psn_out[f] = psn;
}

// Apply, several frames per wave.  A one-frame wave is a chain of dependent
// round trips (its metadata -> its slot's bitmap and first copies -> the
// payloads -> the stores), and with 131 072 short waves that latency, not HBM,
// set the pass's time (102 us).  A wave now takes kApplyFrames consecutive
// frames and runs each stage for all of them before the next, so every round
// trip carries kApplyFrames frames' loads.  Template parameter: 2 by default
// (82 us per 131 072-frame batch, against 97 at 4 and 113 at 8, where the
// extra registers cost more occupancy than the shared round trips save;
// profiles/r03/apply_frames_sweep.txt); $INCCL_APPLY_FRAMES = 1, 4 or 8 for sweeps.

// payload word i of the frame at `fr`, its payload at byte 54 + 16*wf (2-byte
// aligned), network order -> host order (nts.c:361-363)
__device__ __forceinline__ uint32_t payload_word(const uint8_t* fr, uint32_t wf, int i)
{
    const uint16_t* d16 = reinterpret_cast<const uint16_t*>(fr + 54 + 16 * wf);
    return __builtin_bswap32((uint32_t)d16[2 * i] | ((uint32_t)d16[2 * i + 1] << 16));
}

// Payload words 4 lane .. 4 lane + 3, host order.  With 16-byte aligned rows
// (`wide`): the payload starts at 54 or 70, both 6 mod 16, so lane l loads the
// aligned 16-byte chunk holding payload bytes 16 l - 6 .. 16 l + 9 in ONE
// dwordx4 load and takes bytes 16 l + 10 .. 16 l + 15 from lane l+1's chunk
// (lane 63 reads those six bytes, still inside the frame, as two dwords).  The
// 2-byte-load fallback takes eight loads per lane.  Call in uniform control flow.
__device__ __forceinline__ void payload16(const uint8_t* fr, uint32_t wf, int lane, bool wide, uint32_t (&w)[4])
{
    if (wide) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const u4* c = reinterpret_cast<const u4*>(fr) + (3 + wf);
        const u4 a = c[lane];
        uint32_t n0 = (uint32_t)__shfl_down((int)a.x, 1, kWave), n1 = (uint32_t)__shfl_down((int)a.y, 1, kWave);
        if (lane == kWave - 1) {
            const uint32_t* t = reinterpret_cast<const uint32_t*>(c + kWave);
            n0 = t[0];
            n1 = t[1];
        }
        w[0] = __builtin_bswap32(__builtin_amdgcn_alignbyte(a.z, a.y, 2));
        w[1] = __builtin_bswap32(__builtin_amdgcn_alignbyte(a.w, a.z, 2));
        w[2] = __builtin_bswap32(__builtin_amdgcn_alignbyte(n0, a.w, 2));
        w[3] = __builtin_bswap32(__builtin_amdgcn_alignbyte(n1, n0, 2));
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = payload_word(fr, wf, 4 * lane + j);
    }
}

template <int kApplyFrames, bool kNtAgg = true>
__global__ __launch_bounds__(kWave * 16) void k_ingress_apply(InccSwitchState s,
                                                                         const uint8_t* __restrict__ frames,
                                                                         int64_t stride, int64_t count,
                                                                         const int32_t* __restrict__ ports,
                                                                         int32_t* __restrict__ action,
                                                                         const uint32_t* __restrict__ psns, bool wide)
{
    const int w = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    const int64_t f0 = ((int64_t)blockIdx.x * (blockDim.x / kWave) + w) * kApplyFrames;
    if (f0 >= count) return;
    const int fan = s.fan_in;
    const uint32_t tag = ~(*s.gen + 1u), result_bit = 1u << fan;   // this batch's generation (k_ingress_commit)
    // stage A: each frame's action, port and PSN
    int act[kApplyFrames], port[kApplyFrames];
    uint32_t psn[kApplyFrames];
#pragma unroll
    for (int k = 0; k < kApplyFrames; ++k) {
        const bool in = f0 + k < count;
        act[k] = in ? action[f0 + k] : 0;
        port[k] = in ? ports[f0 + k] : 0;
        psn[k] = in ? psns[f0 + k] : 0;
    }
    // stage B: the slot as it was before the batch, and lane p < fan_in: the
    // first-copy key of port p
    uint32_t pre[kApplyFrames];
    uint64_t key[kApplyFrames];
#pragma unroll
    for (int k = 0; k < kApplyFrames; ++k) {
        const bool live = act[k] == kActPending;
        const uint32_t slot = psn[k] & (s.slots - 1);
        pre[k] = live ? s.arrival[slot] : 0u;
        key[k] = live && lane < fan ? s.first[(size_t)slot * fan + lane] : 0ull;
    }
    // stage C: classify (nts.c:353-372) and find the slot leaders
    int out_act[kApplyFrames];
    bool lead[kApplyFrames];
    uint64_t counted_ports[kApplyFrames];
    uint32_t first_of[kApplyFrames], done_at[kApplyFrames];
#pragma unroll
    for (int k = 0; k < kApplyFrames; ++k) {
        const int64_t f = f0 + k;
        const bool live = act[k] == kActPending;
        const uint32_t bit = 1u << port[k];
        // lane p < fan_in: when port p's counted arrival happens, as 1 + frame
        // index; 0 = before the batch, ~0 = not by the end of the batch
        uint32_t at = 0, mine = 0xFFFFFFFFu, fo = 0xFFFFFFFFu;
        bool counted = false;
        if (lane < fan) {
            const uint64_t e = key[k];
            const bool in_batch = (uint32_t)(e >> 32) == tag;
            const uint32_t ef = ((uint32_t)e) >> 1;
            at = (pre[k] & (1u << lane)) ? 0u : (in_batch ? ef + 1u : 0xFFFFFFFFu);
            mine = in_batch ? ef : 0xFFFFFFFFu;
            fo = (uint32_t)e;                                   // frame << 1 | wf
            counted = in_batch && !(pre[k] & (1u << lane));
        }
        counted_ports[k] = __ballot(counted);
        first_of[k] = fo;
        mine = (uint32_t)__shfl((int)mine, port[k] & (kWave - 1), kWave);
        uint32_t d = at;                                        // max over ports: the completing arrival
#pragma unroll
        for (int o = 16; o >= 1; o >>= 1) {
            const uint32_t v = (uint32_t)__shfl_xor((int)d, o, kWave);
            d = v > d ? v : d;
        }
        done_at[k] = d = (uint32_t)__shfl((int)d, 0, kWave);
        const bool arrival = live && !(pre[k] & bit) && mine == (uint32_t)f;   // the counted arrival: nts.c:359-363
        if (arrival) {
            out_act[k] = (d == (uint32_t)f + 1u) ? INCCL_SW_COMPLETED : INCCL_SW_ABSORBED;   // nts.c:365
        } else {                                                 // retransmit: nts.c:353-357
            const bool done_before = (pre[k] & result_bit) != 0;
            const bool done_earlier = d != 0u && d != 0xFFFFFFFFu && d - 1u < (uint32_t)f;
            out_act[k] = (done_before || done_earlier) ? INCCL_SW_REPLAY : INCCL_SW_DROPPED;
        }
        // The slot's counted arrivals of this batch are summed by ONE wave --
        // the one holding the lowest counted port's frame -- into the slot's
        // partial from earlier batches, with plain loads and stores: the same
        // wrap-around sum as one atomic add per arrival (nts.c:361-363 /
        // :443-445; integer addition commutes), without the atomics.
        lead[k] = arrival && port[k] == __builtin_ctzll(counted_ports[k]);
        // (the shuffle runs on every lane: a bpermute from a lane that is
        // inactive in a divergent branch does not return that lane's value)
        const uint32_t wf = (uint32_t)__shfl((int)fo, port[k] & (kWave - 1), kWave) & 1u;
        if (arrival && lane < 4) {                               // reth_keeper, nts.c:442
            if (wf) {
                const uint16_t* r = reinterpret_cast<const uint16_t*>(frames + f * stride + 54);
                s.reth[((size_t)(psn[k] & (s.slots - 1)) * fan + port[k]) * 4 + lane] =
                    (uint32_t)r[2 * lane] | ((uint32_t)r[2 * lane + 1] << 16);
            }
        }
    }
    // stage D: the leaders' sums.  Every leader's slot partial and its two lowest
    // counted ports' payloads are loaded before any is added (fan-in 2 needs no
    // more); further ports, if any, follow.  Lane l owns words 4 l .. 4 l + 3:
    // one dwordx4 per lane moves the slot's 1 KiB.
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    uint32_t acc[kApplyFrames][4], p0[kApplyFrames][4], p1[kApplyFrames][4];
#pragma unroll
    for (int k = 0; k < kApplyFrames; ++k) {
        if (!lead[k]) continue;
        // a slot whose arrival bitmap was empty before the batch holds zeros
        // (reset, or recycled since its last use: nts.c:235-242), so its partial
        // is not read -- in the common case, every port of a PSN in one batch,
        // that saves a quarter of the pass's bytes
        if (pre[k] != 0u) {
            const u4 g = reinterpret_cast<const u4*>(s.agg + (size_t)(psn[k] & (s.slots - 1)) * kLanes)[lane];
            acc[k][0] = g.x; acc[k][1] = g.y; acc[k][2] = g.z; acc[k][3] = g.w;
        } else {
            acc[k][0] = acc[k][1] = acc[k][2] = acc[k][3] = 0u;
        }
        uint64_t m = counted_ports[k];
        const uint32_t e0 = (uint32_t)__shfl((int)first_of[k], __builtin_ctzll(m), kWave);
        m &= m - 1;
        payload16(frames + (int64_t)(e0 >> 1) * stride, e0 & 1u, lane, wide, p0[k]);
        if (m) {
            const uint32_t e1 = (uint32_t)__shfl((int)first_of[k], __builtin_ctzll(m), kWave);
            payload16(frames + (int64_t)(e1 >> 1) * stride, e1 & 1u, lane, wide, p1[k]);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) p1[k][j] = 0u;
        }
    }
#pragma unroll
    for (int k = 0; k < kApplyFrames; ++k) {
        if (!lead[k]) continue;
        const uint32_t slot = psn[k] & (s.slots - 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[k][j] += p0[k][j] + p1[k][j];
        uint64_t m = counted_ports[k];
        m &= m - 1;
        m &= m - 1;
        for (; m; m &= m - 1) {                                  // ports beyond the first two
            const uint32_t e = (uint32_t)__shfl((int)first_of[k], __builtin_ctzll(m), kWave);
            uint32_t pq[4];
            payload16(frames + (int64_t)(e >> 1) * stride, e & 1u, lane, wide, pq);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[k][j] += pq[j];
        }
        {
            const u4 o = u4{acc[k][0], acc[k][1], acc[k][2], acc[k][3]};
            u4* dst = reinterpret_cast<u4*>(s.agg + (size_t)slot * kLanes) + lane;
            if constexpr (kNtAgg)   // non-temporal: 1.3 us off egress (profiles/r03/store_policy/)
                __builtin_nontemporal_store(o, dst);
            else
                *dst = o;
        }
        // clear_state_data(psn + WINDOW) when the PSN completes in this batch
        // (nts.c:235-242, :367): slot psn + slots/2, which no frame of the batch
        // touches (a batch's PSNs are less than slots/2 apart).  Its bitmap, degree
        // and RETH keeper are cleared; its 1 KiB of aggregator words are not: a
        // slot whose bitmap is empty is summed from zero without reading them
        // (above), and nothing else reads a slot before its next counted arrival
        // rewrites them (egress reads completed slots only) -- 67 MB fewer stores
        // per 131 072-frame batch
        if (done_at[k] != 0xFFFFFFFFu) {
            const uint32_t rs = (psn[k] + (s.slots >> 1)) & (s.slots - 1);
            for (int i = lane; i < fan * 4; i += kWave) s.reth[(size_t)rs * fan * 4 + i] = 0;
            if (lane == 0) {
                s.arrival[rs] = 0;
                s.degree[rs] = 0;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kApplyFrames; ++k)
        if (lane == 0 && act[k] == kActPending && f0 + k < count) action[f0 + k] = out_act[k];
}

__global__ __launch_bounds__(kClaimBlock) void k_ingress_commit(InccSwitchState s, int64_t count,
                                                                const int32_t* __restrict__ ports,
                                                                const int32_t* __restrict__ action,
                                                                const uint32_t* __restrict__ psns)
{
    const int64_t f = (int64_t)blockIdx.x * kClaimBlock + threadIdx.x;
    // the batch is done with its generation (claim and apply ran before this
    // launch): the next batch's is one higher
    if (f == 0) *s.gen = *s.gen + 1u;
    if (f >= count) return;
    const int act = action[f];
    if (act != INCCL_SW_ABSORBED && act != INCCL_SW_COMPLETED) return;
    const uint32_t slot = psns[f] & (s.slots - 1);
    atomicOr(&s.arrival[slot], (1u << ports[f]) | (act == INCCL_SW_COMPLETED ? 1u << s.fan_in : 0u));   // nts.c:359, :366
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
// host: CRC tables (util.c:141-159) and the zero-append operators per tree level
// ---------------------------------------------------------------------------
uint32_t host_tab[256];
uint32_t host_seg[kSeg][2][16];
uint32_t host_segb[kSeg][256];
uint32_t host_lane_shift[8][16][kWave];
uint32_t host_lane16[8][16][kWave];
uint32_t host_seg34[kSeg2][2][16];
uint32_t host_lane_shift32[8][16][32];
uint32_t host_var[5 + kVarBytes][2][16];
uint32_t host_z1024[8][16];
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
    for (int j = 0; j < kSeg; ++j)
        for (uint32_t v = 0; v < 256; ++v) host_segb[j][v] = zeros_append(host_tab[v], kSeg - 1 - j);
    // Z_n is linear: Z_{n+17}(x) = Z_17(Z_n(x)), so lanes are filled from 63 down
    for (int n = 0; n < 8; ++n)
        for (uint32_t v = 0; v < 16; ++v) {
            uint32_t x = v << (4 * n);
            for (int lane = kWave - 1; lane >= 0; --lane) {
                host_lane_shift[n][v][lane] = x;
                x = zeros_append(x, kSeg);
            }
        }
    // the paired ICRC (k_icrc_pair): 34-byte segments, Z_{34 (31 - lane')}
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
    // egress by linearity (k_egress): Z_{16 (63 - lane)}, each variable header
    // byte's contribution shifted to the message end, and Z_1024
    for (int n = 0; n < 8; ++n)
        for (uint32_t v = 0; v < 16; ++v) {
            uint32_t x = v << (4 * n);
            host_z1024[n][v] = zeros_append(x, 1024);
            for (int lane = kWave - 1; lane >= 0; --lane) {
                host_lane16[n][v][lane] = x;
                x = zeros_append(x, 16);
            }
        }
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
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_lane_shift), host_lane_shift, sizeof(host_lane_shift));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_segb), host_segb, sizeof(host_segb));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_lane16), host_lane16, sizeof(host_lane16));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_var), host_var, sizeof(host_var));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_z1024), host_z1024, sizeof(host_z1024));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_seg34), host_seg34, sizeof(host_seg34));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_lane_shift32), host_lane_shift32, sizeof(host_lane_shift32));
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

// persistent blocks per CU (43-46 KiB of LDS each, so up to three fit).  The
// ICRC kernel is fastest at three (65.9 vs 78.4 us per 131 072 frames at two).
// Egress was fastest at two while it staged every output frame in LDS (189 us
// at three); with the payload stored from registers it takes three.
// INCCL_ICRC_BLOCKS_PER_CU / INCCL_EGRESS_BLOCKS_PER_CU override for sweeps.
int blocks_per_cu(const char* env, int dflt)
{
    const char* e = getenv(env);
    const int v = e ? atoi(e) : 0;
    return (v >= 1 && v <= 8) ? v : dflt;
}

// waves per apply workgroup: 4 by default, $INCCL_APPLY_WPB = 1, 2, 8 or 16 for sweeps
int apply_wpb()
{
    static const int v = [] {
        const char* e = getenv("INCCL_APPLY_WPB");
        const int x = e ? atoi(e) : kWavesPerBlock;
        return (x == 1 || x == 2 || x == 4 || x == 8 || x == 16) ? x : kWavesPerBlock;
    }();
    return v;
}

inline int grid_for(int64_t waves)
{
    const int64_t blocks = (waves + apply_wpb() - 1) / apply_wpb();
    return (int)(blocks < 1 ? 1 : blocks);
}

}  // namespace

extern "C" {

int inccl_k_frames_init(void) { return ensure_tables(); }

int inccl_k_icrc(const uint8_t* frames, size_t stride, size_t count, uint32_t* out, void* stream)
{
    if ((frames == nullptr || out == nullptr) && count) return INCCL_ERR_ARG;
    if (count == 0) return 0;
    if ((stride & 3) || stride < INCCL_FRAME_MIN_STRIDE || ((uintptr_t)frames & 3)) return INCCL_ERR_ARG;
    int rc = ensure_tables();
    if (rc) return rc;
    static const bool byte_tables = [] {
        const char* e = getenv("INCCL_ICRC_BYTE_TABLES");
        return e && atoi(e) != 0;
    }();
    // 16-wave blocks share one copy of the tables: two per CU hold 32 waves (the
    // most a CU runs), where 8-wave blocks fit three (24 waves) in the LDS;
    // $INCCL_ICRC_WAVES=8 selects the 8-wave form (A/B)
    static const int waves = [] {
        const char* e = getenv("INCCL_ICRC_WAVES");
        return e && atoi(e) == 8 ? 8 : 16;
    }();
    const int64_t blocks = ((int64_t)count + waves - 1) / waves;
    // persistent: tables loaded once per block
    const int64_t cap =
        (int64_t)num_cus() * blocks_per_cu("INCCL_ICRC_BLOCKS_PER_CU", waves == 16 ? 2 : (byte_tables ? 2 : 3));
    const int grid = (int)(blocks < cap ? blocks : cap);
    hipStream_t st = (hipStream_t)stream;
    // two frames per wave (k_icrc_pair, 49.0 vs 52.8-54.9 us per 131 072 frames);
    // $INCCL_ICRC_PAIR=0 selects one frame per wave (A/B)
    static const bool pair = [] {
        const char* e = getenv("INCCL_ICRC_PAIR");
        return !(e && atoi(e) == 0);
    }();
    // two frames per wave without LDS staging (k_icrc_direct), the default: 47.9-49.8 vs
    // 49.2-54.4 us for k_icrc_pair over this round's runs (profiles/r03/icrc_direct/);
    // $INCCL_ICRC_DIRECT=0 selects k_icrc_pair, $INCCL_ICRC_PAIRS_PER_PASS=2 two pairs a
    // pass (50.9-51.4 us: more bytes in flight do not help)
    static const bool direct = [] {
        const char* e = getenv("INCCL_ICRC_DIRECT");
        return !(e && atoi(e) == 0);
    }();
    if (pair && direct && !byte_tables && count < (1ull << 29) && stride < (1ull << 29)) {   // 32-bit offsets
        const int64_t pairs = ((int64_t)count + 1) / 2, need = (pairs + 7) / 8;
        const int64_t pcap = (int64_t)num_cus() * blocks_per_cu("INCCL_ICRC_BLOCKS_PER_CU", 4);
        static const int pp = [] {
            const char* e = getenv("INCCL_ICRC_PAIRS_PER_PASS");
            return e && atoi(e) == 2 ? 2 : 1;
        }();
        const int64_t groups = (pairs + pp - 1) / pp, gneed = (groups + 7) / 8;
        // mask bytes and the zeroed leading bytes from one 32-entry (AND, OR) LDS table
        // (2, the default): 43.6-47.0 vs 48.0-49.2 us for the 16-entry mask table with
        // per-byte zeroing (1), itself 46.0-48.2 vs 47.0-50.8 us for the VALU spread (0),
        // in paired runs (profiles/r03/icrc_mask_lds/, icrc_mask_zero/); $INCCL_ICRC_MASK_LDS
        // selects 0 or 1 for A/B
        static const int mask_lds = [] {
            const char* e = getenv("INCCL_ICRC_MASK_LDS");
            return e ? atoi(e) : 2;
        }();
        if (pp == 1 && mask_lds == 2)
            hipLaunchKernelGGL((k_icrc_direct<8, 1, 2>), dim3((unsigned)(need < pcap ? need : pcap)), dim3(kWave * 8), 0,
                               st, frames, (int64_t)stride, (int64_t)count, out);
        else if (pp == 1 && mask_lds == 1)
            hipLaunchKernelGGL((k_icrc_direct<8, 1, 1>), dim3((unsigned)(need < pcap ? need : pcap)), dim3(kWave * 8), 0,
                               st, frames, (int64_t)stride, (int64_t)count, out);
        else if (pp == 1)
            hipLaunchKernelGGL((k_icrc_direct<8, 1>), dim3((unsigned)(need < pcap ? need : pcap)), dim3(kWave * 8), 0, st,
                               frames, (int64_t)stride, (int64_t)count, out);
        else
            hipLaunchKernelGGL((k_icrc_direct<8, 2>), dim3((unsigned)(gneed < pcap ? gneed : pcap)), dim3(kWave * 8), 0,
                               st, frames, (int64_t)stride, (int64_t)count, out);
        return (int)hipGetLastError();
    }
    if (pair && !byte_tables) {
        // 8-wave blocks: 2 x 1152 B of staging per wave + 20.6 KiB of tables = 39 KiB
        const int64_t pairs = ((int64_t)count + 1) / 2, need = (pairs + 7) / 8;
        const int64_t pcap = (int64_t)num_cus() * 4;   // four per CU: 32 waves
        hipLaunchKernelGGL((k_icrc_pair<8>), dim3((unsigned)(need < pcap ? need : pcap)), dim3(kWave * 8), 0, st, frames,
                           (int64_t)stride, (int64_t)count, out);
        return (int)hipGetLastError();
    }
    if (byte_tables)
        hipLaunchKernelGGL((k_icrc<true, 8>), dim3(grid), dim3(kWave * 8), 0, st, frames, (int64_t)stride, (int64_t)count, out);
    else if (waves == 16)
        hipLaunchKernelGGL((k_icrc<false, 16>), dim3(grid), dim3(kWave * 16), 0, st, frames, (int64_t)stride, (int64_t)count,
                           out);
    else
        hipLaunchKernelGGL((k_icrc<false, 8>), dim3(grid), dim3(kWave * 8), 0, st, frames, (int64_t)stride, (int64_t)count,
                           out);
    return (int)hipGetLastError();
}

int inccl_k_switch_ingress(const InccSwitchState* s, const uint8_t* frames, size_t stride, size_t count,
                           const int32_t* ports, int32_t* action, uint32_t* psn_out, void* stream)
{
    if (count == 0) return 0;
    if (!s || !frames || !ports || !action || !psn_out || (stride & 3) || stride < INCCL_FRAME_MIN_STRIDE ||
        ((uintptr_t)frames & 3) || count >= 0x7FFFFFFFull)
        return INCCL_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    const dim3 lanes((unsigned)(((int64_t)count + kClaimBlock - 1) / kClaimBlock));
    hipLaunchKernelGGL(k_ingress_claim, lanes, dim3(kClaimBlock), 0, st, *s, frames, (int64_t)stride, (int64_t)count,
                       ports, action, psn_out);
    // 16-byte aligned rows: apply loads each payload with one dwordx4 per lane
    const bool wide = ((uintptr_t)frames & 15) == 0 && (stride & 15) == 0;
    static const int apply_frames = [] {
        const char* e = getenv("INCCL_APPLY_FRAMES");
        const int v = e ? atoi(e) : 2;
        return (v == 1 || v == 4 || v == 8) ? v : 2;
    }();
    // $INCCL_APPLY_NT=0: plain aggregate stores (A/B of the non-temporal default)
    static const bool apply_nt = [] {
        const char* e = getenv("INCCL_APPLY_NT");
        return !(e && atoi(e) == 0);
    }();
    const int64_t waves = ((int64_t)count + apply_frames - 1) / apply_frames;
    if (apply_frames == 1)
        hipLaunchKernelGGL(k_ingress_apply<1>, dim3(grid_for(waves)), dim3(kWave * apply_wpb()), 0, st, *s, frames,
                           (int64_t)stride, (int64_t)count, ports, action, psn_out, wide);
    else if (apply_frames == 4)
        hipLaunchKernelGGL(k_ingress_apply<4>, dim3(grid_for(waves)), dim3(kWave * apply_wpb()), 0, st, *s, frames,
                           (int64_t)stride, (int64_t)count, ports, action, psn_out, wide);
    else if (apply_frames == 2 && !apply_nt)
        hipLaunchKernelGGL((k_ingress_apply<2, false>), dim3(grid_for(waves)), dim3(kWave * apply_wpb()), 0, st, *s,
                           frames, (int64_t)stride, (int64_t)count, ports, action, psn_out, wide);
    else if (apply_frames == 2)
        hipLaunchKernelGGL(k_ingress_apply<2>, dim3(grid_for(waves)), dim3(kWave * apply_wpb()), 0, st, *s, frames,
                           (int64_t)stride, (int64_t)count, ports, action, psn_out, wide);
    else if (apply_frames == 8)
        hipLaunchKernelGGL(k_ingress_apply<8>, dim3(grid_for(waves)), dim3(kWave * apply_wpb()), 0, st, *s, frames,
                           (int64_t)stride, (int64_t)count, ports, action, psn_out, wide);
    else
        hipLaunchKernelGGL(k_ingress_apply<2>, dim3(grid_for(waves)), dim3(kWave * apply_wpb()), 0, st, *s, frames,
                           (int64_t)stride, (int64_t)count, ports, action, psn_out, wide);
    hipLaunchKernelGGL(k_ingress_commit, lanes, dim3(kClaimBlock), 0, st, *s, (int64_t)count, ports, action, psn_out);
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
    // persistent grid: the CRC tables are loaded once per block
    const int64_t need = ((int64_t)count + kEgressWaves - 1) / kEgressWaves;
    const int64_t cap = (int64_t)num_cus() * blocks_per_cu("INCCL_EGRESS_BLOCKS_PER_CU", 3);
    const int eg = (int)(need < cap ? (need < 1 ? 1 : need) : cap);
    // fan-in 2, 3, 4, 8: the straight-line kernel (k_egress_fixed); others, or
    // $INCCL_EGRESS_GENERIC=1 (A/B), the generic one
    static const bool generic = [] {
        const char* e = getenv("INCCL_EGRESS_GENERIC");
        return e && atoi(e) != 0;
    }();
    const bool o16 = ((out_stride & 15) == 0) && (((uintptr_t)out & 15) == 0);
    // non-temporal output stores (the frames are not re-read here): egress 65.3 vs
    // 71.0 us (sc1 70.2-70.4, sc1|nt 67.6-68.0), and the next batch's apply 55.5 vs
    // 65.2 us, no longer behind 144 MB of dirty lines (profiles/r03/store_policy/);
    // $INCCL_EGRESS_NT=0 for A/B
    static const bool nt = [] {
        const char* e = getenv("INCCL_EGRESS_NT");
        return !(e && atoi(e) == 0);
    }();
    const dim3 g(eg), b(kWave * kEgressWaves);
    const int64_t is = (int64_t)in_stride, os = (int64_t)out_stride, n = (int64_t)count;
#define INCCL_EGRESS_FIXED(F)                                                                                   \
    case F:                                                                                                     \
        if (o16 && nt)                                                                                          \
            hipLaunchKernelGGL((k_egress_fixed<F, true, kAuxNt>), g, b, 0, st, *s, in_frames, is, n, ports,     \
                               action, psns, tmpl, out, os, out_len);                                           \
        else if (o16)                                                                                           \
            hipLaunchKernelGGL((k_egress_fixed<F, true>), g, b, 0, st, *s, in_frames, is, n, ports, action,    \
                               psns, tmpl, out, os, out_len);                                                   \
        else if (nt)                                                                                            \
            hipLaunchKernelGGL((k_egress_fixed<F, false, kAuxNt>), g, b, 0, st, *s, in_frames, is, n, ports,    \
                               action, psns, tmpl, out, os, out_len);                                           \
        else                                                                                                    \
            hipLaunchKernelGGL((k_egress_fixed<F, false>), g, b, 0, st, *s, in_frames, is, n, ports, action,   \
                               psns, tmpl, out, os, out_len);                                                   \
        return (int)hipGetLastError();
    if (!generic) {
        switch (s->fan_in) {
            INCCL_EGRESS_FIXED(2)
            INCCL_EGRESS_FIXED(3)
            INCCL_EGRESS_FIXED(4)
            INCCL_EGRESS_FIXED(8)
        default: break;
        }
    }
#undef INCCL_EGRESS_FIXED
    hipLaunchKernelGGL(k_egress, g, b, 0, st, *s, in_frames, is, n, ports, action, psns, tmpl, out, os, out_len);
    return (int)hipGetLastError();
}

}  // extern "C"
