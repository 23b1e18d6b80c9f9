// tune_icrc.hip -- the standalone RoCE ICRC (util.c:250-286) variants the
// product's k_icrc was chosen over, each checked and timed:
//   one frame per wave, frame staged in LDS, nibble or byte tables, 8- or 16-wave blocks (k_icrc_lds);
//   two frames per wave, staged in LDS (k_icrc_pair);
//   two frames per wave, no LDS staging (k_icrc_direct), one or two pairs per pass, the mask bytes
//   from the VALU spread (0), a 16-entry LDS table (1) or the (AND, OR) table that also clears the
//   leading bytes (2: the product).
// Every variant's ICRCs are compared with the product's inccl_icrc_frames (libinccl_amd.so, itself
// checked against the oracle in tests/test_gpu_switch.py) and with a byte-serial host CRC, over random
// frames of every IP length class, 16- and 4-byte aligned row strides and odd counts; then each is
// timed on 131 072 frames of 1082 / 1098 bytes (the switch bench's batch).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I container_inc_amd/csrc tools/tune/tune_icrc.hip \
//        -o tools/tune/tune_icrc -L container_inc_amd -linccl_amd -Wl,-rpath,$PWD/container_inc_amd
// Measured history: DESIGN.md "ICRC" (profiles/r03/icrc_*).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "inccl_amd.h"

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

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
__global__ __launch_bounds__(kWave* kIcrcWaves) void k_icrc_lds(const uint8_t* __restrict__ frames, int64_t stride,
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

uint32_t host_tab[256];
uint32_t host_seg[kSeg][2][16];
uint32_t host_segb[kSeg][256];
uint32_t host_lane_shift[8][16][kWave];
uint32_t host_seg34[kSeg2][2][16];
uint32_t host_lane_shift32[8][16][32];
bool g_tables_ready[64];
std::mutex g_tables_mu;

uint32_t zeros_append(uint32_t c, int nbytes)
{
    for (int i = 0; i < nbytes; ++i) c = (c >> 8) ^ host_tab[c & 0xFF];
    return c;
}

int masked_pos_host(int i)
{
    static const int pos[kNumMasked] = {10, 11, 12, 13, 15, 22, 24, 25, 40, 41, 46};
    return pos[i];
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
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_seg), host_seg, sizeof(host_seg));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_lane_shift), host_lane_shift, sizeof(host_lane_shift));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_segb), host_segb, sizeof(host_segb));
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


// the ICRC the hard way: the message is 4 x 0xFF, then frame bytes 14 .. 14 + ip_total - 5 with the
// masked bytes (tos, ttl, IP checksum, UDP checksum, BTH resv8a) as 0xFF; raw CRC-32 from 0, inverted
uint32_t host_icrc(const uint8_t* f, int64_t stride)
{
    const int ipt = (f[16] << 8) | f[17];
    if (ipt < 28 || ipt > kWin || 14 + ipt > kFrameMax || 14 + ipt > stride) return 0;
    uint32_t c = 0;
    auto feed = [&](uint32_t b) { c = (c >> 8) ^ host_tab[(c ^ b) & 0xFF]; };
    for (int i = 0; i < 4; ++i) feed(0xFF);
    for (int i = 14; i < 14 + ipt - 4; ++i) {
        bool m = false;
        for (int k = 4; k < kNumMasked; ++k) m = m || i == masked_pos_host(k);
        feed(m ? 0xFFu : f[i]);
    }
    return ~c;
}

typedef void (*Launch)(const uint8_t*, int64_t, int64_t, uint32_t*, hipStream_t);

template <bool kByte, int kW>
void run_lds(const uint8_t* fr, int64_t stride, int64_t n, uint32_t* out, hipStream_t st)
{
    const int64_t blocks = (n + kW - 1) / kW, cap = (int64_t)num_cus() * (kW == 16 ? 2 : (kByte ? 2 : 3));
    hipLaunchKernelGGL((k_icrc_lds<kByte, kW>), dim3((unsigned)(blocks < cap ? blocks : cap)), dim3(kWave * kW), 0, st,
                       fr, stride, n, out);
}
void run_pair(const uint8_t* fr, int64_t stride, int64_t n, uint32_t* out, hipStream_t st)
{
    const int64_t need = ((n + 1) / 2 + 7) / 8, cap = (int64_t)num_cus() * 4;
    hipLaunchKernelGGL((k_icrc_pair<8>), dim3((unsigned)(need < cap ? need : cap)), dim3(kWave * 8), 0, st, fr, stride,
                       n, out);
}
template <int kPP, int kMask>
void run_direct(const uint8_t* fr, int64_t stride, int64_t n, uint32_t* out, hipStream_t st)
{
    const int64_t groups = ((n + 1) / 2 + kPP - 1) / kPP, need = (groups + 7) / 8, cap = (int64_t)num_cus() * 4;
    hipLaunchKernelGGL((k_icrc_direct<8, kPP, kMask>), dim3((unsigned)(need < cap ? need : cap)), dim3(kWave * 8), 0,
                       st, fr, stride, n, out);
}
void run_product(const uint8_t* fr, int64_t stride, int64_t n, uint32_t* out, hipStream_t st)
{
    if (inccl_icrc_frames(fr, (size_t)stride, (size_t)n, out, st) != 0) {
        fprintf(stderr, "inccl_icrc_frames: %s\n", inccl_last_error());
        exit(1);
    }
}

struct Variant {
    const char* name;
    Launch fn;
};
const Variant kVariants[] = {
    {"product inccl_icrc_frames", run_product},
    {"lds nibble 16 waves", run_lds<false, 16>},
    {"lds nibble 8 waves", run_lds<false, 8>},
    {"lds byte tables 8 waves", run_lds<true, 8>},
    {"pair lds", run_pair},
    {"direct mask valu", run_direct<1, 0>},
    {"direct mask lds", run_direct<1, 1>},
    {"direct and-or table", run_direct<1, 2>},
    {"direct two pairs per pass", run_direct<2, 0>},
};

uint64_t rng_state = 0x9E3779B97F4A7C15ull;
uint32_t rnd()
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return (uint32_t)rng_state;
}

// rows of random bytes with a given IP total length at bytes 16-17
std::vector<uint8_t> make_rows(int64_t n, int64_t stride, const std::vector<int>& lens)
{
    std::vector<uint8_t> h((size_t)(n * stride));
    for (auto& b : h) b = (uint8_t)rnd();
    for (int64_t i = 0; i < n; ++i) {
        const int ipt = lens[(size_t)i % lens.size()];
        h[(size_t)(i * stride + 16)] = (uint8_t)(ipt >> 8);
        h[(size_t)(i * stride + 17)] = (uint8_t)ipt;
    }
    return h;
}

int check_all()
{
    int bad = 0;
    std::vector<int> lens;
    for (int l = 28; l <= 60; ++l) lens.push_back(l);
    for (int i = 0; i < 60; ++i) lens.push_back(28 + (int)(rnd() % (kWin - 27)));
    for (int l = 1060; l <= kWin; ++l) lens.push_back(l);
    lens.push_back(1084);
    lens.push_back(1068);
    const int64_t strides[] = {1100, 1104, 1152, 1240};
    const int64_t counts[] = {1, 5, 7, 9, 3001};
    for (int64_t stride : strides)
        for (int64_t n : counts) {
            std::vector<uint8_t> h = make_rows(n, stride, lens);
            uint8_t* d = nullptr;
            uint32_t* o = nullptr;
            CHECK(hipMalloc(&d, h.size()));
            CHECK(hipMalloc(&o, 4 * n));
            CHECK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
            std::vector<uint32_t> want((size_t)n), got((size_t)n);
            for (int64_t i = 0; i < n; ++i) want[(size_t)i] = host_icrc(&h[(size_t)(i * stride)], stride);
            for (const Variant& v : kVariants) {
                CHECK(hipMemset(o, 0xA5, 4 * n));
                v.fn(d, stride, n, o, 0);
                CHECK(hipDeviceSynchronize());
                CHECK(hipMemcpy(got.data(), o, 4 * n, hipMemcpyDeviceToHost));
                int64_t mism = 0;
                for (int64_t i = 0; i < n; ++i) mism += got[(size_t)i] != want[(size_t)i];
                if (mism) {
                    printf("MISMATCH %s stride %lld count %lld: %lld frames\n", v.name, (long long)stride, (long long)n,
                           (long long)mism);
                    ++bad;
                }
            }
            CHECK(hipFree(d));
            CHECK(hipFree(o));
        }
    printf("{\"check\": \"%s\", \"variants\": %d}\n", bad ? "FAILED" : "ok", (int)(sizeof(kVariants) / sizeof(kVariants[0])));
    return bad;
}

void time_all(int reps)
{
    const int64_t n = 131072, stride = 1152;
    std::vector<int> lens = {1084, 1068, 1068, 1068};   // one WRITE_FIRST (1098-B frame) in four, as the switch bench
    std::vector<uint8_t> h = make_rows(n, stride, lens);
    uint8_t* d = nullptr;
    uint32_t* o = nullptr;
    CHECK(hipMalloc(&d, h.size()));
    CHECK(hipMalloc(&o, 4 * n));
    CHECK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < reps; ++rep)
        for (const Variant& v : kVariants) {
            for (int i = 0; i < 3; ++i) v.fn(d, stride, n, o, 0);
            CHECK(hipEventRecord(e0, 0));
            const int iters = 20;
            for (int i = 0; i < iters; ++i) v.fn(d, stride, n, o, 0);
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double us = 1e3 * ms / iters;
            printf("{\"variant\": \"%s\", \"frames\": %lld, \"us\": %.2f, \"frame_GBs\": %.1f}\n", v.name, (long long)n, us,
                   n * 1084.0 / (us * 1e-6) / 1e9);
        }
    CHECK(hipFree(d));
    CHECK(hipFree(o));
}

}  // namespace

int main(int argc, char** argv)
{
    CHECK(hipSetDevice(0));
    if (ensure_tables() != 0) return 1;
    const int bad = check_all();
    if (bad) return 2;
    time_all(argc > 1 ? atoi(argv[1]) : 2);
    return 0;
}
