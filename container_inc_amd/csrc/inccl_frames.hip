// inccl_frames.hip -- the reference's switch dataplane on the GPU (gfx950):
// RoCEv2 frame parse, per-PSN idempotent aggregation, egress frame build and
// the RoCE ICRC (CRC-32).  Reference: repository/src/non_termination_switch.c
// (nts.c) :303-501 for the pipeline and :55-60 / :231-250 for its state;
// repository/src/util.c:331-442 (build_eth_packet), :250-286 (compute_icrc),
// :141-195 (crc32), :106-127 (ipv4_checksum).
//
// One wave64 per frame.  A frame is staged in LDS with dword loads; the ICRC
// input (4 x 0xFF -- the CRC init folded into the message -- then the masked IP
// .. payload bytes) is right-aligned in a 1088-byte window (64 lanes x 17 B) so
// leading zeros do not change the raw CRC.  Each lane runs a byte-table CRC over
// its 17 bytes; a 6-level shuffle tree combines lane CRCs with "append N zero
// bytes" operators held as 4 x 256-entry tables per level in LDS.
//
// State on the GPU (slots = PSN ring size, power of two; the reference uses 16):
//   agg[slots][256] int32        aggregator        (nts.c:55)
//   arrival[slots] uint32        port bitmap + bit fan_in = "result known" (nts.c:59, :366)
//   degree[slots] int32          arrivals incl. retransmits (nts.c:60, :351)
//   reth[slots][fan_in][16 B]    RETH of each child's WRITE_FIRST (nts.c:57, :442)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "inccl_frames.h"

namespace {

constexpr int kWave = 64;
constexpr int kWin = 1088;            // 64 lanes x 17 bytes
constexpr int kSeg = 17;
constexpr int kFrameMax = 1152;       // staged frame bytes (>= 1098)
constexpr int kWavesPerBlock = 4;
constexpr int kEgressWaves = 8;       // 512-lane blocks, CU-sized persistent grid
constexpr int kLanes = 256;           // int32 lanes per packet (nts.c:55)

__device__ uint32_t g_crc_tab[256];          // util.c:141-150 table 0
__device__ uint32_t g_shift_tab[6][4][256];

struct CrcLds {
    uint32_t tab[256];
    uint32_t sh[6][4][256];
};

__device__ __forceinline__ void load_tables(CrcLds& t)
{
    for (int i = threadIdx.x; i < 256; i += blockDim.x) t.tab[i] = g_crc_tab[i];
    uint32_t* dst = &t.sh[0][0][0];
    const uint32_t* src = &g_shift_tab[0][0][0];
    for (int i = threadIdx.x; i < 6 * 4 * 256; i += blockDim.x) dst[i] = src[i];
}

__device__ __forceinline__ uint8_t frame_byte(const uint8_t* fr, int off)
{
    // ICRC masks (util.c:266-270): tos, ttl, IP checksum, UDP checksum, BTH resv8a
    if (off == 15 || off == 22 || off == 24 || off == 25 || off == 40 || off == 41 || off == 46) return 0xFF;
    return fr[off];
}

// ICRC of the frame staged at `fr` (LDS); result valid in every lane.
__device__ uint32_t icrc_wave(const uint8_t* fr, const CrcLds& t, int lane)
{
    const int ip_total = ((int)fr[16] << 8) | fr[17];
    const int L = ip_total;                       // 4 (init) + ip_total - 4 (no ICRC)
    const int lead = kWin - L;                    // zero bytes before the message
    uint8_t b[kSeg];
#pragma unroll
    for (int j = 0; j < kSeg; ++j) {
        const int m = lane * kSeg + j - lead;
        b[j] = (m < 0) ? (uint8_t)0 : ((m < 4) ? (uint8_t)0xFF : frame_byte(fr, 14 + m - 4));
    }
    // byte-table CRC (util.c:190-192 form).  The kernel is bound by LDS lookups,
    // not by this chain's latency: a slice-by-4 variant (4 KiB of tables, one
    // block fewer per CU) measured slower in k_egress (356 vs 289 us / 131k frames).
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < kSeg; ++j) c = (c >> 8) ^ t.tab[(c ^ b[j]) & 0xFFu];
    // tree: at level l the block of lane L (low l bits zero) absorbs block L + 2^l:
    // crc = shift(crc_left, |right| = 17 * 2^l bytes) ^ crc_right.  Only left lanes
    // (the block representatives) are updated; lane 0 ends with the whole window.
#pragma unroll
    for (int l = 0; l < 6; ++l) {
        const uint32_t other = (uint32_t)__shfl_xor((int)c, 1 << l, kWave);
        const uint32_t shifted =
            t.sh[l][0][c & 0xFF] ^ t.sh[l][1][(c >> 8) & 0xFF] ^ t.sh[l][2][(c >> 16) & 0xFF] ^ t.sh[l][3][c >> 24];
        c = shifted ^ other;   // meaningful in left lanes only
    }
    return ~(uint32_t)__shfl((int)c, 0, kWave);
}

// stage `bytes` of a global frame into LDS (dword loads; frames are 4-B aligned)
__device__ __forceinline__ void stage_frame(uint8_t* lds, const uint8_t* g, int bytes, int lane)
{
    const uint32_t* src = reinterpret_cast<const uint32_t*>(g);
    uint32_t* dst = reinterpret_cast<uint32_t*>(lds);
    const int words = (bytes + 3) >> 2;
    for (int i = lane; i < words; i += kWave) dst[i] = src[i];
}

__global__ __launch_bounds__(kWave* kWavesPerBlock) void k_icrc(const uint8_t* __restrict__ frames, int64_t stride,
                                                                int64_t count, uint32_t* __restrict__ out)
{
    __shared__ CrcLds t;
    __shared__ __attribute__((aligned(16))) uint8_t buf[kWavesPerBlock][kFrameMax];
    load_tables(t);
    __syncthreads();
    const int w = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    for (int64_t f0 = (int64_t)blockIdx.x * kWavesPerBlock; f0 < count; f0 += (int64_t)gridDim.x * kWavesPerBlock) {
        const int64_t f = f0 + w;
        if (f < count) {
            const uint8_t* g = frames + f * stride;
            const int ip_total = ((int)g[16] << 8) | g[17];
            const int bytes = 14 + ip_total;
            if (ip_total < 28 || ip_total > kWin || bytes > kFrameMax) {
                if (lane == 0) out[f] = 0;
            } else {
                stage_frame(buf[w], g, bytes, lane);
                __builtin_amdgcn_wave_barrier();
                const uint32_t crc = icrc_wave(buf[w], t, lane);
                if (lane == 0) out[f] = crc;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

__device__ __forceinline__ uint32_t be32(const uint8_t* p)
{
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

__device__ __forceinline__ bool is_data_opcode(uint8_t op)
{
    return op == 0x00 || op == 0x01 || op == 0x02 || op == 0x04 || op == 0x07 || op == 0x08;   // nts.c:314-319
}
__device__ __forceinline__ bool is_write_first(uint8_t op) { return op == 0x06 || op == 0x0A; }   // nts.c:327-328

// Ingress (nts.c:303-483, root branch): one wave per frame.
__global__ __launch_bounds__(kWave* kWavesPerBlock) void k_ingress(InccSwitchState s, const uint8_t* __restrict__ frames,
                                                                   int64_t stride, int64_t count,
                                                                   const int32_t* __restrict__ ports,
                                                                   int32_t* __restrict__ action,
                                                                   uint32_t* __restrict__ psn_out)
{
    const int w = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    const int64_t f = (int64_t)blockIdx.x * kWavesPerBlock + w;
    if (f >= count) return;
    const uint8_t* fr = frames + f * stride;
    const int port = ports[f];
    const uint8_t op = fr[42];
    const uint32_t psn = be32(fr + 50) & 0x00FFFFFFu;          // nts.c:311
    const int udp_len = ((int)fr[38] << 8) | fr[39];
    int act = INCCL_SW_IGNORED;
    if (port < 0 || port >= s.fan_in) act = INCCL_SW_INVALID;
    else if (op == 0x11) act = INCCL_SW_ACK;                    // nts.c:336-342, :403-406 (reflect)
    else if (is_data_opcode(op) || is_write_first(op)) {
        const bool wf = is_write_first(op);
        const int data_len = udp_len - 12 - 8 - 4 - (wf ? 16 : 0);   // nts.c:349, :429
        if (data_len != kLanes * 4) act = INCCL_SW_INVALID;     // nts.c:350 assert
        else {
            const uint32_t slot = psn & (s.slots - 1);
            const uint32_t bit = 1u << port;
            const uint32_t result_bit = 1u << s.fan_in;
            uint32_t old = 0;
            if (lane == 0) {
                atomicAdd(&s.degree[slot], 1);                   // nts.c:351 / :431
                old = atomicOr(&s.arrival[slot], bit);           // nts.c:359 / :441
            }
            old = (uint32_t)__shfl((int)old, 0, kWave);
            if (old & bit) {
                act = (old & result_bit) ? INCCL_SW_REPLAY : INCCL_SW_DROPPED;   // nts.c:353-357
            } else {
                const uint8_t* data = fr + 54 + (wf ? 16 : 0);
                // the payload starts at byte 54 (70 with RETH): 2-byte aligned only
                const uint16_t* d16 = reinterpret_cast<const uint16_t*>(data);
                if (wf && lane < 4) {                            // reth_keeper, nts.c:442
                    const uint16_t* r = reinterpret_cast<const uint16_t*>(fr + 54);
                    s.reth[((size_t)slot * s.fan_in + port) * 4 + lane] =
                        (uint32_t)r[2 * lane] | ((uint32_t)r[2 * lane + 1] << 16);
                }
                int32_t* agg = s.agg + (size_t)slot * kLanes;
                // word i = j*64 + lane: each wave-instruction adds 256 contiguous
                // bytes (the full-rate atomic shape, MI355X_MICROARCH.md atomics)
#pragma unroll
                for (int j = 0; j < 4; ++j) {                    // nts.c:361-363 / :443-445
                    const int i = j * kWave + lane;
                    const uint32_t raw = (uint32_t)d16[2 * i] | ((uint32_t)d16[2 * i + 1] << 16);
                    atomicAdd(&agg[i], (int32_t)__builtin_bswap32(raw));
                }
                const uint32_t mask = 0xffffffffu >> (32 - s.fan_in);
                act = (((old | bit) & mask) == mask) ? INCCL_SW_COMPLETED : INCCL_SW_ABSORBED;   // nts.c:365
            }
        }
    }
    if (lane == 0) {
        action[f] = act;
        psn_out[f] = psn;
    }
}

__device__ __forceinline__ void put16(uint8_t* p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

// Header image of child c's egress frames (util.c:348-388) with opcode and PSN
// left zero: identical for every frame of that child and RETH flag, so each
// block builds the 2*fan_in images once into LDS and frames copy them word-wise.
constexpr int kHdrImg = 72;   // 70 header bytes (with RETH slot) rounded to dwords

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

__device__ void egress_one(const InccSwitchState& s, const uint8_t* __restrict__ in_frames, int64_t in_stride,
                           const int32_t* __restrict__ ports, const int32_t* __restrict__ action,
                           const uint32_t* __restrict__ psns, const uint8_t (*himg)[kHdrImg],
                           uint8_t* __restrict__ out, int64_t out_stride, bool out16,
                           int32_t* __restrict__ out_len, const CrcLds& t, uint8_t* frbuf, int64_t g, int lane)
{
    const int fan = s.fan_in;
    const int64_t f = g / fan;
    const int c = (int)(g % fan);
    const int act = action[f];
    const bool emit = (act == INCCL_SW_COMPLETED) || (act == INCCL_SW_REPLAY && ports[f] == c);
    if (!emit) {
        if (lane == 0) out_len[g] = 0;
        return;
    }
    const uint32_t psn = psns[f];
    const uint32_t slot = psn & (s.slots - 1);
    const uint8_t op = in_frames[f * in_stride + 42];
    const bool wf = is_write_first(op);
    const int total = 14 + 20 + 8 + 12 + (wf ? 16 : 0) + kLanes * 4 + 4;   // util.c:341-345
    uint8_t* fr = frbuf;
    if (lane < kHdrImg / 4)
        reinterpret_cast<uint32_t*>(fr)[lane] = reinterpret_cast<const uint32_t*>(himg[c * 2 + (wf ? 1 : 0)])[lane];
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {                                                 // util.c:378, :386
        const uint32_t p = psn | 0x80000000u;
        fr[42] = op;
        fr[50] = (uint8_t)(p >> 24); fr[51] = (uint8_t)(p >> 16); fr[52] = (uint8_t)(p >> 8); fr[53] = (uint8_t)p;
    }
    // offsets 54 / 70 are 2-byte aligned: 16-bit LDS stores
    if (wf && lane < 4) {                                            // util.c:409-417, reth_keeper[slot][c]
        const uint32_t r = s.reth[((size_t)slot * fan + c) * 4 + lane];
        uint16_t* r16 = reinterpret_cast<uint16_t*>(fr + 54);
        r16[2 * lane] = (uint16_t)r;
        r16[2 * lane + 1] = (uint16_t)(r >> 16);
    }
    const int doff = 54 + (wf ? 16 : 0);
    const int32_t* agg = s.agg + (size_t)slot * kLanes;
    uint16_t* d16 = reinterpret_cast<uint16_t*>(fr + doff);
#pragma unroll
    for (int j = 0; j < 4; ++j) {                                    // util.c:403-405 / :419-421 htonl
        const int i = j * kWave + lane;
        const uint32_t be = __builtin_bswap32((uint32_t)agg[i]);
        d16[2 * i] = (uint16_t)be;
        d16[2 * i + 1] = (uint16_t)(be >> 16);
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t crc = icrc_wave(fr, t, lane);                    // util.c:424-426
    if (lane == 0) {                                                 // stored host order (LE)
        fr[total - 4] = (uint8_t)crc;
        fr[total - 3] = (uint8_t)(crc >> 8);
        fr[total - 2] = (uint8_t)(crc >> 16);
        fr[total - 1] = (uint8_t)(crc >> 24);
    }
    __builtin_amdgcn_wave_barrier();
    uint8_t* o = out + g * out_stride;
    if (out16) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        for (int i = lane; i < (total + 15) / 16; i += kWave)
            reinterpret_cast<u4*>(o)[i] = reinterpret_cast<const u4*>(fr)[i];
    } else {
        for (int i = lane; i < (total + 3) / 4; i += kWave)
            reinterpret_cast<uint32_t*>(o)[i] = reinterpret_cast<const uint32_t*>(fr)[i];
    }
    if (lane == 0) out_len[g] = total;
    // the result is known from now on: later retransmits replay (nts.c:366)
    if (act == INCCL_SW_COMPLETED && c == 0 && lane == 0) atomicOr(&s.arrival[slot], 1u << fan);
    __builtin_amdgcn_wave_barrier();
}

// Egress (nts.c:365-372 / :447-453 broadcast, :353-356 / :435-438 replay;
// frames per util.c:331-442): wave (f, c) builds child c's copy of frame f.
__global__ __launch_bounds__(kWave* kEgressWaves) void k_egress(InccSwitchState s, const uint8_t* __restrict__ in_frames,
                                                               int64_t in_stride, int64_t count,
                                                               const int32_t* __restrict__ ports,
                                                               const int32_t* __restrict__ action,
                                                               const uint32_t* __restrict__ psns,
                                                               const InccFrameTemplate* __restrict__ tmpl,
                                                               uint8_t* __restrict__ out, int64_t out_stride,
                                                               int32_t* __restrict__ out_len)
{
    __shared__ CrcLds t;
    __shared__ __attribute__((aligned(16))) uint8_t buf[kEgressWaves][kFrameMax];
    __shared__ __attribute__((aligned(16))) uint8_t himg[2 * 31][kHdrImg];
    load_tables(t);
    const int fan = s.fan_in;
    for (int i = threadIdx.x; i < 2 * fan; i += blockDim.x) build_header_image(himg[i], tmpl[i >> 1], (i & 1) != 0);
    __syncthreads();
    const int w = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    const bool out16 = ((out_stride & 15) == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
    for (int64_t g = (int64_t)blockIdx.x * kEgressWaves + w; g < count * fan; g += (int64_t)gridDim.x * kEgressWaves)
        egress_one(s, in_frames, in_stride, ports, action, psns, himg, out, out_stride, out16, out_len, t, buf[w], g,
                   lane);
}

// clear_state_data(psn + WINDOW) for every slot completed in the batch (nts.c:235-242, :367)
__global__ void k_recycle(InccSwitchState s, int64_t count, const int32_t* __restrict__ action,
                          const uint32_t* __restrict__ psns)
{
    const int64_t f = blockIdx.x;
    if (f >= count || action[f] != INCCL_SW_COMPLETED) return;
    const uint32_t slot = (psns[f] + (s.slots >> 1)) & (s.slots - 1);
    int32_t* agg = s.agg + (size_t)slot * kLanes;
    for (int i = threadIdx.x; i < kLanes; i += blockDim.x) agg[i] = 0;
    for (int i = threadIdx.x; i < s.fan_in * 4; i += blockDim.x) s.reth[(size_t)slot * s.fan_in * 4 + i] = 0;
    if (threadIdx.x == 0) {
        s.arrival[slot] = 0;
        s.degree[slot] = 0;
    }
}

// ---------------------------------------------------------------------------
// host: CRC tables (util.c:141-159) and the zero-append operators per tree level
// ---------------------------------------------------------------------------
uint32_t host_tab[256];
uint32_t host_shift[6][4][256];
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
    for (int l = 0; l < 6; ++l)
        for (int b = 0; b < 4; ++b)
            for (uint32_t v = 0; v < 256; ++v) host_shift[l][b][v] = zeros_append(v << (8 * b), kSeg << l);
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_crc_tab), host_tab, sizeof(host_tab));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_shift_tab), host_shift, sizeof(host_shift));
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

inline int grid_for(int64_t waves)
{
    const int64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    return (int)(blocks < 1 ? 1 : blocks);
}

}  // namespace

extern "C" {

int inccl_k_frames_init(void) { return ensure_tables(); }

int inccl_k_icrc(const uint8_t* frames, size_t stride, size_t count, uint32_t* out, void* stream)
{
    if ((frames == nullptr || out == nullptr) && count) return INCCL_ERR_ARG;
    if ((stride & 3) || ((uintptr_t)frames & 3)) return INCCL_ERR_ARG;
    if (count == 0) return 0;
    int rc = ensure_tables();
    if (rc) return rc;
    const int64_t blocks = ((int64_t)count + kWavesPerBlock - 1) / kWavesPerBlock;
    const int64_t cap = (int64_t)num_cus() * 4;
    const int grid = (int)(blocks < cap ? blocks : cap);
    hipLaunchKernelGGL(k_icrc, dim3(grid), dim3(kWave * kWavesPerBlock), 0, (hipStream_t)stream, frames,
                       (int64_t)stride, (int64_t)count, out);
    return (int)hipGetLastError();
}

int inccl_k_switch_ingress(const InccSwitchState* s, const uint8_t* frames, size_t stride, size_t count,
                           const int32_t* ports, int32_t* action, uint32_t* psn_out, void* stream)
{
    if (count == 0) return 0;
    if (!s || !frames || !ports || !action || !psn_out || (stride & 3) || ((uintptr_t)frames & 3)) return INCCL_ERR_ARG;
    hipLaunchKernelGGL(k_ingress, dim3(grid_for((int64_t)count)), dim3(kWave * kWavesPerBlock), 0,
                       (hipStream_t)stream, *s, frames, (int64_t)stride, (int64_t)count, ports, action, psn_out);
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
    // persistent grid: the 25 KiB CRC tables are loaded once per block
    const int64_t need = ((int64_t)count * s->fan_in + kEgressWaves - 1) / kEgressWaves;
    const int64_t cap = (int64_t)num_cus() * 4;
    const int eg = (int)(need < cap ? (need < 1 ? 1 : need) : cap);
    hipLaunchKernelGGL(k_egress, dim3(eg), dim3(kWave * kEgressWaves), 0, st, *s,
                       in_frames, (int64_t)in_stride, (int64_t)count, ports, action, psns, tmpl, out,
                       (int64_t)out_stride, out_len);
    hipLaunchKernelGGL(k_recycle, dim3((unsigned)count), dim3(256), 0, st, *s, (int64_t)count, action, psns);
    return (int)hipGetLastError();
}

}  // extern "C"
