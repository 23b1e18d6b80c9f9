// inccl_peer.hip -- the p2p engine's two kernels that read other GPUs' memory
// (csrc/p2p.c): the pull reduce-scatter and the all-gather.
//
// Peer buffers are mapped over HIP IPC.  Remote VRAM may be cached
// non-coherently in this GPU's L2, and these kernels re-read the same peer
// addresses on every call.  So every load of peer memory is a system-scope
// `buffer_load_dwordx4 ... sc0 sc1` (+ `nt` in the reduce): coherent and
// L1-bypassing.  The producers'
// stores are write-through (`sc1`, as the stream kernel's): they leave
// the L2 at once and reach memory before the host barrier that separates the
// phases, and nothing is left dirty for the kernel boundary to write back.
//
//   k_peer_reduce<R>:  out[i] = dequant( sum_{j<R} peer_j[i] )   int32 -> fp32
//       the reference switch's aggregate (non_termination_switch.c:361-363)
//       over the W ranks' shards, fused with the new dequantise stage
//       (DEQ = false: the plain int32 sum, for the int32 allreduce)
//   k_peer_gather:     dst[off_j + i] = src_j[i]  for every rank j; consecutive
//       workgroups take consecutive ranks, so the resident workgroups read
//       from every peer at once (segment-major dispatch would drain the peers
//       one xGMI link at a time)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "inccl_kernels.h"
#include "inccl_stream.h"

namespace {

using namespace inccl_dev;

// Peer loads are system scope (sc0 sc1).  The pull-reduce's also carry the
// nontemporal hint, which leaves the scope bits (and so coherence) unchanged:
// 7.15 TB/s with it against 5.83 without on local HBM
// (tools/tune/tune_peer.hip, profiles/r02/tune_peer.jsonl; W = 8: 6.31 vs 5.14),
// 170 -> 115 us per call in the 2-rank one-GPU step.  The gather reads result
// shards that were just written through to the Infinity Cache; there the hint
// cost 147 -> 172 us, so its loads stay without it.
constexpr int kAuxSys = 1 | 16;         // buffer instruction cache policy: sc0 | sc1
constexpr int kAuxSysNT = 1 | 2 | 16;   // sc0 | nt | sc1
constexpr int kAuxWT = 16;              // sc1: write-through store

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

template <int AUX = kAuxSys>
__device__ __forceinline__ u32x4 ld_sys16(const void* tile_base, uint32_t tile_bytes, uint32_t off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(rsrc(tile_base, tile_bytes), (int)off, 0, AUX);
}

// DEQ = false: the int32 sum itself (the reference's int32 allreduce,
// inccl_allreduce_write over the IPC engines), no dequantise stage
template <int R, int BLOCK, bool DEQ>
__global__ __launch_bounds__(BLOCK) void k_peer_reduce(SrcPtrs src, float* __restrict__ dst, int64_t n4, Scale sc)
{
    const float inv = DEQ ? deq_scale(sc, resolve_k(sc)) : 1.0f;
    u32x4* __restrict__ out = reinterpret_cast<u32x4*>(dst);
    for (int64_t base = (int64_t)blockIdx.x * BLOCK; base < n4; base += (int64_t)gridDim.x * BLOCK) {
        const int64_t i = base + threadIdx.x;
        const int64_t left = n4 - base;
        const uint32_t tile_bytes = (uint32_t)((left < BLOCK ? left : BLOCK) * 16);
        u32x4 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r)   // out-of-range lanes read 0 (buffer range check)
            v[r] = ld_sys16<kAuxSysNT>(reinterpret_cast<const u32x4*>(src.p[r]) + base, tile_bytes, threadIdx.x * 16u);
        if (i < n4) {
            u32x4 acc = v[0];
#pragma unroll
            for (int r = 1; r < R; ++r) {
                acc.x += v[r].x;
                acc.y += v[r].y;
                acc.z += v[r].z;
                acc.w += v[r].w;
            }
            u32x4 o = acc;
            if constexpr (DEQ) {
                o.x = __float_as_uint((float)(int32_t)acc.x * inv);
                o.y = __float_as_uint((float)(int32_t)acc.y * inv);
                o.z = __float_as_uint((float)(int32_t)acc.z * inv);
                o.w = __float_as_uint((float)(int32_t)acc.w * inv);
            }
            __builtin_amdgcn_raw_buffer_store_b128(o, rsrc(out + base, tile_bytes), (int)(threadIdx.x * 16u), 0, kAuxWT);
        }
    }
}

// The pull-reduce with a 2-byte result (inccl_allreduce_bf16 / _f16 on the p2p
// engine): the same 16-B system-scope loads of 4 int32 partials per peer and
// lane, summed, dequantised and narrowed (v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32,
// K = BF16 / F16) into 8 bytes per lane, written through.
template <int R, int BLOCK, int K>
__global__ __launch_bounds__(BLOCK) void k_peer_reduce16(SrcPtrs src, uint16_t* __restrict__ dst, int64_t n4, Scale sc)
{
    const float inv = deq_scale(sc, resolve_k(sc));
    for (int64_t base = (int64_t)blockIdx.x * BLOCK; base < n4; base += (int64_t)gridDim.x * BLOCK) {
        const int64_t i = base + threadIdx.x;
        const int64_t left = n4 - base;
        const uint32_t tile_in = (uint32_t)((left < BLOCK ? left : BLOCK) * 16);
        u32x4 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r)   // out-of-range lanes read 0 (buffer range check)
            v[r] = ld_sys16<kAuxSysNT>(reinterpret_cast<const u32x4*>(src.p[r]) + base, tile_in, threadIdx.x * 16u);
        if (i < n4) {
            u32x4 acc = v[0];
#pragma unroll
            for (int r = 1; r < R; ++r) {
                acc.x += v[r].x;
                acc.y += v[r].y;
                acc.z += v[r].z;
                acc.w += v[r].w;
            }
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 o = {deq16x2<K>(acc.x, acc.y, inv), deq16x2<K>(acc.z, acc.w, inv)};
            __builtin_amdgcn_raw_buffer_store_b64(o, rsrc(dst + base * 4, tile_in / 2), (int)(threadIdx.x * 8u), 0,
                                                  kAuxWT);
        }
    }
}

struct Segs {
    const void* src[kMaxR];
    int64_t off[kMaxR];
    int64_t cnt[kMaxR];
    int tail16[kMaxR];   // 2-byte gathers: one more element after cnt words (the low half of word cnt)
    int nseg;
};

constexpr int kGatherBlock = 256;
constexpr int kGatherU = 4;   // float4 per lane per tile

__global__ __launch_bounds__(kGatherBlock) void k_peer_gather(Segs s, uint32_t* __restrict__ dst)
{
    const int j = (int)(blockIdx.x % (unsigned)s.nseg);          // interleaved: every link busy at once
    const int64_t xb = blockIdx.x / (unsigned)s.nseg, gxs = gridDim.x / (unsigned)s.nseg;
    const int64_t cnt = s.cnt[j];
    uint32_t* __restrict__ d = dst + s.off[j];
    const uint32_t* src = reinterpret_cast<const uint32_t*>(s.src[j]);
    const int64_t n4 = cnt >> 2;
    const int64_t tile = (int64_t)kGatherBlock * kGatherU;
    const bool dvec = (reinterpret_cast<uintptr_t>(d) & 15u) == 0;
    for (int64_t base = xb * tile; base < n4; base += gxs * tile) {
        const int64_t left = n4 - base;
        const uint32_t tile_bytes = (uint32_t)((left < tile ? left : tile) * 16);
        const u32x4* tb = reinterpret_cast<const u32x4*>(src) + base;
        u32x4 v[kGatherU];
#pragma unroll
        for (int u = 0; u < kGatherU; ++u)
            v[u] = ld_sys16(tb, tile_bytes, (threadIdx.x + u * kGatherBlock) * 16u);
#pragma unroll
        for (int u = 0; u < kGatherU; ++u) {
            const int64_t i = base + threadIdx.x + (int64_t)u * kGatherBlock;
            if (i < n4) {
                if (dvec) {
                    __builtin_amdgcn_raw_buffer_store_b128(v[u], rsrc(reinterpret_cast<u32x4*>(d) + base, tile_bytes),
                                                           (int)((threadIdx.x + u * kGatherBlock) * 16u), 0, kAuxWT);
                } else {
                    d[4 * i] = v[u].x;
                    d[4 * i + 1] = v[u].y;
                    d[4 * i + 2] = v[u].z;
                    d[4 * i + 3] = v[u].w;
                }
            }
        }
    }
    if (xb == 0) {   // ragged tail of the last shard
        for (int64_t i = (n4 << 2) + threadIdx.x; i < cnt; i += kGatherBlock)
            d[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (s.tail16[j] && threadIdx.x == 0)   // an odd element count of 2-byte elements
            reinterpret_cast<uint16_t*>(d + cnt)[0] =
                (uint16_t)(__hip_atomic_load(src + cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & 0xffffu);
    }
}

template <int R, bool DEQ = true>
hipError_t launch_reduce_R(const SrcPtrs& s, float* dst, int64_t n4, const Scale& sc, hipStream_t st)
{
    constexpr int B = Geometry<R>::BLOCK;
    const int64_t grid = (n4 + B - 1) / B;
    hipLaunchKernelGGL((k_peer_reduce<R, B, DEQ>), dim3((unsigned)grid), dim3(B), 0, st, s, dst, n4, sc);
    return hipGetLastError();
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace

extern "C" int inccl_k_peer_reduce(const void* const* peers, int W, float* dst, size_t n, int scale_exp,
                                   const uint32_t* amax_bits_dev, int scale_R, int out_shift, void* stream)
{
    if (W < 1 || W > kMaxR || dst == nullptr || (n & 3) != 0 || !aligned16(dst)) return INCCL_ERR_ARG;
    if (n == 0) return 0;
    SrcPtrs s = {};
    for (int j = 0; j < W; ++j) {
        if (peers[j] == nullptr || !aligned16(peers[j])) return INCCL_ERR_ARG;
        s.p[j] = peers[j];
    }
    Scale sc{scale_exp, amax_bits_dev, scale_R > 0 ? scale_R : W, out_shift};
    const int64_t n4 = (int64_t)(n >> 2);
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    switch (W) {
        case 1: e = launch_reduce_R<1>(s, dst, n4, sc, st); break;
        case 2: e = launch_reduce_R<2>(s, dst, n4, sc, st); break;
        case 3: e = launch_reduce_R<3>(s, dst, n4, sc, st); break;
        case 4: e = launch_reduce_R<4>(s, dst, n4, sc, st); break;
        case 5: e = launch_reduce_R<5>(s, dst, n4, sc, st); break;
        case 6: e = launch_reduce_R<6>(s, dst, n4, sc, st); break;
        case 7: e = launch_reduce_R<7>(s, dst, n4, sc, st); break;
        default: e = launch_reduce_R<8>(s, dst, n4, sc, st); break;
    }
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int inccl_k_peer_reduce16(int kind, const void* const* peers, int W, uint16_t* dst, size_t n,
                                     int scale_exp, const uint32_t* amax_bits_dev, int scale_R, int out_shift,
                                     void* stream)
{
    if ((kind != BF16 && kind != F16) || W < 1 || W > kMaxR || dst == nullptr || (n & 3) != 0 || (reinterpret_cast<uintptr_t>(dst) & 7u) != 0)
        return INCCL_ERR_ARG;
    if (n == 0) return 0;
    SrcPtrs s = {};
    for (int j = 0; j < W; ++j) {
        if (peers[j] == nullptr || !aligned16(peers[j])) return INCCL_ERR_ARG;
        s.p[j] = peers[j];
    }
    Scale sc{scale_exp, amax_bits_dev, scale_R > 0 ? scale_R : W, out_shift};
    const int64_t n4 = (int64_t)(n >> 2);
    hipStream_t st = (hipStream_t)stream;
    switch (W) {
#define INCCL_PR16(WW)                                                                                                \
    case WW: {                                                                                                         \
        constexpr int B = Geometry<WW>::BLOCK;                                                                         \
        const dim3 g((unsigned)((n4 + B - 1) / B));                                                                    \
        if (kind == F16)                                                                                               \
            hipLaunchKernelGGL((k_peer_reduce16<WW, B, F16>), g, dim3(B), 0, st, s, dst, n4, sc);                      \
        else                                                                                                           \
            hipLaunchKernelGGL((k_peer_reduce16<WW, B, BF16>), g, dim3(B), 0, st, s, dst, n4, sc);                     \
        break;                                                                                                         \
    }
        INCCL_PR16(1) INCCL_PR16(2) INCCL_PR16(3) INCCL_PR16(4) INCCL_PR16(5) INCCL_PR16(6) INCCL_PR16(7)
        default: INCCL_PR16(8)
#undef INCCL_PR16
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int inccl_k_peer_sum_q32(const void* const* peers, int W, int32_t* dst, size_t n, void* stream)
{
    if (W < 1 || W > kMaxR || dst == nullptr || (n & 3) != 0 || !aligned16(dst)) return INCCL_ERR_ARG;
    if (n == 0) return 0;
    SrcPtrs s = {};
    for (int j = 0; j < W; ++j) {
        if (peers[j] == nullptr || !aligned16(peers[j])) return INCCL_ERR_ARG;
        s.p[j] = peers[j];
    }
    const Scale sc{0, nullptr, W};
    const int64_t n4 = (int64_t)(n >> 2);
    float* d = reinterpret_cast<float*>(dst);   // 32-bit words; no float arithmetic without DEQ
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    switch (W) {
        case 1: e = launch_reduce_R<1, false>(s, d, n4, sc, st); break;
        case 2: e = launch_reduce_R<2, false>(s, d, n4, sc, st); break;
        case 3: e = launch_reduce_R<3, false>(s, d, n4, sc, st); break;
        case 4: e = launch_reduce_R<4, false>(s, d, n4, sc, st); break;
        case 5: e = launch_reduce_R<5, false>(s, d, n4, sc, st); break;
        case 6: e = launch_reduce_R<6, false>(s, d, n4, sc, st); break;
        case 7: e = launch_reduce_R<7, false>(s, d, n4, sc, st); break;
        default: e = launch_reduce_R<8, false>(s, d, n4, sc, st); break;
    }
    return e == hipSuccess ? 0 : (int)e;
}

static int launch_gather(Segs& s, int64_t maxc, void* dst, void* stream);

extern "C" int inccl_k_peer_gather(const void* const* src, const int64_t* off, const int64_t* cnt, int nseg, void* dst,
                                   void* stream)
{
    if (nseg < 1 || nseg > kMaxR || dst == nullptr) return INCCL_ERR_ARG;
    Segs s = {};
    s.nseg = nseg;
    int64_t maxc = 0;
    for (int j = 0; j < nseg; ++j) {
        if ((src[j] == nullptr && cnt[j] > 0) || cnt[j] < 0 || !aligned16(src[j])) return INCCL_ERR_ARG;
        s.src[j] = src[j];
        s.off[j] = off[j];
        s.cnt[j] = cnt[j];
        maxc = cnt[j] > maxc ? cnt[j] : maxc;
    }
    return launch_gather(s, maxc, dst, stream);
}

// 2-byte elements (bf16 result shards): whole 4-byte words, plus the odd last
// element of a segment.  dst must be 4-byte aligned and every offset even.
extern "C" int inccl_k_peer_gather16(const void* const* src, const int64_t* off, const int64_t* cnt, int nseg,
                                     void* dst, void* stream)
{
    if (nseg < 1 || nseg > kMaxR || dst == nullptr || (reinterpret_cast<uintptr_t>(dst) & 3u) != 0)
        return INCCL_ERR_ARG;
    Segs s = {};
    s.nseg = nseg;
    int64_t maxc = 0;
    for (int j = 0; j < nseg; ++j) {
        if ((src[j] == nullptr && cnt[j] > 0) || cnt[j] < 0 || (off[j] & 1) || !aligned16(src[j])) return INCCL_ERR_ARG;
        s.src[j] = src[j];
        s.off[j] = off[j] >> 1;
        s.cnt[j] = cnt[j] >> 1;
        s.tail16[j] = (int)(cnt[j] & 1);
        const int64_t c = s.cnt[j] + s.tail16[j];
        maxc = c > maxc ? c : maxc;
    }
    return launch_gather(s, maxc, dst, stream);
}

static int launch_gather(Segs& s, int64_t maxc, void* dst, void* stream)
{
    const int nseg = s.nseg;
    if (maxc == 0) return 0;
    const int64_t tile = (int64_t)kGatherBlock * kGatherU * 4;
    int64_t gx = (maxc + tile - 1) / tile;
    if (gx < 1) gx = 1;
    hipLaunchKernelGGL(k_peer_gather, dim3((unsigned)(gx * nseg)), dim3(kGatherBlock), 0, (hipStream_t)stream, s,
                       reinterpret_cast<uint32_t*>(dst));
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}
