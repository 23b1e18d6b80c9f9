// inccl_kernels.hip -- CDNA4 (gfx950) kernels of the INCCL aggregation hot path.
//
// Every kernel here is element-wise and HBM-bound (a few VALU ops per 4-byte
// element): no MFMA, no LDS staging of the stream.  One generic streaming
// kernel covers the whole per-element family of the reference path:
//
//   input  kind  F32      fp32 gradient, quantised on load  (new front stage)
//                Q32      int32 host order                   (nts.c:361 aggregator lanes)
//                Q32BE    int32 big-endian wire word         (api.c:301 / nts.c:362 ntohl)
//   output kind  F32      dequantised fp32                   (new back stage)
//                Q32      int32 host order                   (api.c:429 decode)
//                Q32BE    int32 big-endian wire word         (util.c:404 egress htonl)
//
//   out[i] = OUT( sum_{r<R} IN(src_r[i]) )     sum in uint32 = exact mod-2^32 wrap.
//
// So quantise = <F32,Q32,1>, dequantise = <Q32,F32,1>, the fused single-GPU
// bucket reduce = <F32,F32,R>, the switch aggregate = <Q32BE,Q32BE,R>, the
// multi-GPU first stage = <F32,Q32,R>, and the byte swap codec = <Q32BE,Q32,1>.
//
// Layout: each lane moves 16 B per access (global_load_dwordx4 = one 1 KiB
// wave-instruction = exactly one reference packet payload of 256 lanes,
// nts.c:55).  A workgroup of BLOCK lanes owns a tile of BLOCK*U float4 per
// input and issues all R*U nontemporal loads before touching them, then writes
// U write-through (sc1) float4 stores; BLOCK/U per R come from measured sweeps
// (Geometry<R> in inccl_stream.h: 512 x 2 at R = 2, 512 x 1 at R = 3, 1024 x 1
// otherwise).  One workgroup per tile by default (a grid-stride loop covers a
// capped grid).
//
// The horizontal reductions (absmax for automatic scaling, the position
// weighted checksum) use wave64 __shfl_xor trees, an LDS stage across the
// block's waves and one global atomic per block.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "inccl_kernels.h"
#include "inccl_stream.h"

namespace {

using namespace inccl_dev;

// Element-granular variant: the scalar tail after the float4 body, and the whole
// range when any pointer is not 16-B aligned.
template <int IN, int OUT, int R>
__global__ __launch_bounds__(kBlock) void k_stream_scalar(SrcPtrs src, void* __restrict__ dst, int64_t begin,
                                                          int64_t n, Scale sc)
{
    const int k = resolve_k(sc);
    const float scale = pow2f(k);
    const float inv = deq_scale(sc, k);
    uint32_t* __restrict__ out = reinterpret_cast<uint32_t*>(dst);
    for (int64_t i = begin + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        uint32_t acc = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) acc += load_xform<IN>(reinterpret_cast<const uint32_t*>(src.p[r])[i], scale);
        out[i] = store_xform<OUT>(acc, inv);
    }
}

// bf16 streaming kernel k_stream16 and its helpers: inccl_stream.h (shared with
// tools/tune/tune_bf16.hip)

// element-granular bf16 variant: the tail after the 8-element groups, or the
// whole range when a pointer is not 16-B aligned
template <int IN, int OUT, int R>
__global__ __launch_bounds__(kBlock) void k_stream16_scalar(SrcPtrs src, void* __restrict__ dst, int64_t begin,
                                                            int64_t n, Scale sc)
{
    const int k = resolve_k(sc);
    const float scale = pow2f(k);
    const float inv = deq_scale(sc, k);
    for (int64_t i = begin + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        uint32_t acc = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if constexpr (is16(IN))
                acc += quant16<IN>(reinterpret_cast<const uint16_t*>(src.p[r])[i], scale);
            else
                acc += reinterpret_cast<const uint32_t*>(src.p[r])[i];
        }
        if constexpr (is16(OUT))
            reinterpret_cast<uint16_t*>(dst)[i] = (uint16_t)deq16x2<OUT>(acc, 0u, inv);
        else
            reinterpret_cast<uint32_t*>(dst)[i] = acc;
    }
}

// ---- horizontal reductions: wave64 shuffle -> LDS -> one atomic per block ----
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)v, off, 64);
        v = v > o ? v : o;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
    return v;
}

// |x| bits of a float; NaN -> 0 (ignored, as orc_absmax_f32).  Non-negative
// IEEE floats order like their bit patterns, so max over bits == max over values.
// NF (INCCL_ABSMAX_FLAG_NONFINITE): a NaN or +-Inf instead sets bit 31, which
// no |x| has, so the max over every element -- and over the ranks -- carries it
// (deq_scale then makes every result NaN).
template <bool NF = false>
__device__ __forceinline__ uint32_t abs_bits(uint32_t b)
{
    const uint32_t a = b & 0x7fffffffu;
    if constexpr (NF) return a >= 0x7f800000u ? 0x80000000u | a : a;
    else return a > 0x7f800000u ? 0u : a;
}

// absmax over 2-byte buckets (E: BF16 or F16), as the fp32 bits of the widened values
template <bool NF>
__device__ __forceinline__ uint32_t abs_bits_bf16(uint32_t h) { return abs_bits<NF>(h << 16); }
template <bool NF>
__device__ __forceinline__ uint32_t abs_bits_f16(uint32_t h) { return abs_bits<NF>(__float_as_uint(f16_widen(h))); }
template <int E, bool NF>
__device__ __forceinline__ uint32_t abs_bits16(uint32_t h)
{
    if constexpr (E == F16) return abs_bits_f16<NF>(h);
    else return abs_bits_bf16<NF>(h);
}

// element kind of k_absmax: F32, BF16 or F16
template <int E, bool NF>
__device__ __forceinline__ uint32_t amax_quad(u32x4 x)
{
    if constexpr (E != F32)
        return max(max(max(abs_bits16<E, NF>(x.x & 0xffffu), abs_bits16<E, NF>(x.x >> 16)),
                       max(abs_bits16<E, NF>(x.y & 0xffffu), abs_bits16<E, NF>(x.y >> 16))),
                   max(max(abs_bits16<E, NF>(x.z & 0xffffu), abs_bits16<E, NF>(x.z >> 16)),
                       max(abs_bits16<E, NF>(x.w & 0xffffu), abs_bits16<E, NF>(x.w >> 16))));
    else
        return max(max(abs_bits<NF>(x.x), abs_bits<NF>(x.y)), max(abs_bits<NF>(x.z), abs_bits<NF>(x.w)));
}

// max |x| over R buckets of fp32 (E = F32), bf16 or fp16 elements.
// Geometry from tools/tune/tune_absmax.hip (R = 2 x 256 MiB fp32,
// profiles/r02/tune_absmax.jsonl): 512 lanes x 2 quads per input and step, all
// 2R loads in flight before the first compare, grid capped at 2 workgroups per
// CU -- 0.83-0.84 of HBM, against 0.73 for the round-1 form (256 x 1, 8 per CU).
constexpr int kAmBlock = 512, kAmU = 2;

template <int R, int E, bool NF>
__global__ __launch_bounds__(kAmBlock) void k_absmax(SrcPtrs src, int64_t n, uint32_t* __restrict__ out, int vec)
{
    constexpr bool B16 = E != F32;
    constexpr int EPQ = B16 ? 8 : 4;   // elements per 16-B quad
    __shared__ uint32_t part[kAmBlock / 64];
    uint32_t m = 0;
    const int64_t nq = vec ? n / EPQ : 0;   // a bucket not 16-B aligned: element loads only
    const int64_t tile = (int64_t)kAmBlock * kAmU;
    for (int64_t base = (int64_t)blockIdx.x * tile; base < nq; base += (int64_t)gridDim.x * tile) {
        u32x4 v[R][kAmU];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < kAmU; ++u) {
                const int64_t i = base + threadIdx.x + (int64_t)u * kAmBlock;
                v[r][u] = i < nq ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src.p[r]) + i)
                                 : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < kAmU; ++u) {
                const uint32_t a = amax_quad<E, NF>(v[r][u]);
                m = m > a ? m : a;
            }
    }
    const int64_t stride = (int64_t)gridDim.x * kAmBlock;
#pragma unroll
    for (int r = 0; r < R; ++r)
        for (int64_t i = nq * EPQ + (int64_t)blockIdx.x * kAmBlock + threadIdx.x; i < n; i += stride) {
            const uint32_t a = B16 ? abs_bits16<E, NF>(reinterpret_cast<const uint16_t*>(src.p[r])[i])
                                   : abs_bits<NF>(reinterpret_cast<const uint32_t*>(src.p[r])[i]);
            m = m > a ? m : a;
        }
    m = wave_max_u32(m);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) part[wave] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t b = part[0];
#pragma unroll
        for (int w = 1; w < kAmBlock / 64; ++w) b = b > part[w] ? b : part[w];
        atomicMax(out, b);
    }
}

// cs = sum_i (2*(base+i)+1) * q[i]  mod 2^32  (orc_checksum_q32); linear in q.
__global__ __launch_bounds__(kBlock) void k_checksum(const uint32_t* __restrict__ q, int64_t n, uint64_t base,
                                                     uint32_t* __restrict__ out)
{
    __shared__ uint32_t part[kBlock / 64];
    uint32_t s = 0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    const int64_t n4 = n >> 2;
    const u32x4* q4 = reinterpret_cast<const u32x4*>(q);
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += stride) {
        const u32x4 x = q4[i];
        const uint32_t w = 2u * (uint32_t)(base + (uint64_t)(i << 2)) + 1u;
        s += w * x.x + (w + 2u) * x.y + (w + 4u) * x.z + (w + 6u) * x.w;
    }
    for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        s += (2u * (uint32_t)(base + (uint64_t)i) + 1u) * q[i];
    s = wave_sum_u32(s);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) part[wave] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t b = 0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) b += part[w];
        atomicAdd(out, b);
    }
}

// ---------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------
int g_num_cus = 0;
int g_grid_cap = 0;   // 0 -> default; settable for tuning sweeps
bool g_nt_loads = true;

int num_cus()
{
    if (g_num_cus == 0) {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            g_num_cus = v;
        else
            g_num_cus = 256;
    }
    return g_num_cus;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

template <int IN, int OUT, int R>
int launch_stream_R(const SrcPtrs& s, void* dst, int64_t n, const Scale& sc, hipStream_t st)
{
    bool vec = aligned16(dst);
    for (int r = 0; r < R; ++r) vec = vec && aligned16(s.p[r]);
    int64_t done = 0;
    if (vec) {
        const int64_t n4 = n >> 2;
        if (n4 > 0) {
            constexpr int U = Geometry<R>::U;
            constexpr int B = Geometry<R>::BLOCK;
            const int64_t tiles = (n4 + (int64_t)B * U - 1) / ((int64_t)B * U);
            // One workgroup per tile by default (measured on MI355X, 2 x 256 MiB
            // fused: one-shot 6.51 TB/s vs 6.23 TB/s for a 16-per-CU grid-stride cap).
            const int64_t cap = g_grid_cap > 0 ? g_grid_cap : (int64_t)0x7fffffff;
            const int grid = (int)(tiles < cap ? tiles : cap);
            if (g_nt_loads)
                hipLaunchKernelGGL((k_stream_vec<IN, OUT, R, true, B, U>), dim3(grid), dim3(B), 0, st, s, dst, n4, sc);
            else
                hipLaunchKernelGGL((k_stream_vec<IN, OUT, R, false, B, U>), dim3(grid), dim3(B), 0, st, s, dst, n4, sc);
        }
        done = n4 << 2;
    }
    if (done < n) {
        const int64_t rem = n - done;
        int64_t blocks = (rem + kBlock - 1) / kBlock;
        const int64_t cap = (int64_t)num_cus() * 8;
        const int grid = (int)(blocks < cap ? blocks : cap);
        hipLaunchKernelGGL((k_stream_scalar<IN, OUT, R>), dim3(grid), dim3(kBlock), 0, st, s, dst, done, n, sc);
    }
    return (int)hipGetLastError();
}

template <int IN, int OUT>
int launch_stream(const void* const* srcs, int R, void* dst, int64_t n, const Scale& sc, hipStream_t st)
{
    if (R < 1 || R > kMaxR) return INCCL_ERR_ARG;
    if (n <= 0) return 0;
    SrcPtrs s = {};
    for (int r = 0; r < R; ++r) {
        if (srcs[r] == nullptr) return INCCL_ERR_ARG;
        s.p[r] = srcs[r];
    }
    switch (R) {
    case 1: return launch_stream_R<IN, OUT, 1>(s, dst, n, sc, st);
    case 2: return launch_stream_R<IN, OUT, 2>(s, dst, n, sc, st);
    case 3: return launch_stream_R<IN, OUT, 3>(s, dst, n, sc, st);
    case 4: return launch_stream_R<IN, OUT, 4>(s, dst, n, sc, st);
    case 5: return launch_stream_R<IN, OUT, 5>(s, dst, n, sc, st);
    case 6: return launch_stream_R<IN, OUT, 6>(s, dst, n, sc, st);
    case 7: return launch_stream_R<IN, OUT, 7>(s, dst, n, sc, st);
    default: return launch_stream_R<IN, OUT, 8>(s, dst, n, sc, st);
    }
}

// bf16 geometry per R, from tools/tune/tune_bf16.hip on MI355X (256 MiB bf16
// buckets, profiles/r02/tune_bf16.jsonl): R <= 2 -> 512 lanes x 1 group
// (R = 2: 0.89-0.90 of HBM repeated, 0.80-0.81 rotated, against 0.88-0.89 /
// 0.79 at 512 x 2); R >= 3 -> 256 x 2 (R = 8: 0.79 / 0.74; 512 x 1 drops to 0.72
// rotated).  A memory-only kernel of the same access pattern reaches 0.86 / 0.78
// at R = 2: the arithmetic is hidden.
template <int R>
struct B16Geometry {
    static constexpr int BLOCK = R <= 2 ? 512 : 256;
    static constexpr int U = R <= 2 ? 1 : 2;
};

template <int IN, int OUT, int R>
int launch_stream16_R(const SrcPtrs& s, void* dst, int64_t n, const Scale& sc, hipStream_t st)
{
    bool vec = aligned16(dst);
    for (int r = 0; r < R; ++r) vec = vec && aligned16(s.p[r]);
    int64_t done = 0;
    if (vec) {
        const int64_t n8 = n >> 3;
        if (n8 > 0) {
            constexpr int B = B16Geometry<R>::BLOCK, U = B16Geometry<R>::U;
            const int64_t tiles = (n8 + (int64_t)B * U - 1) / ((int64_t)B * U);
            const int64_t cap = g_grid_cap > 0 ? g_grid_cap : (int64_t)0x7fffffff;
            const int grid = (int)(tiles < cap ? tiles : cap);
            hipLaunchKernelGGL((k_stream16<IN, OUT, R, B, U>), dim3(grid), dim3(B), 0, st, s, dst, n8, sc);
        }
        done = n8 << 3;
    }
    if (done < n) {
        const int64_t blocks = (n - done + kBlock - 1) / kBlock;
        const int64_t cap = (int64_t)num_cus() * 8;
        const int grid = (int)(blocks < cap ? blocks : cap);
        hipLaunchKernelGGL((k_stream16_scalar<IN, OUT, R>), dim3(grid), dim3(kBlock), 0, st, s, dst, done, n, sc);
    }
    return (int)hipGetLastError();
}

template <int IN, int OUT>
int launch_stream16(const void* const* srcs, int R, void* dst, int64_t n, const Scale& sc, hipStream_t st)
{
    if (R < 1 || R > kMaxR) return INCCL_ERR_ARG;
    if (n <= 0) return 0;
    SrcPtrs s = {};
    for (int r = 0; r < R; ++r) {
        if (srcs[r] == nullptr) return INCCL_ERR_ARG;
        s.p[r] = srcs[r];
    }
    switch (R) {
    case 1: return launch_stream16_R<IN, OUT, 1>(s, dst, n, sc, st);
    case 2: return launch_stream16_R<IN, OUT, 2>(s, dst, n, sc, st);
    case 3: return launch_stream16_R<IN, OUT, 3>(s, dst, n, sc, st);
    case 4: return launch_stream16_R<IN, OUT, 4>(s, dst, n, sc, st);
    case 5: return launch_stream16_R<IN, OUT, 5>(s, dst, n, sc, st);
    case 6: return launch_stream16_R<IN, OUT, 6>(s, dst, n, sc, st);
    case 7: return launch_stream16_R<IN, OUT, 7>(s, dst, n, sc, st);
    default: return launch_stream16_R<IN, OUT, 8>(s, dst, n, sc, st);
    }
}

int dispatch(int in_kind, int out_kind, const void* const* srcs, int R, void* dst, int64_t n, const Scale& sc,
             hipStream_t st)
{
    if (in_kind == BF16 && out_kind == BF16) return launch_stream16<BF16, BF16>(srcs, R, dst, n, sc, st);
    if (in_kind == BF16 && out_kind == Q32) return launch_stream16<BF16, Q32>(srcs, R, dst, n, sc, st);
    if (in_kind == Q32 && out_kind == BF16) return launch_stream16<Q32, BF16>(srcs, R, dst, n, sc, st);
    if (in_kind == F16 && out_kind == F16) return launch_stream16<F16, F16>(srcs, R, dst, n, sc, st);
    if (in_kind == F16 && out_kind == Q32) return launch_stream16<F16, Q32>(srcs, R, dst, n, sc, st);
    if (in_kind == Q32 && out_kind == F16) return launch_stream16<Q32, F16>(srcs, R, dst, n, sc, st);
#define INCCL_CASE(I, O) \
    if (in_kind == I && out_kind == O) return launch_stream<I, O>(srcs, R, dst, n, sc, st);
    INCCL_CASE(F32, F32) INCCL_CASE(F32, Q32) INCCL_CASE(F32, Q32BE)
    INCCL_CASE(Q32, F32) INCCL_CASE(Q32, Q32) INCCL_CASE(Q32, Q32BE)
    INCCL_CASE(Q32BE, F32) INCCL_CASE(Q32BE, Q32) INCCL_CASE(Q32BE, Q32BE)
#undef INCCL_CASE
    return INCCL_ERR_ARG;
}

bool scale_ok(int k) { return k >= INCCL_SCALE_MIN && k <= INCCL_SCALE_MAX; }

}  // namespace

namespace {

template <int E>
int launch_absmax(const void* const* srcs, int R, size_t n, uint32_t* amax_bits_dev, int zero_first, hipStream_t st)
{
    constexpr bool B16 = E != F32;
    if (R < 1 || R > kMaxR || amax_bits_dev == nullptr) return INCCL_ERR_ARG;
    SrcPtrs s = {};
    int vec = 1;
    for (int r = 0; r < R; ++r) {
        if (srcs[r] == nullptr) return INCCL_ERR_ARG;
        s.p[r] = srcs[r];
        vec = vec && aligned16(srcs[r]);
    }
    if (zero_first & ~(1 | INCCL_ABSMAX_FLAG_NONFINITE)) return INCCL_ERR_ARG;
    if (zero_first & 1) {
        hipError_t e = hipMemsetAsync(amax_bits_dev, 0, sizeof(uint32_t), st);
        if (e != hipSuccess) return (int)e;
    }
    const bool nf = (zero_first & INCCL_ABSMAX_FLAG_NONFINITE) != 0;
    if (n == 0) return 0;
    const int64_t tiles = ((int64_t)(n / (B16 ? 8 : 4)) + (int64_t)kAmBlock * kAmU - 1) / ((int64_t)kAmBlock * kAmU);
    const int64_t cap = (int64_t)num_cus() * 2;
    const int grid = (int)(tiles < 1 ? 1 : (tiles < cap ? tiles : cap));
    switch (R) {
#define INCCL_AM(RR)                                                                                             \
    case RR:                                                                                                     \
        if (nf)                                                                                                  \
            hipLaunchKernelGGL((k_absmax<RR, E, true>), dim3(grid), dim3(kAmBlock), 0, st, s, (int64_t)n,         \
                               amax_bits_dev, vec);                                                              \
        else                                                                                                     \
            hipLaunchKernelGGL((k_absmax<RR, E, false>), dim3(grid), dim3(kAmBlock), 0, st, s, (int64_t)n,        \
                               amax_bits_dev, vec);                                                              \
        break;
        INCCL_AM(1) INCCL_AM(2) INCCL_AM(3) INCCL_AM(4) INCCL_AM(5) INCCL_AM(6) INCCL_AM(7) INCCL_AM(8)
#undef INCCL_AM
    }
    return (int)hipGetLastError();
}

}  // namespace

extern "C" {

int inccl_k_stream_s(int in_kind, int out_kind, const void* const* srcs, int R, void* dst, size_t n, int scale_exp,
                     const uint32_t* amax_bits_dev, int scale_R, int out_shift, void* stream)
{
    if (amax_bits_dev == nullptr && !scale_ok(scale_exp)) return INCCL_ERR_ARG;
    if (dst == nullptr && n > 0) return INCCL_ERR_ARG;
    if (out_shift < 0 || out_shift > 8) return INCCL_ERR_ARG;
    Scale sc{scale_exp, amax_bits_dev, scale_R > 0 ? scale_R : R, out_shift};
    return dispatch(in_kind, out_kind, srcs, R, dst, (int64_t)n, sc, (hipStream_t)stream);
}

int inccl_k_stream(int in_kind, int out_kind, const void* const* srcs, int R, void* dst, size_t n, int scale_exp,
                   const uint32_t* amax_bits_dev, int scale_R, void* stream)
{
    return inccl_k_stream_s(in_kind, out_kind, srcs, R, dst, n, scale_exp, amax_bits_dev, scale_R, 0, stream);
}

int inccl_k_absmax(const float* const* srcs, int R, size_t n, uint32_t* amax_bits_dev, int zero_first, void* stream)
{
    return launch_absmax<F32>(reinterpret_cast<const void* const*>(srcs), R, n, amax_bits_dev, zero_first,
                              (hipStream_t)stream);
}

int inccl_k_absmax_bf16(const uint16_t* const* srcs, int R, size_t n, uint32_t* amax_bits_dev, int zero_first,
                        void* stream)
{
    return launch_absmax<BF16>(reinterpret_cast<const void* const*>(srcs), R, n, amax_bits_dev, zero_first,
                               (hipStream_t)stream);
}

int inccl_k_absmax_f16(const uint16_t* const* srcs, int R, size_t n, uint32_t* amax_bits_dev, int zero_first,
                       void* stream)
{
    return launch_absmax<F16>(reinterpret_cast<const void* const*>(srcs), R, n, amax_bits_dev, zero_first,
                              (hipStream_t)stream);
}

int inccl_k_checksum(const int32_t* q, size_t n, uint64_t index_base, uint32_t* out_dev, int zero_first, void* stream)
{
    hipStream_t st = (hipStream_t)stream;
    if (out_dev == nullptr || (q == nullptr && n > 0) || !aligned16(q)) return INCCL_ERR_ARG;
    if (zero_first) {
        hipError_t e = hipMemsetAsync(out_dev, 0, sizeof(uint32_t), st);
        if (e != hipSuccess) return (int)e;
    }
    if (n == 0) return 0;
    const int64_t blocks = ((int64_t)(n >> 2) + kBlock - 1) / kBlock;
    const int64_t cap = (int64_t)num_cus() * 8;
    const int grid = (int)(blocks < 1 ? 1 : (blocks < cap ? blocks : cap));
    hipLaunchKernelGGL(k_checksum, dim3(grid), dim3(kBlock), 0, st, reinterpret_cast<const uint32_t*>(q),
                       (int64_t)n, index_base, out_dev);
    return (int)hipGetLastError();
}

void inccl_k_set_tuning(int grid_cap, int nt_loads)
{
    g_grid_cap = grid_cap;
    g_nt_loads = nt_loads != 0;
}

}  // extern "C"
