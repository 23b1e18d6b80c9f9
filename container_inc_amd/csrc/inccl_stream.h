// inccl_stream.h -- device code of the generic streaming kernel (HIP, gfx950).
// Shared by the product (inccl_kernels.hip) and the variant tuner
// (tools/tune/tune_stream.hip), so the tuner measures exactly this code.
// See inccl_kernels.hip for the kernel family and the layout.
#ifndef INCCL_STREAM_H
#define INCCL_STREAM_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "inccl_amd.h"

namespace inccl_dev {

constexpr int kBlock = 256;   // default workgroup size
constexpr int kMaxR = INCCL_MAX_LOCAL_INPUTS;

enum Kind { F32 = 0, Q32 = 1, Q32BE = 2, BF16 = 3, F16 = 4 };

struct SrcPtrs {
    const void* p[kMaxR];
};

// Quantiser scale source: a static exponent, or the absmax word written by
// k_absmax (auto scaling, spec = orc_choose_scale).
struct Scale {
    int k;
    const uint32_t* amax_bits;  // nullptr -> use k
    int scale_R;                // contributors for auto scale
    int out_shift;              // dequantise with 2^-(k + out_shift): the sum / 2^out_shift
                                // (inccl_comm_set_average); exact, so bit-equal to dividing after
};

__device__ __forceinline__ float pow2f(int k) { return __uint_as_float((uint32_t)(k + 127) << 23); }

struct Scale;
__device__ __forceinline__ float deq_scale(const Scale& s, int k);

// Same arithmetic as orc_choose_scale (oracle/inccl_oracle.c).
__device__ __forceinline__ int choose_scale(float amax, int R)
{
    if (!(amax > 0.0f)) return INCCL_SCALE_MAX;
    if (__builtin_isinf(amax)) return INCCL_SCALE_MIN;
    double t = (double)amax * (double)R;
    int e;
    double m = frexp(t, &e);
    int k = (m == 0.5) ? (31 - e) : (30 - e);
    k = k < INCCL_SCALE_MIN ? INCCL_SCALE_MIN : k;
    k = k > INCCL_SCALE_MAX ? INCCL_SCALE_MAX : k;
    return k;
}

// the dequantise multiplier 2^-(k + out_shift); NaN when the auto scale's word
// carries bit 31 (INCCL_ABSMAX_FLAG_NONFINITE: some input of some rank was NaN
// or +-Inf), so that every result of the call is NaN
__device__ __forceinline__ float deq_scale(const Scale& s, int k)
{
    const float inv = pow2f(-k - s.out_shift);
    if (s.amax_bits != nullptr && (__builtin_nontemporal_load(s.amax_bits) >> 31)) return __builtin_nanf("");
    return inv;
}

__device__ __forceinline__ int resolve_k(const Scale& s)
{
    if (s.amax_bits == nullptr) return s.k;
    const uint32_t bits = __builtin_nontemporal_load(s.amax_bits);
    return choose_scale(__uint_as_float(bits), s.scale_R);
}

// sat_i32(rne(y)) with NaN -> 0: v_rndne_f32 then v_cvt_i32_f32, whose
// conversion saturates to [INT32_MIN, INT32_MAX] and maps NaN to 0 -- exactly
// the spec (orc_quantise_one), in 2 VALU ops where a compare/select form of the
// same rule takes 7.  (The saturation and NaN cases are in the GPU parity tests.)
__device__ __forceinline__ uint32_t quant_sat(float y)
{
    const float r = __builtin_rintf(y);
    int32_t q;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(q) : "v"(r));
    return (uint32_t)q;
}

// q = sat_i32(rne(x * 2^k)), NaN -> 0  (orc_quantise_one)
__device__ __forceinline__ uint32_t quant1(float x, float scale) { return quant_sat(x * scale); }

template <int IN>
__device__ __forceinline__ uint32_t load_xform(uint32_t raw, float scale)
{
    if constexpr (IN == F32) return quant1(__uint_as_float(raw), scale);
    else if constexpr (IN == Q32BE) return __builtin_bswap32(raw);
    else return raw;
}

template <int OUT>
__device__ __forceinline__ uint32_t store_xform(uint32_t acc, float inv)
{
    if constexpr (OUT == F32) return __float_as_uint((float)(int32_t)acc * inv);
    else if constexpr (OUT == Q32BE) return __builtin_bswap32(acc);
    else return acc;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Tile geometry per fan-in R, from the variant sweeps on MI355X.  Round 1
// (nontemporal stores; tools/tune/tune_stream.hip -> profiles/r01_tune_stream.jsonl,
// 2 x 256 MiB): one float4 per lane per input (U = 1) beat deeper per-lane
// unrolling for every R (e.g. R = 2: 6.96 TB/s at 512 x 1 vs 6.47 at 256 x 4);
// 512-lane workgroups win at R = 2..3, 1024-lane ones at R = 1 and R >= 4.
// Round 2 re-ran them with write-through stores (below, and
// profiles/r02/tune_stream_geometry_wt.jsonl, tune_r8.jsonl, tune_r1.jsonl).
template <int R>
struct Unroll {
    static constexpr int U = 1;
};
// R = 2 with write-through stores (round 2, tools/tune/tune_cold.hip,
// profiles/r02/tune_store_policy_wt.jsonl): 512 x 2 beats 512 x 1 both on
// repeated steps (110.7 vs 111.5-111.8 us) and on cold data (124.5-124.9 vs
// 125.1-127.2 us)
template <>
struct Unroll<2> {
    static constexpr int U = 2;
};
template <int R>
struct Geometry {
    static constexpr int BLOCK = (R == 2 || R == 3) ? 512 : 1024;
    static constexpr int U = Unroll<R>::U;
};

// Output store policy.  kStoreWT (sc1, write-through: the line leaves the L2)
// measured best on MI355X (tools/tune/tune_cold.hip, R = 2 x 256 MiB): 7.40 TB/s
// on repeated steps and 6.29-6.33 TB/s on cold data, against 6.96 / 6.10-6.13 for
// nontemporal stores and 7.06 / 6.14 for plain ones.  Write-through leaves no
// dirty output lines in L2: the inputs keep more of the caches, and the kernel
// boundary has nothing to write back.
constexpr int kStorePlain = 0, kStoreNT = 1, kStoreWT = 2;
constexpr int kAuxSc1 = 16;   // buffer instruction cache policy bit sc1

template <int IN, int OUT, int R, bool NT, int BLOCK = kBlock, int U = Unroll<R>::U, int SP = kStoreWT>
__global__ __launch_bounds__(BLOCK) void k_stream_vec(SrcPtrs src, void* __restrict__ dst, int64_t n4, Scale sc)
{
    const int k = resolve_k(sc);
    const float scale = pow2f(k);
    const float inv = deq_scale(sc, k);
    const int64_t tile_elems = (int64_t)BLOCK * U;
    const int64_t stride = (int64_t)gridDim.x * tile_elems;
    u32x4* __restrict__ out = reinterpret_cast<u32x4*>(dst);

    for (int64_t base = (int64_t)blockIdx.x * tile_elems; base < n4; base += stride) {
        const int64_t i0 = base + threadIdx.x;
        if (base + tile_elems <= n4) {
            // the tile's output through a buffer resource: the store's cache
            // policy is then explicit (a plain pointer store cannot carry sc1)
            const __amdgpu_buffer_rsrc_t orsrc =
                __builtin_amdgcn_make_buffer_rsrc(out + base, 0, (int)(tile_elems * 16), 0x00020000);
            u32x4 v[R][U];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const u32x4* p = reinterpret_cast<const u32x4*>(src.p[r]) + i0 + (int64_t)u * BLOCK;
                    v[r][u] = NT ? __builtin_nontemporal_load(p) : *p;
                }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    acc.x += load_xform<IN>(v[r][u].x, scale);
                    acc.y += load_xform<IN>(v[r][u].y, scale);
                    acc.z += load_xform<IN>(v[r][u].z, scale);
                    acc.w += load_xform<IN>(v[r][u].w, scale);
                }
                u32x4 o;
                o.x = store_xform<OUT>(acc.x, inv);
                o.y = store_xform<OUT>(acc.y, inv);
                o.z = store_xform<OUT>(acc.z, inv);
                o.w = store_xform<OUT>(acc.w, inv);
                if constexpr (SP == kStoreWT)
                    __builtin_amdgcn_raw_buffer_store_b128(o, orsrc, (int)((threadIdx.x + u * BLOCK) * 16), 0, kAuxSc1);
                else if constexpr (SP == kStoreNT)
                    __builtin_nontemporal_store(o, out + i0 + (int64_t)u * BLOCK);
                else
                    out[i0 + (int64_t)u * BLOCK] = o;
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = i0 + (int64_t)u * BLOCK;
                if (i < n4) {
                    u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const u32x4 x = reinterpret_cast<const u32x4*>(src.p[r])[i];
                        acc.x += load_xform<IN>(x.x, scale);
                        acc.y += load_xform<IN>(x.y, scale);
                        acc.z += load_xform<IN>(x.z, scale);
                        acc.w += load_xform<IN>(x.w, scale);
                    }
                    u32x4 o;
                    o.x = store_xform<OUT>(acc.x, inv);
                    o.y = store_xform<OUT>(acc.y, inv);
                    o.z = store_xform<OUT>(acc.z, inv);
                    o.w = store_xform<OUT>(acc.w, inv);
                    out[i] = o;
                }
            }
        }
    }
}

// ---- bfloat16 buckets: 2-byte elements, 8 per 16-B lane access ------------
// A bf16 value widens to fp32 exactly (its bits << 16), so quantisation is the
// fp32 rule on the widened value (quant_sat above: v_mul, v_rndne, saturating
// v_cvt_i32_f32); the dequantised fp32 sum narrows with round to nearest even
// through gfx950's v_cvt_pk_bf16_f32, one op per pair.  Twice the elements per
// byte of the fp32 path: with the earlier compare/select quantise (8 VALU ops an
// element) this kernel was issue-bound at 0.76 of HBM.  The sums are finite
// (|(float)s * 2^-k| <= 2^95): no NaN or overflow case in the narrowing.
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));


__device__ __forceinline__ uint32_t bf16_quant(uint32_t h, float scale) { return quant_sat(__uint_as_float(h << 16) * scale); }

__device__ __forceinline__ uint32_t deq_bf16x2(uint32_t a, uint32_t b, float inv)
{
    const f32x2 f = {(float)(int32_t)a * inv, (float)(int32_t)b * inv};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2));
}

// ---- IEEE binary16 (fp16) buckets: the same kernel, another 2-byte format ----
// A half widens to fp32 exactly (v_cvt_f32_f16: subnormals, Inf, NaN kept), so
// quantisation is again the fp32 rule on the widened value; the dequantised
// fp32 sum narrows with round to nearest even (v_cvt_f16_f32 under the default
// mode), overflowing to +-Inf past 65504 as IEEE narrowing does
// (orc_f32_to_f16).
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float f16_widen(uint32_t h) { return (float)__builtin_bit_cast(_Float16, (uint16_t)h); }

__device__ __forceinline__ uint32_t f16_quant(uint32_t h, float scale) { return quant_sat(f16_widen(h) * scale); }

__device__ __forceinline__ uint32_t deq_f16x2(uint32_t a, uint32_t b, float inv)
{
    const f32x2 f = {(float)(int32_t)a * inv, (float)(int32_t)b * inv};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, f16x2));
}

// a 2-byte format's element h (low 16 bits) quantised, and a pair of sums narrowed
template <int K>
__device__ __forceinline__ uint32_t quant16(uint32_t h, float scale)
{
    if constexpr (K == F16) return f16_quant(h, scale);
    else return bf16_quant(h, scale);
}
template <int K>
__device__ __forceinline__ uint32_t deq16x2(uint32_t a, uint32_t b, float inv)
{
    if constexpr (K == F16) return deq_f16x2(a, b, inv);
    else return deq_bf16x2(a, b, inv);
}
constexpr bool is16(int k) { return k == BF16 || k == F16; }

// out = OUT(sum_r IN(src_r)) over 8-element groups; IN, OUT in {BF16, F16,
// Q32}, not both Q32.  A workgroup owns BLOCK * U groups per tile; every load
// of the tile is issued before the arithmetic; full tiles store write-through
// (sc1) through a buffer resource as k_stream_vec does.
template <int IN, int OUT, int R, int BLOCK, int U>
__global__ __launch_bounds__(BLOCK) void k_stream16(SrcPtrs src, void* __restrict__ dst, int64_t n8, Scale sc)
{
    constexpr int VI = is16(IN) ? 1 : 2;    // u32x4 per group per input
    constexpr int VO = is16(OUT) ? 1 : 2;   // u32x4 per group of output
    const int k = resolve_k(sc);
    const float scale = pow2f(k);
    const float inv = deq_scale(sc, k);
    const int64_t tile = (int64_t)BLOCK * U;
    u32x4* __restrict__ out = reinterpret_cast<u32x4*>(dst);

    for (int64_t base = (int64_t)blockIdx.x * tile; base < n8; base += (int64_t)gridDim.x * tile) {
        const bool full = base + tile <= n8;
        u32x4 v[U][R][VI];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t g = base + threadIdx.x + (int64_t)u * BLOCK;
            if (full || g < n8)
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int w = 0; w < VI; ++w)
                        v[u][r][w] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src.p[r]) + g * VI + w);
        }
        __amdgpu_buffer_rsrc_t orsrc;
        if (full) orsrc = __builtin_amdgcn_make_buffer_rsrc(out + base * VO, 0, (int)(tile * VO * 16), 0x00020000);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t g = base + threadIdx.x + (int64_t)u * BLOCK;
            if (!full && g >= n8) continue;
            uint32_t acc[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if constexpr (is16(IN)) {
                    const u32x4 x = v[u][r][0];
                    acc[0] += quant16<IN>(x.x & 0xffffu, scale); acc[1] += quant16<IN>(x.x >> 16, scale);
                    acc[2] += quant16<IN>(x.y & 0xffffu, scale); acc[3] += quant16<IN>(x.y >> 16, scale);
                    acc[4] += quant16<IN>(x.z & 0xffffu, scale); acc[5] += quant16<IN>(x.z >> 16, scale);
                    acc[6] += quant16<IN>(x.w & 0xffffu, scale); acc[7] += quant16<IN>(x.w >> 16, scale);
                } else {
                    const u32x4 a = v[u][r][0], b = v[u][r][1];
                    acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
                    acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
                }
            }
            u32x4 o[VO];
            if constexpr (is16(OUT)) {
                o[0].x = deq16x2<OUT>(acc[0], acc[1], inv);
                o[0].y = deq16x2<OUT>(acc[2], acc[3], inv);
                o[0].z = deq16x2<OUT>(acc[4], acc[5], inv);
                o[0].w = deq16x2<OUT>(acc[6], acc[7], inv);
            } else {
                o[0] = u32x4{acc[0], acc[1], acc[2], acc[3]};
                o[VO - 1] = u32x4{acc[4], acc[5], acc[6], acc[7]};
            }
#pragma unroll
            for (int w = 0; w < VO; ++w) {
                if (full)
                    __builtin_amdgcn_raw_buffer_store_b128(o[w], orsrc,
                                                           (int)(((threadIdx.x + u * BLOCK) * VO + w) * 16), 0, kAuxSc1);
                else
                    out[g * VO + w] = o[w];
            }
        }
    }
}

}  // namespace inccl_dev

#endif
