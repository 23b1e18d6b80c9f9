// tune_cold.hip -- the fused quantise+sum+dequantise kernel (R = 2, 256 MiB
// buckets) measured COLD: every launch rotates to a different one of S input /
// output sets (S * 768 MiB >> the 256 MiB Infinity Cache), so no launch finds
// its operands on die.  Variants: the product kernel at several geometries and
// cache policies, a per-XCD contiguous tile mapping, and memory-only references
// (2-read + 1-write add, copy) timed the same way.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I container_inc_amd/csrc tools/tune/tune_cold.hip -o tools/tune/tune_cold
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "inccl_stream.h"

using namespace inccl_dev;

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));  \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int kMaxSets = 4;
static int S = 4;   // sets rotated (argv[2]); 1 = every launch on the same set

__global__ void k_fill(float* p, int64_t n, uint32_t seed)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
        p[i] = ((float)(h & 0xFFFFFF) / 16777216.0f - 0.5f) * 8.0f;
    }
}

// one tile per workgroup, tiles dealt so that the workgroups of one XCD (b % 8,
// round-robin dispatch) stream one contiguous eighth of the buffers
template <int BLOCK, int U, bool NT, bool NTS>
__global__ __launch_bounds__(BLOCK) void k_xcd(SrcPtrs src, u32x4* __restrict__ out, int64_t n4, Scale sc)
{
    const float scale = pow2f(sc.k), inv = pow2f(-sc.k);
    const int64_t tiles = n4 / ((int64_t)BLOCK * U), per = tiles / 8;
    const int64_t b = blockIdx.x;
    const int64_t t = (b % 8) * per + b / 8;
    const u32x4* a = reinterpret_cast<const u32x4*>(src.p[0]);
    const u32x4* c = reinterpret_cast<const u32x4*>(src.p[1]);
    u32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = (t * U + u) * BLOCK + threadIdx.x;
        x[u] = NT ? __builtin_nontemporal_load(a + i) : a[i];
        y[u] = NT ? __builtin_nontemporal_load(c + i) : c[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = (t * U + u) * BLOCK + threadIdx.x;
        u32x4 o;
        o.x = __float_as_uint((float)(int32_t)(quant1(__uint_as_float(x[u].x), scale) + quant1(__uint_as_float(y[u].x), scale)) * inv);
        o.y = __float_as_uint((float)(int32_t)(quant1(__uint_as_float(x[u].y), scale) + quant1(__uint_as_float(y[u].y), scale)) * inv);
        o.z = __float_as_uint((float)(int32_t)(quant1(__uint_as_float(x[u].z), scale) + quant1(__uint_as_float(y[u].z), scale)) * inv);
        o.w = __float_as_uint((float)(int32_t)(quant1(__uint_as_float(x[u].w), scale) + quant1(__uint_as_float(y[u].w), scale)) * inv);
        if (NTS) __builtin_nontemporal_store(o, out + i);
        else out[i] = o;
    }
}

// the product kernel's tile (512 x 1) with the output stored through a buffer
// resource and an explicit cache policy: AUX = 16 (sc1: write-through, the line
// leaves L2) / 17 (sc0 sc1) / 2 (nt) / 0 (plain)
template <int BLOCK, int AUX>
__global__ __launch_bounds__(BLOCK) void k_store_policy(SrcPtrs src, u32x4* __restrict__ out, int64_t n4, Scale sc)
{
    const float scale = pow2f(sc.k), inv = pow2f(-sc.k);
    const int64_t t = blockIdx.x;
    const int64_t i = t * BLOCK + threadIdx.x;
    const u32x4* a = reinterpret_cast<const u32x4*>(src.p[0]);
    const u32x4* c = reinterpret_cast<const u32x4*>(src.p[1]);
    const u32x4 x = __builtin_nontemporal_load(a + i);
    const u32x4 y = __builtin_nontemporal_load(c + i);
    u32x4 o;
    o.x = __float_as_uint((float)(int32_t)(quant1(__uint_as_float(x.x), scale) + quant1(__uint_as_float(y.x), scale)) * inv);
    o.y = __float_as_uint((float)(int32_t)(quant1(__uint_as_float(x.y), scale) + quant1(__uint_as_float(y.y), scale)) * inv);
    o.z = __float_as_uint((float)(int32_t)(quant1(__uint_as_float(x.z), scale) + quant1(__uint_as_float(y.z), scale)) * inv);
    o.w = __float_as_uint((float)(int32_t)(quant1(__uint_as_float(x.w), scale) + quant1(__uint_as_float(y.w), scale)) * inv);
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(out + t * BLOCK, 0, BLOCK * 16, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(o, r, (int)(threadIdx.x * 16), 0, AUX);
}

// loads and stores through buffer resources with explicit cache policies
// (LAUX / SAUX: 0 plain, 2 nt, 16 sc1, 17 sc0 sc1), U float4 per lane per input
template <int BLOCK, int U, int LAUX, int SAUX>
__global__ __launch_bounds__(BLOCK) void k_policy(SrcPtrs src, u32x4* __restrict__ out, int64_t n4, Scale sc)
{
    const float scale = pow2f(sc.k), inv = pow2f(-sc.k);
    const int64_t base = (int64_t)blockIdx.x * BLOCK * U;
    const __amdgpu_buffer_rsrc_t ra =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(src.p[0]) , 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(src.p[1]), 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
    u32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int off = (int)((base + u * BLOCK + threadIdx.x) * 16);
        x[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, LAUX);
        y[u] = __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, LAUX);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        u32x4 o;
        o.x = __float_as_uint((float)(int32_t)(quant1(__uint_as_float(x[u].x), scale) + quant1(__uint_as_float(y[u].x), scale)) * inv);
        o.y = __float_as_uint((float)(int32_t)(quant1(__uint_as_float(x[u].y), scale) + quant1(__uint_as_float(y[u].y), scale)) * inv);
        o.z = __float_as_uint((float)(int32_t)(quant1(__uint_as_float(x[u].z), scale) + quant1(__uint_as_float(y[u].z), scale)) * inv);
        o.w = __float_as_uint((float)(int32_t)(quant1(__uint_as_float(x[u].w), scale) + quant1(__uint_as_float(y[u].w), scale)) * inv);
        __builtin_amdgcn_raw_buffer_store_b128(o, ro, (int)((base + u * BLOCK + threadIdx.x) * 16), 0, SAUX);
    }
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_add2(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                                u32x4* __restrict__ o, int64_t n4)
{
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i) + __builtin_nontemporal_load(b + i), o + i);
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ o, int64_t n4)
{
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), o + i);
}

static hipEvent_t e0, e1;
static float *A[kMaxSets], *B[kMaxSets], *O[kMaxSets];
static int64_t n, n4;

static bool g_hot = false;   // hot: every launch on set 0 (the bench's repeated step)

template <class F>
static float cold_ms(F f, int iters = 40)
{
    if (g_hot) {
        for (int i = 0; i < 3; ++i) f(0);
        CHECK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) f(0);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        return ms / iters;
    }
    for (int i = 0; i < S; ++i) f(i);
    CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) f(i % S);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms / iters;
}

static void report(const char* name, int block, int u, int depth, int nt, int nts, float ms, double bytes)
{
    printf("{\"mode\": \"%s\", \"kernel\": \"%s\", \"block\": %d, \"U\": %d, \"tiles_per_block\": %d, \"nt\": %d, \"nts\": %d, "
           "\"us\": %.2f, \"GBs\": %.1f}\n", g_hot ? "hot" : "cold", name, block, u, depth, nt, nts, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

template <int BLOCK, int U, bool NT, int SP>
static void product(int depth)
{
    const int64_t tiles = n4 / ((int64_t)BLOCK * U);
    const int64_t grid = tiles / depth;
    float ms = cold_ms([&](int s) {
        SrcPtrs p = {};
        p.p[0] = A[s];
        p.p[1] = B[s];
        Scale sc{25, nullptr, 2};
        hipLaunchKernelGGL((k_stream_vec<F32, F32, 2, NT, BLOCK, U, SP>), dim3((unsigned)grid), dim3(BLOCK), 0, 0, p,
                           O[s], n4, sc);
    });
    report("fused", BLOCK, U, depth, NT, SP, ms, 12.0 * n);
}

template <int BLOCK, int U, bool NT, bool NTS>
static void xcd()
{
    float ms = cold_ms([&](int s) {
        SrcPtrs p = {};
        p.p[0] = A[s];
        p.p[1] = B[s];
        Scale sc{25, nullptr, 2};
        hipLaunchKernelGGL((k_xcd<BLOCK, U, NT, NTS>), dim3((unsigned)(n4 / BLOCK / U)), dim3(BLOCK), 0, 0, p,
                           (u32x4*)O[s], n4, sc);
    });
    report("fused_xcd_contiguous", BLOCK, U, 1, NT, NTS, ms, 12.0 * n);
}

template <int BLOCK, int AUX>
static void store_policy()
{
    float ms = cold_ms([&](int s) {
        SrcPtrs p = {};
        p.p[0] = A[s];
        p.p[1] = B[s];
        Scale sc{25, nullptr, 2};
        hipLaunchKernelGGL((k_store_policy<BLOCK, AUX>), dim3((unsigned)(n4 / BLOCK)), dim3(BLOCK), 0, 0, p,
                           (u32x4*)O[s], n4, sc);
    });
    char name[64];
    snprintf(name, sizeof(name), "fused_store_aux%d", AUX);
    report(name, BLOCK, 1, 1, 1, AUX, ms, 12.0 * n);
}

template <int BLOCK, int U, int LAUX, int SAUX>
static void policy2()
{
    float ms = cold_ms([&](int s) {
        SrcPtrs p = {};
        p.p[0] = A[s];
        p.p[1] = B[s];
        Scale sc{25, nullptr, 2};
        hipLaunchKernelGGL((k_policy<BLOCK, U, LAUX, SAUX>), dim3((unsigned)(n4 / BLOCK / U)), dim3(BLOCK), 0, 0, p,
                           (u32x4*)O[s], n4, sc);
    });
    char name[64];
    snprintf(name, sizeof(name), "fused_load%d_store%d", LAUX, SAUX);
    report(name, BLOCK, U, 1, LAUX, SAUX, ms, 12.0 * n);
}

template <int BLOCK>
static void refs()
{
    float ms = cold_ms([&](int s) {
        hipLaunchKernelGGL((k_add2<BLOCK>), dim3((unsigned)(n4 / BLOCK)), dim3(BLOCK), 0, 0, (const u32x4*)A[s],
                           (const u32x4*)B[s], (u32x4*)O[s], n4);
    });
    report("add2_ref", BLOCK, 1, 1, 1, 1, ms, 12.0 * n);
    ms = cold_ms([&](int s) {
        hipLaunchKernelGGL((k_copy<BLOCK>), dim3((unsigned)(n4 / BLOCK)), dim3(BLOCK), 0, 0, (const u32x4*)A[s],
                           (u32x4*)O[s], n4);
    });
    report("copy_ref", BLOCK, 1, 1, 1, 1, ms, 8.0 * n);
}

// usage: tune_cold [MiB per bucket = 256] [sets = 4] [gap bytes]; e.g. 1024 1: the 1 GiB bucket, 3 GiB per launch
int main(int argc, char** argv)
{
    const int64_t mib = argc > 1 ? atoll(argv[1]) : 256;
    S = argc > 2 ? atoi(argv[2]) : 4;
    if (S < 1 || S > kMaxSets) S = 4;
    n = mib << 18;
    n4 = n >> 2;
    // argv[3] = gap: the three buckets of a set carved from one allocation with
    // `gap` bytes between them (DRAM channel / bank placement), else three allocations
    const int64_t gap = argc > 3 ? atoll(argv[3]) : -1;
    for (int s = 0; s < S; ++s) {
        if (gap >= 0) {
            char* base = nullptr;
            CHECK(hipMalloc(&base, 3 * n * 4 + 2 * gap));
            A[s] = (float*)base;
            B[s] = (float*)(base + n * 4 + gap);
            O[s] = (float*)(base + 2 * (n * 4 + gap));
        } else {
            CHECK(hipMalloc(&A[s], n * 4));
            CHECK(hipMalloc(&B[s], n * 4));
            CHECK(hipMalloc(&O[s], n * 4));
        }
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, A[s], n, 1u + 3 * s);
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, B[s], n, 2u + 3 * s);
    }
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < (S > 1 ? 4 : 2); ++rep) {
        g_hot = S > 1 ? (rep & 1) : 0;
        product<512, 2, true, kStoreWT>(1);   // the product since round 2 (write-through stores, 512 x 2)
        product<512, 1, true, kStoreWT>(1);
        product<512, 2, true, kStoreNT>(1);
        product<1024, 1, true, kStoreWT>(1);
        product<256, 2, true, kStoreWT>(1);
        product<512, 4, true, kStoreWT>(1);
        product<512, 2, false, kStoreWT>(1);
        refs<512>();
    }
    return 0;
}
