// tune_stream.hip -- variant sweep of the product streaming kernel
// (container_inc_amd/csrc/inccl_stream.h) on two resident 256 MiB fp32 buckets,
// plus two memory-only references measured the same way: a float4 copy
// (1 read + 1 write) and a 2-read + 1-write add without the quantiser.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I container_inc_amd/csrc tools/tune/tune_stream.hip
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

__global__ void k_fill(float* p, int64_t n, uint32_t seed)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
        p[i] = ((float)(h & 0xFFFFFF) / 16777216.0f - 0.5f) * 8.0f;
    }
}

template <int BLOCK, int U>
__global__ __launch_bounds__(BLOCK) void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ o, int64_t n4)
{
    const int64_t base = (int64_t)blockIdx.x * BLOCK * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(a + base + (int64_t)u * BLOCK);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], o + base + (int64_t)u * BLOCK);
}

template <int BLOCK, int U>
__global__ __launch_bounds__(BLOCK) void k_add2(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                                u32x4* __restrict__ o, int64_t n4)
{
    const int64_t base = (int64_t)blockIdx.x * BLOCK * U + threadIdx.x;
    u32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        x[u] = __builtin_nontemporal_load(a + base + (int64_t)u * BLOCK);
        y[u] = __builtin_nontemporal_load(b + base + (int64_t)u * BLOCK);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(x[u] + y[u], o + base + (int64_t)u * BLOCK);
}

static hipEvent_t e0, e1;
static const int ITERS = 40;

template <class F>
static float time_ms(F f)
{
    for (int i = 0; i < 3; ++i) f();
    CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < ITERS; ++i) f();
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms / ITERS;
}

template <int IN, int OUT, int R, int BLOCK, int U>
static void variant(const SrcPtrs& s, void* out, int64_t n4, const char* name)
{
    Scale sc{25, nullptr, R};
    const int64_t tiles = n4 / ((int64_t)BLOCK * U);
    float ms = time_ms([&] {
        hipLaunchKernelGGL((k_stream_vec<IN, OUT, R, true, BLOCK, U>), dim3((unsigned)tiles), dim3(BLOCK), 0, 0, s,
                           out, n4, sc);
    });
    const double bytes = 16.0 * n4 * (R + 1);
    printf("{\"kernel\": \"%s\", \"R\": %d, \"block\": %d, \"U\": %d, \"grid\": %lld, \"ms\": %.5f, \"GBs\": %.1f}\n",
           name, R, BLOCK, U, (long long)tiles, ms, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

// cache-policy and grid-stride depth variants at the product geometry (R = 2: 512 x 1)
template <bool NT, bool NTS>
static void policy(const SrcPtrs& s, void* out, int64_t n4, int depth)
{
    Scale sc{25, nullptr, 2};
    const int64_t tiles = n4 / 512;
    const int64_t grid = tiles / depth;
    float ms = time_ms([&] {
        hipLaunchKernelGGL((k_stream_vec<F32, F32, 2, NT, 512, 1, NTS ? kStoreNT : kStorePlain>), dim3((unsigned)grid), dim3(512), 0, 0, s, out,
                           n4, sc);
    });
    printf("{\"kernel\": \"fused_policy\", \"R\": 2, \"nt_loads\": %d, \"nt_stores\": %d, \"tiles_per_block\": %d, "
           "\"ms\": %.5f, \"GBs\": %.1f}\n", NT, NTS, depth, ms, 48.0 * n4 / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

template <int IN, int OUT, int R>
static void sweep(const SrcPtrs& s, void* out, int64_t n4, const char* name)
{
    variant<IN, OUT, R, 256, 1>(s, out, n4, name);
    variant<IN, OUT, R, 256, 2>(s, out, n4, name);
    variant<IN, OUT, R, 256, 4>(s, out, n4, name);
    variant<IN, OUT, R, 512, 1>(s, out, n4, name);
    variant<IN, OUT, R, 512, 2>(s, out, n4, name);
    variant<IN, OUT, R, 1024, 1>(s, out, n4, name);
    variant<IN, OUT, R, 1024, 2>(s, out, n4, name);
}

template <int BLOCK, int U>
static void refs(const u32x4* a, const u32x4* b, u32x4* o, int64_t n4, int64_t n)
{
    const int64_t tiles = n4 / ((int64_t)BLOCK * U);
    float ms = time_ms([&] { hipLaunchKernelGGL((k_copy<BLOCK, U>), dim3((unsigned)tiles), dim3(BLOCK), 0, 0, a, o, n4); });
    printf("{\"kernel\": \"copy\", \"block\": %d, \"U\": %d, \"ms\": %.5f, \"GBs\": %.1f}\n", BLOCK, U, ms,
           8.0 * n / (ms * 1e-3) / 1e9);
    ms = time_ms([&] { hipLaunchKernelGGL((k_add2<BLOCK, U>), dim3((unsigned)tiles), dim3(BLOCK), 0, 0, a, b, o, n4); });
    printf("{\"kernel\": \"add2\", \"block\": %d, \"U\": %d, \"ms\": %.5f, \"GBs\": %.1f}\n", BLOCK, U, ms,
           12.0 * n / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

int main()
{
    const int64_t n = 1ll << 26, n4 = n >> 2;
    float *a, *b, *o;
    CHECK(hipMalloc(&a, n * 4));
    CHECK(hipMalloc(&b, n * 4));
    CHECK(hipMalloc(&o, n * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, a, n, 1u);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, b, n, 2u);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    float* extra[6];
    for (int i = 0; i < 6; ++i) {
        CHECK(hipMalloc(&extra[i], n * 4));
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, extra[i], n, 3u + i);
    }
    CHECK(hipDeviceSynchronize());
    SrcPtrs s = {};
    s.p[0] = a;
    s.p[1] = b;
    for (int i = 0; i < 6; ++i) s.p[2 + i] = extra[i];
    if (getenv("TUNE_POLICY")) {
        for (int rep = 0; rep < 3; ++rep)
            for (int depth : {1, 2, 4, 8}) {
                policy<true, true>(s, o, n4, depth);
                policy<false, true>(s, o, n4, depth);
                policy<true, false>(s, o, n4, depth);
                policy<false, false>(s, o, n4, depth);
            }
        return 0;
    }
    for (int rep = 0; rep < 2; ++rep) {
        sweep<F32, F32, 2>(s, o, n4, "fused");
        sweep<F32, F32, 1>(s, o, n4, "fused");
        sweep<F32, F32, 4>(s, o, n4, "fused");
        sweep<F32, F32, 8>(s, o, n4, "fused");
        sweep<F32, Q32, 2>(s, o, n4, "quant_sum");
        sweep<Q32, F32, 1>(s, o, n4, "dequant");
        refs<256, 4>((const u32x4*)a, (const u32x4*)b, (u32x4*)o, n4, n);
        refs<512, 1>((const u32x4*)a, (const u32x4*)b, (u32x4*)o, n4, n);
        refs<1024, 1>((const u32x4*)a, (const u32x4*)b, (u32x4*)o, n4, n);
    }
    return 0;
}
