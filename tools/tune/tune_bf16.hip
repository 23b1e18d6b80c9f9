// tune_bf16.hip -- geometry sweep of the bf16 fused kernel k_stream16<BF16,BF16,R>
// (inccl_stream.h) on R resident 256 MiB bf16 buckets: workgroup size x groups
// of 8 elements per lane, repeated launches on one set ("hot") and rotated over
// two sets ("rot", 2 x (R+1) x 256 MiB, beyond the Infinity Cache).  Beside it a
// memory-only reference with the same access pattern (R nontemporal streams
// summed as integers, one write-through store) bounds what the geometry can reach.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I container_inc_amd/csrc tools/tune/tune_bf16.hip -o tools/tune/tune_bf16 [-DTUNE_R=2]
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

#ifndef TUNE_R
#define TUNE_R 2
#endif
constexpr int R = TUNE_R;

__global__ void k_fill(uint16_t* p, int64_t n, uint32_t seed)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
        const float f = ((float)(h & 0xFFFFFF) / 16777216.0f - 0.5f) * 8.0f;
        p[i] = (uint16_t)(__float_as_uint(f) >> 16);
    }
}

// memory only: R nontemporal streams of 16 B per lane, integer sum, one store
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_memref(SrcPtrs s, u32x4* __restrict__ o, int64_t n8)
{
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n8) return;
    u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int r = 0; r < R; ++r) acc += __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s.p[r]) + i);
    o[i] = acc;
}

static hipEvent_t e0, e1;
static uint16_t* X[2][R];
static uint16_t* O[2];
static int64_t n, n8;

template <class F>
static float time_ms(F f, int iters = 40)
{
    for (int i = 0; i < 5; ++i) f(i);
    CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) f(i);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms / iters;
}

static void report(const char* name, int block, int u, float hot, float rot)
{
    const double bytes = (R + 1) * 2.0 * (double)n;
    printf("{\"R\": %d, \"kernel\": \"%s\", \"block\": %d, \"U\": %d, \"hot_us\": %.2f, \"hot_frac\": %.4f, "
           "\"rot_us\": %.2f, \"rot_frac\": %.4f}\n",
           R, name, block, u, hot * 1e3, bytes / (hot * 1e-3) / 8e12, rot * 1e3, bytes / (rot * 1e-3) / 8e12);
    fflush(stdout);
}

static SrcPtrs set(int s)
{
    SrcPtrs p = {};
    for (int r = 0; r < R; ++r) p.p[r] = X[s][r];
    return p;
}

template <int BLOCK, int U>
static void variant()
{
    const int64_t grid = (n8 + (int64_t)BLOCK * U - 1) / ((int64_t)BLOCK * U);
    Scale sc{25, nullptr, R};
    auto launch = [&](int s) {
        hipLaunchKernelGGL((k_stream16<BF16, BF16, R, BLOCK, U>), dim3((unsigned)grid), dim3(BLOCK), 0, 0, set(s),
                           (void*)O[s], n8, sc);
    };
    const float hot = time_ms([&](int) { launch(0); });
    const float rot = time_ms([&](int i) { launch(i & 1); });
    report("k_stream16", BLOCK, U, hot, rot);
}

int main()
{
    n = 1ll << 27;   // 256 MiB of bf16
    n8 = n >> 3;
    for (int s = 0; s < 2; ++s) {
        for (int r = 0; r < R; ++r) {
            CHECK(hipMalloc(&X[s][r], n * 2));
            hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, X[s][r], n, 11u + r + 100u * s);
        }
        CHECK(hipMalloc(&O[s], n * 2));
    }
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep) {
        variant<512, 2>();   // the product geometry
        variant<512, 1>();
        variant<256, 1>();
        variant<256, 2>();
        variant<256, 4>();
        variant<1024, 1>();
        variant<1024, 2>();
        variant<512, 4>();
        const float hot = time_ms([&](int) {
            hipLaunchKernelGGL((k_memref<512>), dim3((unsigned)(n8 / 512)), dim3(512), 0, 0, set(0), (u32x4*)O[0], n8);
        });
        const float rot = time_ms([&](int i) {
            hipLaunchKernelGGL((k_memref<512>), dim3((unsigned)(n8 / 512)), dim3(512), 0, 0, set(i & 1),
                               (u32x4*)O[i & 1], n8);
        });
        report("memory_ref", 512, 1, hot, rot);
    }
    return 0;
}
