// tune_r8.hip -- the fused kernel with R = 8 local buckets of 256 MiB (BASELINE
// config 2's largest R): 9 streams per launch, 2.25 GiB, far beyond the
// Infinity Cache whether repeated or rotated.  Variants: workgroup size, quads
// per lane, grid-stride depth, nontemporal vs plain loads; write-through stores
// (the product's policy); a 9-stream memory-only reference.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I container_inc_amd/csrc tools/tune/tune_r8.hip -o tools/tune/tune_r8
// (-DTUNE_R=1 -o tools/tune/tune_r1: the same sweep at R = 1)
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
#define TUNE_R 8   // -DTUNE_R=1 for config 2's R = 1
#endif
constexpr int R = TUNE_R;

__global__ void k_fill(float* p, int64_t n, uint32_t seed)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
        p[i] = ((float)(h & 0xFFFFFF) / 16777216.0f - 0.5f) * 8.0f;
    }
}

// memory only: sum of 8 nontemporal streams, one plain store
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_sum8(SrcPtrs s, u32x4* __restrict__ o, int64_t n4)
{
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int r = 0; r < R; ++r) acc += __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s.p[r]) + i);
    o[i] = acc;
}

static hipEvent_t e0, e1;
static float* XS[2][R];   // input sets (argv[1] = 2: launches alternate between them, cold)
static float* OS[2];
static int g_sets = 1, g_turn = 0;
static float** X = XS[0];
static float* O;
// the next launch's set
static void next_set()
{
    const int s = g_turn++ % g_sets;
    X = XS[s];
    O = OS[s];
}
static int64_t n, n4;

template <class F>
static float time_ms(F f, int iters = 30)
{
    for (int i = 0; i < 5; ++i) f();
    CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) f();
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms / iters;
}

static void report(const char* name, int block, int u, int64_t grid, int nt, float ms)
{
    const double bytes = (R + 1) * 4.0 * (double)n;
    printf("{\"R\": %d, \"kernel\": \"%s\", \"block\": %d, \"U\": %d, \"grid\": %lld, \"nt\": %d, \"us\": %.2f, "
           "\"TBs\": %.3f, \"frac\": %.4f}\n",
           R, name, block, u, (long long)grid, nt, ms * 1e3, bytes / (ms * 1e-3) / 1e12, bytes / (ms * 1e-3) / 8e12);
    fflush(stdout);
}

template <int BLOCK, int U, bool NT>
static void product(int depth)
{
    const int64_t tiles = n4 / ((int64_t)BLOCK * U);
    const int64_t grid = tiles / depth;
    Scale sc{25, nullptr, R};
    float ms = time_ms([&]() {
        next_set();
        SrcPtrs p = {};
        for (int r = 0; r < R; ++r) p.p[r] = X[r];
        hipLaunchKernelGGL((k_stream_vec<F32, F32, R, NT, BLOCK, U, kStoreWT>), dim3((unsigned)grid), dim3(BLOCK), 0, 0,
                           p, O, n4, sc);
    });
    report("fused", BLOCK, U, grid, NT, ms);
}

// usage: tune_r8 [sets = 1]; 2 alternates two input / output sets (4.5 GiB: cold)
int main(int argc, char** argv)
{
    g_sets = argc > 1 && atoi(argv[1]) == 2 ? 2 : 1;
    n = 1ll << 26;
    n4 = n >> 2;
    for (int s = 0; s < g_sets; ++s) {
        for (int r = 0; r < R; ++r) {
            CHECK(hipMalloc(&XS[s][r], n * 4));
            hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, XS[s][r], n, 11u + r + 16 * s);
        }
        CHECK(hipMalloc(&OS[s], n * 4));
    }
    next_set();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep) {
        product<1024, 1, true>(1);   // the product geometry for R = 8
        product<1024, 1, false>(1);
        product<512, 1, true>(1);
        product<512, 1, false>(1);
        product<256, 1, true>(1);
        product<256, 2, true>(1);
        product<512, 2, true>(1);
        product<1024, 1, true>(2);
        product<1024, 1, true>(4);
        product<512, 1, true>(4);
        float ms = time_ms([&]() {
            next_set();
            SrcPtrs p = {};
            for (int r = 0; r < R; ++r) p.p[r] = X[r];
            hipLaunchKernelGGL((k_sum8<512>), dim3((unsigned)(n4 / 512)), dim3(512), 0, 0, p, (u32x4*)O, n4);
        });
        report("sum8_memory_ref", 512, 1, n4 / 512, 1, ms);
    }
    return 0;
}
