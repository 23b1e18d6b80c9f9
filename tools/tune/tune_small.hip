// tune_small.hip -- the fused kernel (R = 2) on SMALL resident buckets (4 and
// 16 MiB), launched back to back on one stream exactly as bench.py's `sizes`
// rows time it: where do the 6.9 us of a 4 MiB launch go?  Variants: tile
// geometry, grid-stride depth, load policy (nt / plain), store policy
// (write-through / nt / plain), against an empty kernel (the launch floor) and
// a plain copy of the same bytes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I container_inc_amd/csrc tools/tune/tune_small.hip -o tools/tune/tune_small
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

__global__ void k_empty(int* p)
{
    if (p && threadIdx.x == 1023) p[0] = 0;
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ o, int64_t n4)
{
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n4) o[i] = a[i];
}

static hipEvent_t e0, e1;
static float *A, *B, *O;
static int64_t n, n4;
static const int kIters = 400;

template <class F>
static float time_ms(F f)
{
    for (int i = 0; i < 20; ++i) f();
    CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < kIters; ++i) f();
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms / kIters;
}

static void report(const char* name, int block, int u, int grid, int nt, int sp, float ms, double bytes)
{
    printf("{\"bucket_mib\": %lld, \"kernel\": \"%s\", \"block\": %d, \"U\": %d, \"grid\": %d, \"nt\": %d, \"store\": %d, "
           "\"us\": %.2f, \"GBs\": %.1f}\n",
           (long long)(n * 4 >> 20), name, block, u, grid, nt, sp, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

template <int BLOCK, int U, bool NT, int SP>
static void product(int depth)
{
    const int64_t tiles = (n4 + (int64_t)BLOCK * U - 1) / ((int64_t)BLOCK * U);
    int64_t grid = tiles / depth;
    if (grid < 1) grid = 1;
    SrcPtrs p = {};
    p.p[0] = A;
    p.p[1] = B;
    Scale sc{25, nullptr, 2};
    float ms = time_ms([&]() {
        hipLaunchKernelGGL((k_stream_vec<F32, F32, 2, NT, BLOCK, U, SP>), dim3((unsigned)grid), dim3(BLOCK), 0, 0, p, O,
                           n4, sc);
    });
    report("fused", BLOCK, U, (int)grid, NT, SP, ms, 12.0 * n);
}

static void floor_refs()
{
    float ms = time_ms([&]() { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, (int*)nullptr); });
    report("empty_1wg", 64, 0, 1, 0, 0, ms, 0.0);
    const int grid512 = (int)((n4 + 511) / 512);
    ms = time_ms([&]() { hipLaunchKernelGGL(k_empty, dim3(grid512), dim3(512), 0, 0, (int*)nullptr); });
    report("empty_same_grid", 512, 0, grid512, 0, 0, ms, 0.0);
    ms = time_ms([&]() {
        hipLaunchKernelGGL((k_copy<512>), dim3(grid512), dim3(512), 0, 0, (const u32x4*)A, (u32x4*)O, n4);
    });
    report("copy_plain", 512, 1, grid512, 0, 0, ms, 8.0 * n);
}

int main()
{
    const int64_t mibs[] = {4, 16, 32, 48, 64, 96, 128, 256, 1024};
    for (int64_t mib : mibs) {
        n = mib << 18;   // floats
        n4 = n >> 2;
        CHECK(hipMalloc(&A, n * 4));
        CHECK(hipMalloc(&B, n * 4));
        CHECK(hipMalloc(&O, n * 4));
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, A, n, 1u);
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, B, n, 2u);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        for (int rep = 0; rep < 2; ++rep) {
            if (mib > 16) {   // the load-policy crossover: nt vs plain loads, write-through stores
                product<512, 1, true, kStoreWT>(1);
                product<512, 1, false, kStoreWT>(1);
                continue;
            }
            floor_refs();
            product<512, 1, true, kStoreWT>(1);    // the product at every size
            product<512, 1, false, kStoreWT>(1);
            product<512, 1, false, kStorePlain>(1);
            product<512, 1, true, kStoreNT>(1);
            product<512, 1, false, kStoreNT>(1);
            product<256, 1, true, kStoreWT>(1);
            product<256, 1, false, kStorePlain>(1);
            product<1024, 1, true, kStoreWT>(1);
            product<512, 2, true, kStoreWT>(1);
            product<256, 2, false, kStorePlain>(1);
            product<512, 1, true, kStoreWT>(2);
            product<512, 1, false, kStorePlain>(2);
            product<256, 1, false, kStorePlain>(4);
        }
        CHECK(hipFree(A));
        CHECK(hipFree(B));
        CHECK(hipFree(O));
    }
    return 0;
}
