// tune_absmax.hip -- the auto-scale absmax pass (k_absmax in inccl_kernels.hip)
// over R = 2 resident 256 MiB fp32 buckets: the product form (one float4 per
// lane per input and grid-stride step, grid capped at 8 workgroups per CU)
// against deeper per-lane unrolling and other grid caps.  Reads only: algorithmic
// bytes R * 4 * n.  The product now uses 512 x 2 at 2 workgroups per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I container_inc_amd/csrc tools/tune/tune_absmax.hip -o tools/tune/tune_absmax
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

constexpr int R = 2;

__global__ void k_fill(float* p, int64_t n, uint32_t seed)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
        p[i] = ((float)(h & 0xFFFFFF) / 16777216.0f - 0.5f) * 8.0f;
    }
}

__device__ __forceinline__ uint32_t abs_bits(uint32_t b)
{
    const uint32_t a = b & 0x7fffffffu;
    return a > 0x7f800000u ? 0u : a;
}

__device__ __forceinline__ uint32_t amax4(u32x4 x)
{
    return max(max(abs_bits(x.x), abs_bits(x.y)), max(abs_bits(x.z), abs_bits(x.w)));
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)v, off, 64);
        v = v > o ? v : o;
    }
    return v;
}

template <int BLOCK>
__device__ __forceinline__ void block_max_atomic(uint32_t m, uint32_t* out)
{
    __shared__ uint32_t part[BLOCK / 64];
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t b = part[0];
#pragma unroll
        for (int w = 1; w < BLOCK / 64; ++w) b = b > part[w] ? b : part[w];
        atomicMax(out, b);
    }
}

// U float4 per lane per input per grid-stride step, all R*U loads issued first
template <int BLOCK, int U>
__global__ __launch_bounds__(BLOCK) void k_amax(SrcPtrs src, int64_t n4, uint32_t* out)
{
    uint32_t m = 0;
    const int64_t tile = (int64_t)BLOCK * U;
    for (int64_t base = (int64_t)blockIdx.x * tile; base < n4; base += (int64_t)gridDim.x * tile) {
        u32x4 v[R][U];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = base + threadIdx.x + (int64_t)u * BLOCK;
                v[r][u] = i < n4 ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src.p[r]) + i)
                                 : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t a = amax4(v[r][u]);
                m = m > a ? m : a;
            }
    }
    block_max_atomic<BLOCK>(m, out);
}

static hipEvent_t e0, e1;
static float* X[R];
static uint32_t* W;
static int64_t n, n4;

template <class F>
static float time_ms(F f, int iters = 40)
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

template <int BLOCK, int U>
static void variant(int64_t grid_cap)
{
    SrcPtrs p = {};
    for (int r = 0; r < R; ++r) p.p[r] = X[r];
    const int64_t tiles = (n4 + (int64_t)BLOCK * U - 1) / ((int64_t)BLOCK * U);
    const int64_t grid = tiles < grid_cap ? tiles : grid_cap;
    const float ms = time_ms([&]() {
        hipLaunchKernelGGL((k_amax<BLOCK, U>), dim3((unsigned)grid), dim3(BLOCK), 0, 0, p, n4, W);
    });
    const double bytes = R * 4.0 * (double)n;
    printf("{\"kernel\": \"absmax\", \"block\": %d, \"U\": %d, \"grid\": %lld, \"us\": %.2f, \"TBs\": %.3f, "
           "\"frac\": %.4f}\n",
           BLOCK, U, (long long)grid, ms * 1e3, bytes / (ms * 1e-3) / 1e12, bytes / (ms * 1e-3) / 8e12);
    fflush(stdout);
}

int main()
{
    n = 1ll << 26;
    n4 = n >> 2;
    for (int r = 0; r < R; ++r) {
        CHECK(hipMalloc(&X[r], n * 4));
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, X[r], n, 11u + r);
    }
    CHECK(hipMalloc(&W, 16));
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int rep = 0; rep < 2; ++rep) {
        variant<256, 1>(cus * 8);   // the round-2 product form
        variant<1024, 2>(cus * 2);
        variant<1024, 2>(cus * 1);
        variant<1024, 2>(cus * 3);
        variant<1024, 2>(cus * 4);
        variant<1024, 1>(cus * 2);
        variant<1024, 1>(cus * 4);
        variant<512, 2>(cus * 2);
        variant<512, 2>(cus * 3);
        variant<1024, 3>(cus * 2);
    }
    return 0;
}
