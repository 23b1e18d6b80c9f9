// tune_peer.hip -- the p2p engine's pull-reduce (k_peer_reduce's shape: W int32
// shards -> one dequantised fp32 shard) on LOCAL buffers in one process, with
// the peer-load cache policy varied: sc0 sc1 (the product: system-coherent, for
// memory other GPUs write), nt, plain.  Isolates what the policy costs in HBM
// terms; on a real mesh these loads cross xGMI.  W = 2 and 8, 128 MiB shards.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I container_inc_amd/csrc tools/tune/tune_peer.hip -o tools/tune/tune_peer
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

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

template <int W, int BLOCK, int U, int LAUX>
__global__ __launch_bounds__(BLOCK) void k_reduce(SrcPtrs src, float* __restrict__ dst, int64_t n4, float inv)
{
    u32x4* out = reinterpret_cast<u32x4*>(dst);
    const int64_t base = (int64_t)blockIdx.x * BLOCK * U;
    const uint32_t tile_bytes = (uint32_t)(BLOCK * U * 16);
    u32x4 v[U][W];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < W; ++r)
            v[u][r] = __builtin_amdgcn_raw_buffer_load_b128(rsrc(reinterpret_cast<const u32x4*>(src.p[r]) + base, tile_bytes),
                                                            (int)((threadIdx.x + u * BLOCK) * 16u), 0, LAUX);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        u32x4 acc = v[u][0];
#pragma unroll
        for (int r = 1; r < W; ++r) acc += v[u][r];
        u32x4 o;
        o.x = __float_as_uint((float)(int32_t)acc.x * inv);
        o.y = __float_as_uint((float)(int32_t)acc.y * inv);
        o.z = __float_as_uint((float)(int32_t)acc.z * inv);
        o.w = __float_as_uint((float)(int32_t)acc.w * inv);
        __builtin_amdgcn_raw_buffer_store_b128(o, rsrc(out + base, tile_bytes), (int)((threadIdx.x + u * BLOCK) * 16u), 0, 16);
    }
}

static hipEvent_t e0, e1;
static int32_t* P[8];
static float* O;
static const int64_t n = 1ll << 25;   // 128 MiB shards
static const int64_t n4 = n >> 2;

template <int W, int BLOCK, int U, int LAUX>
static void run(const char* policy)
{
    SrcPtrs s = {};
    for (int r = 0; r < W; ++r) s.p[r] = P[r];
    auto f = [&]() {
        hipLaunchKernelGGL((k_reduce<W, BLOCK, U, LAUX>), dim3((unsigned)(n4 / (BLOCK * U))), dim3(BLOCK), 0, 0, s, O, n4,
                           1.0f / 33554432.0f);
    };
    for (int i = 0; i < 5; ++i) f();
    CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < 30; ++i) f();
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 30;
    const double bytes = (W + 1) * 4.0 * n;
    printf("{\"W\": %d, \"policy\": \"%s\", \"block\": %d, \"U\": %d, \"us\": %.2f, \"TBs\": %.3f}\n", W, policy, BLOCK,
           U, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    fflush(stdout);
}

int main()
{
    for (int r = 0; r < 8; ++r) {
        CHECK(hipMalloc(&P[r], n * 4));
        CHECK(hipMemset(P[r], r + 1, n * 4));
    }
    CHECK(hipMalloc(&O, n * 4));
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep) {
        run<2, 512, 1, 17>("sc0sc1 (product)");
        run<2, 512, 1, 19>("sc0sc1nt");
        run<2, 512, 1, 18>("sc1nt");
        run<2, 512, 1, 3>("sc0nt");
        run<2, 512, 1, 2>("nt");
        run<2, 512, 1, 0>("plain");
        run<2, 512, 2, 17>("sc0sc1 U2");
        run<2, 512, 2, 2>("nt U2");
        run<8, 1024, 1, 17>("sc0sc1 (product)");
        run<8, 1024, 1, 19>("sc0sc1nt");
        run<8, 1024, 1, 2>("nt");
        run<8, 1024, 1, 0>("plain");
    }
    return 0;
}
