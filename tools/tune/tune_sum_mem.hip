// tune_sum_mem.hip -- memory-only references for the switch's sum kernel
// (k_ingress_sum, inccl_frames.hip): its HBM traffic with no classification
// and no payload extraction, to price the sum's 35 us against.
//
// Workload = the fan-in-2 sum of one 131 072-frame batch: 65 536 PSNs whose two
// copies are consecutive frames (1152-B rows).  A wave per frame pair, 8-wave
// blocks, as the sum: both rows' chunks 3-66 (lane l: byte 48 + 16 l) and
// chunks 67-68 (lanes 0-1) in one round trip, then the 1 KiB aggregate stored
// (write-through, as the sum does), the leader's 4-B action word, and the
// slot's degree counted by two atomics.  Algorithmic bytes as DESIGN.md counts
// them for the sum: fan_in x 1 KiB read + 1 KiB written per PSN (201 MB).
//
// Variants: the full traffic; without the action word and atomics; nt or plain
// aggregate stores; loads only.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_sum_mem.hip -o tools/tune/tune_sum_mem
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));  \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;
constexpr int kWaves = 8;               // waves per block, as the sum
constexpr int kPsns = 65536;
constexpr int kStride = 1152;           // input row stride
constexpr int kOob = 0x40000000;        // past every buffer: the access is dropped

// STORE: 0 none, else the aggregate store's cache policy + 1 (1 plain, 3 nt,
// 17 write-through); META: the action word and the degree atomics
template <int STORE, bool META>
__global__ __launch_bounds__(kWave* kWaves) void k_sum_mem(const uint8_t* __restrict__ frames, u4* __restrict__ agg,
                                                          int32_t* __restrict__ action, int32_t* __restrict__ degree)
{
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    const int p = blockIdx.x * kWaves + w;   // the PSN; frames 2p, 2p + 1
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(frames) + (size_t)2 * p * kStride, 0, 2 * kStride, 0x00020000);
    u4 x[2], e[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        x[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, k * kStride + 48 + 16 * lane, 0, 0);
        e[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane < 2 ? k * kStride + 1072 + 16 * lane : kOob, 0, 0);
    }
    // something of every loaded word reaches the stored sum, so no load is dead
    const uint32_t t = __builtin_amdgcn_readlane((int)(e[0].x ^ e[1].y ^ e[0].z ^ e[1].w), 0);
    const u4 acc = x[0] + x[1] + t;
    if (STORE) {
        const __amdgpu_buffer_rsrc_t ra =
            __builtin_amdgcn_make_buffer_rsrc(agg + (size_t)p * kWave, 0, 1024, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(acc, ra, 16 * lane, 0, STORE - 1);
    } else if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u) {   // (never: keeps the loads live)
        agg[lane] = acc;
    }
    if (META && lane == 0) {
        action[2 * p + 1] = 2;
        atomicAdd(&degree[p], 1);
        atomicAdd(&degree[p], 1);
    }
}

static hipEvent_t e0, e1;

template <int STORE, bool META>
static void run(const char* name, const uint8_t* frames, u4* agg, int32_t* action, int32_t* degree, int iters)
{
    auto launch = [&]() { k_sum_mem<STORE, META><<<kPsns / kWaves, kWave * kWaves>>>(frames, agg, action, degree); };
    for (int i = 0; i < 3; ++i) launch();
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / iters;
    const double alg = (double)kPsns * 3 * 1024;   // the sum's algorithmic bytes
    printf("{\"variant\": \"%s\", \"store_aux_plus1\": %d, \"meta\": %s, \"us\": %.2f, \"sum_alg_TBs\": %.3f, "
           "\"frac_of_8TBs\": %.3f}\n",
           name, STORE, META ? "true" : "false", us, alg / us * 1e-6, alg / us * 1e-6 / 8.0);
    fflush(stdout);
}

int main(int argc, char** argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 50;
    uint8_t* frames;
    u4* agg;
    int32_t *action, *degree;
    CHECK(hipMalloc(&frames, (size_t)2 * kPsns * kStride));
    CHECK(hipMalloc(&agg, (size_t)kPsns * 1024));
    CHECK(hipMalloc(&action, (size_t)2 * kPsns * 4));
    CHECK(hipMalloc(&degree, (size_t)kPsns * 4));
    CHECK(hipMemset(frames, 3, (size_t)2 * kPsns * kStride));
    CHECK(hipMemset(degree, 0, (size_t)kPsns * 4));
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    run<17, true>("sum traffic: loads, write-through aggregate, action + degree atomics", frames, agg, action, degree, iters);
    run<17, false>("loads + write-through aggregate", frames, agg, action, degree, iters);
    run<3, true>("nt aggregate, action + atomics", frames, agg, action, degree, iters);
    run<1, true>("plain aggregate, action + atomics", frames, agg, action, degree, iters);
    run<0, false>("loads only", frames, agg, action, degree, iters);
    CHECK(hipFree(frames));
    CHECK(hipFree(agg));
    CHECK(hipFree(action));
    CHECK(hipFree(degree));
    return 0;
}
