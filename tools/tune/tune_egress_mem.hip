// tune_egress_mem.hip -- memory-only references for the switch egress kernel
// (k_egress<2, true>, inccl_frames.hip): the same HBM traffic with no frame
// building and no CRC, to price what the egress's 45 us are against.
//
// Workload = the fan-in-2 egress of one 131 072-frame batch: 65 536 completed
// PSNs, each reading its 1 KiB aggregate and writing fan_in = 2 output frames
// of 1082 B into 1152-B rows (a 1024-B store of 64 lanes x 16 B, then a 64-B
// tail store of 4 lanes), the output rows of input frame 2p + 1 (rows 4p + 2
// and 4p + 3: the completing copy is the second of each pair), plus the 4-B
// row lengths of every output row.  Algorithmic bytes as DESIGN.md counts them
// for the egress: 1 KiB per emitting input frame + 1.09 KB per output frame.
//
// Variants: stores only or aggregate read + stores; nt / plain / write-through
// stores; a persistent grid of 2 x 16-wave blocks per CU walking chunks of G
// PSNs (the egress's shape) or one wave per chunk.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_egress_mem.hip -o tools/tune/tune_egress_mem
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
constexpr int kWaves = 16;              // waves per block, as the egress
constexpr int kPsns = 65536;            // completed PSNs per batch
constexpr int kFan = 2;
constexpr int kStride = 1152;           // output row stride
constexpr int kTail = 4;                // 16-B chunks past the first 1024 B (1082-B frames)
constexpr int kOob = 0x40000000;        // an offset past every buffer: the access is dropped

// G PSNs per chunk; PERSIST: a grid of 2 blocks per CU walks the chunks, else a
// wave per chunk.  READ: load the aggregate.  AUX: store cache policy.  ALU:
// dependent VALU operations per PSN on its aggregate before its rows are
// stored; LDS: random 4-byte LDS table lookups per PSN among them (the frame
// work's stand-ins: how much compute the traffic hides)
template <int G, bool PERSIST, bool READ, int AUX, int ALU = 0, int LDS = 0, int ILP = 1>
__global__ __launch_bounds__(kWave* kWaves) void k_egress_mem(const u4* __restrict__ agg, uint8_t* __restrict__ out,
                                                             uint32_t* __restrict__ out_len)
{
    __shared__ uint32_t tab[LDS ? 4096 : 1];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    if (LDS) {
        for (int i = threadIdx.x; i < 4096; i += blockDim.x) tab[i] = (uint32_t)i * 2654435761u;
        __syncthreads();
    }
    const uint32_t chunks = kPsns / G;
    const uint32_t nw = PERSIST ? gridDim.x * kWaves : chunks;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<u4*>(agg), 0, kPsns * 1024, 0x00020000);
    const __amdgpu_buffer_rsrc_t ro =
        __builtin_amdgcn_make_buffer_rsrc(out, 0, kPsns * 2 * kFan * kStride, 0x00020000);   // < kOob
    const __amdgpu_buffer_rsrc_t rl =
        __builtin_amdgcn_make_buffer_rsrc(out_len, 0, 4 * kPsns * 2 * kFan, 0x00020000);
    for (uint32_t ch = blockIdx.x * kWaves + w; ch < chunks; ch += nw) {
        u4 a[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint32_t p = ch * G + g;
            a[g] = READ ? __builtin_amdgcn_raw_buffer_load_b128(ra, (int)(p * 1024 + 16 * lane), 0, 0)
                        : u4{p, (uint32_t)lane, 0u, 0u};
        }
        // the chunk's row lengths: 2 G input frames x kFan rows
        __builtin_amdgcn_raw_buffer_store_b32(lane & 2 ? 1086u : 0u, rl,
                                              lane < 2 * G * kFan ? (int)(4 * (ch * 2 * G * kFan + lane)) : kOob, 0, 0);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint32_t p = ch * G + g;
            if (ALU || LDS) {
                // ALU operations in ILP independent chains (two dependent
                // operations per step of a chain)
                uint32_t hc[ILP];
#pragma unroll
                for (int k = 0; k < ILP; ++k) hc[k] = a[g][k & 3] + (uint32_t)k;
#pragma unroll
                for (int i = 0; i < ALU / ILP; i += 2) {
#pragma unroll
                    for (int k = 0; k < ILP; ++k) {
                        hc[k] ^= hc[k] << 7;
                        hc[k] = __builtin_amdgcn_alignbyte(hc[k], hc[k] ^ 0x9E3779B9u, 1);
                    }
                }
                uint32_t h = 0;
#pragma unroll
                for (int k = 0; k < ILP; ++k) h ^= hc[k];
                uint32_t x = 0;   // independent lookups, as the ICRC's (random words of one table)
#pragma unroll
                for (int i = 0; i < LDS; ++i) x ^= tab[((h >> (i % 20)) + 97u * (uint32_t)i) & 4095u];
                a[g].w ^= h ^ x;
            }
#pragma unroll
            for (int c = 0; c < kFan; ++c) {
                const int64_t row = (int64_t)(2 * p + 1) * kFan + c;
                const u4 v = a[g] + (uint32_t)c;
                __builtin_amdgcn_raw_buffer_store_b128(v, ro, (int)(row * kStride + 16 * lane), 0, AUX);
                __builtin_amdgcn_raw_buffer_store_b128(v, ro, lane < kTail ? (int)(row * kStride + 1024 + 16 * lane) : kOob,
                                                       0, AUX);
            }
        }
    }
}

// Split waves (an upper bound for a specialised egress, no hand-over between
// them): waves 0-7 of each block do the memory-only loop (chunks of 2 PSNs),
// waves 8-15 read the same PSNs' aggregates and do ALU VALU operations per PSN in
// four chains, writing 4 B per PSN (the ICRC a store wave would need).
template <int ALU>
__global__ __launch_bounds__(kWave* kWaves) void k_egress_split(const u4* __restrict__ agg, uint8_t* __restrict__ out,
                                                               uint32_t* __restrict__ out_len, uint32_t* __restrict__ crc)
{
    constexpr int G = 2;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    const bool storer = w < kWaves / 2;
    const uint32_t chunks = kPsns / G, nw = gridDim.x * (kWaves / 2);
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<u4*>(agg), 0, kPsns * 1024, 0x00020000);
    const __amdgpu_buffer_rsrc_t ro =
        __builtin_amdgcn_make_buffer_rsrc(out, 0, kPsns * 2 * kFan * kStride, 0x00020000);
    const __amdgpu_buffer_rsrc_t rl =
        __builtin_amdgcn_make_buffer_rsrc(out_len, 0, 4 * kPsns * 2 * kFan, 0x00020000);
    for (uint32_t ch = blockIdx.x * (kWaves / 2) + (w % (kWaves / 2)); ch < chunks; ch += nw) {
        u4 a[G];
#pragma unroll
        for (int g = 0; g < G; ++g) a[g] = __builtin_amdgcn_raw_buffer_load_b128(ra, (int)((ch * G + g) * 1024 + 16 * lane), 0, 0);
        if (storer) {
            __builtin_amdgcn_raw_buffer_store_b32(lane & 2 ? 1086u : 0u, rl,
                                                  lane < 2 * G * kFan ? (int)(4 * (ch * 2 * G * kFan + lane)) : kOob, 0, 0);
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const uint32_t p = ch * G + g;
#pragma unroll
                for (int c = 0; c < kFan; ++c) {
                    const int64_t row = (int64_t)(2 * p + 1) * kFan + c;
                    const u4 v = a[g] + (uint32_t)c;
                    __builtin_amdgcn_raw_buffer_store_b128(v, ro, (int)(row * kStride + 16 * lane), 0, 2);
                    __builtin_amdgcn_raw_buffer_store_b128(v, ro, lane < kTail ? (int)(row * kStride + 1024 + 16 * lane) : kOob,
                                                           0, 2);
                }
            }
        } else {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                uint32_t hc[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) hc[k] = a[g][k] + (uint32_t)k;
#pragma unroll
                for (int i = 0; i < ALU / 4; i += 2) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        hc[k] ^= hc[k] << 7;
                        hc[k] = __builtin_amdgcn_alignbyte(hc[k], hc[k] ^ 0x9E3779B9u, 1);
                    }
                }
                const uint32_t h = hc[0] ^ hc[1] ^ hc[2] ^ hc[3];
                if (lane == 0) crc[ch * G + g] = h;
            }
        }
    }
}

static hipEvent_t e0, e1;

template <int G, bool PERSIST, bool READ, int AUX, int ALU = 0, int LDS = 0, int ILP = 1>
static void run(const char* name, const u4* agg, uint8_t* out, uint32_t* len, int cus, int iters)
{
    const int blocks = PERSIST ? 2 * cus : (kPsns / G + kWaves - 1) / kWaves;
    auto launch = [&]() { k_egress_mem<G, PERSIST, READ, AUX, ALU, LDS, ILP><<<blocks, kWave * kWaves>>>(agg, out, len); };
    for (int i = 0; i < 3; ++i) launch();
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / iters;
    // the egress's algorithmic bytes: 1 KiB per emitting input frame + 1.09 KB
    // (1082-B frame + 4-B length, the DESIGN.md per-frame figure) per output frame
    const double alg = (double)kPsns * 1024 + (double)kPsns * kFan * 1090;
    const double stored = (double)kPsns * kFan * (1024 + 16 * kTail);
    printf("{\"variant\": \"%s\", \"chunk_psns\": %d, \"persistent\": %s, \"read\": %s, \"store_aux\": %d, "
           "\"valu_per_psn\": %d, \"valu_chains\": %d, \"lds_per_psn\": %d, "
           "\"us\": %.2f, \"egress_alg_TBs\": %.3f, \"frac_of_8TBs\": %.3f, \"store_TBs\": %.3f}\n",
           name, G, PERSIST ? "true" : "false", READ ? "true" : "false", AUX, ALU, ILP, LDS, us, alg / us * 1e-6, alg / us * 1e-6 / 8.0,
           stored / us * 1e-6);
    fflush(stdout);
}

template <int ALU>
static void run_split(const char* name, const u4* agg, uint8_t* out, uint32_t* len, uint32_t* crc, int cus, int iters)
{
    auto launch = [&]() { k_egress_split<ALU><<<2 * cus, kWave * kWaves>>>(agg, out, len, crc); };
    for (int i = 0; i < 3; ++i) launch();
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / iters;
    const double alg = (double)kPsns * 1024 + (double)kPsns * kFan * 1090;
    printf("{\"variant\": \"%s\", \"valu_per_psn\": %d, \"us\": %.2f, \"egress_alg_TBs\": %.3f}\n", name, ALU, us,
           alg / us * 1e-6);
    fflush(stdout);
}

int main(int argc, char** argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 50;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    u4* agg;
    uint8_t* out;
    uint32_t* len;
    CHECK(hipMalloc(&agg, (size_t)kPsns * 1024));
    CHECK(hipMalloc(&out, (size_t)kPsns * 2 * kFan * kStride));
    CHECK(hipMalloc(&len, (size_t)kPsns * 2 * kFan * 4));
    CHECK(hipMemset(agg, 1, (size_t)kPsns * 1024));
    CHECK(hipMemset(out, 0, (size_t)kPsns * 2 * kFan * kStride));
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    // the egress's shape: persistent, chunks of 2 PSNs (4 input frames), nt stores
    run<2, true, true, 2>("egress shape, nt", agg, out, len, cus, iters);
    run<2, true, true, 0>("egress shape, plain", agg, out, len, cus, iters);
    run<2, true, true, 16>("egress shape, write-through", agg, out, len, cus, iters);
    run<2, true, false, 2>("stores only, nt", agg, out, len, cus, iters);
    run<1, true, true, 2>("1 psn per chunk, nt", agg, out, len, cus, iters);
    run<4, true, true, 2>("4 psns per chunk, nt", agg, out, len, cus, iters);
    run<2, false, true, 2>("wave per chunk, nt", agg, out, len, cus, iters);
    run<2, false, false, 2>("wave per chunk, stores only, nt", agg, out, len, cus, iters);
    // the egress shape with compute stand-ins per PSN (the product: about 228
    // VALU and 40 LDS reads per emitting frame)
    run<2, true, true, 2, 100, 0>("egress shape + 100 VALU", agg, out, len, cus, iters);
    run<2, true, true, 2, 200, 0>("egress shape + 200 VALU", agg, out, len, cus, iters);
    run<2, true, true, 2, 400, 0>("egress shape + 400 VALU", agg, out, len, cus, iters);
    run<2, true, true, 2, 0, 40>("egress shape + 40 LDS lookups", agg, out, len, cus, iters);
    run<2, true, true, 2, 200, 40>("egress shape + 200 VALU + 40 LDS lookups", agg, out, len, cus, iters);
    run<2, true, true, 2, 200, 0, 4>("egress shape + 200 VALU in 4 chains", agg, out, len, cus, iters);
    run<2, true, true, 2, 400, 0, 4>("egress shape + 400 VALU in 4 chains", agg, out, len, cus, iters);
    run<2, true, true, 2, 200, 40, 4>("egress shape + 200 VALU in 4 chains + 40 LDS lookups", agg, out, len, cus, iters);
    uint32_t* crc;
    CHECK(hipMalloc(&crc, (size_t)kPsns * 4));
    run_split<0>("split waves: 8 store + 8 read-only", agg, out, len, crc, cus, iters);
    run_split<200>("split waves: 8 store + 8 with 200 VALU in 4 chains", agg, out, len, crc, cus, iters);
    run_split<400>("split waves: 8 store + 8 with 400 VALU in 4 chains", agg, out, len, crc, cus, iters);
    CHECK(hipFree(crc));
    CHECK(hipFree(agg));
    CHECK(hipFree(out));
    CHECK(hipFree(len));
    return 0;
}
