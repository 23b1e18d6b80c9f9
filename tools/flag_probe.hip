// flag_probe.hip -- does a polling load see a flag another workgroup stored?
//
// Asked while the mesh engine's W = 4 one-GPU stalls were open (DESIGN.md "Mesh
// reduce-scatter route", liveness: they were not stale loads): a reader workgroup loads a
// flag word (system-scope load, as the mesh kernel polls), so that the word's
// line is warm; then it tells a writer workgroup to go; the writer waits a
// little and stores the next value (system-scope store, as the mesh kernel's
// flags); the reader polls with loads for up to `limit_us`.  A poll that never
// sees the value while a read-modify-write then does is a stale load.
//
//   flag_probe MEM TRIALS LIMIT_US DELAY_US [WRITER_BLOCK]
//     MEM: uncached | finegrained | coarse   (the mesh buffers are uncached)
//     WRITER_BLOCK: 1 (another XCD than block 0, by round-robin dispatch;
//                   the XCC ids are printed) or 8 (the same XCD)
//   flag_probe ipc-owner FILE TRIALS LIMIT_US DELAY_US   (reader; exports)
//   flag_probe ipc-peer  FILE TRIALS LIMIT_US DELAY_US   (writer; imports)
//     two processes on one GPU, as the mesh ranks of the one-GPU tests: the
//     reader polls its own allocation, the writer stores through its IPC
//     mapping of it.
//
// One line of JSON per run.  Test infrastructure, never linked into the
// library.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                              \
        }                                                                         \
    } while (0)

struct Res {
    uint32_t seen, stale, missing, xcc_r, xcc_w, done_r, done_w, pad;
    uint64_t max_ticks, sum_ticks;
};

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t rmw(uint32_t* p, uint32_t zero)
{
    return __hip_atomic_fetch_add(p, zero, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t xcc_id()
{
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xfu;
}

constexpr uint64_t kBound = 1000000000ull;   // 10 s of s_memrealtime: every wait ends

// flag at word 0, the reader's "go" word at word 64 (another 256-B line)
__device__ void reader(uint32_t* w, int trials, uint64_t limit, uint32_t zero, Res* r)
{
    uint32_t* flag = w;
    uint32_t* go = w + 64;
    uint32_t seen = 0, stale = 0, missing = 0;
    uint64_t mx = 0, sum = 0;
    r->xcc_r = xcc_id();
    for (int t = 1; t <= trials; ++t) {
        (void)ld_sys(flag);   // warm the line with the old value
        st_sys(go, (uint32_t)t);
        const uint64_t t0 = now();
        bool ok = false;
        uint64_t dt = 0;
        while ((dt = now() - t0) < limit) {
            if ((int32_t)(ld_sys(flag) - (uint32_t)t) >= 0) {
                ok = true;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (ok) {
            ++seen;
            sum += dt;
            if (dt > mx) mx = dt;
            continue;
        }
        // the loads gave up: did memory hold the value?
        if ((int32_t)(rmw(flag, zero) - (uint32_t)t) >= 0) ++stale;
        else ++missing;
        const uint64_t t1 = now();   // stay in step, for at most 10 s
        while ((int32_t)(rmw(flag, zero) - (uint32_t)t) < 0 && now() - t1 < kBound) __builtin_amdgcn_s_sleep(1);
        if (now() - t1 >= kBound) break;
    }
    r->seen = seen;
    r->stale = stale;
    r->missing = missing;
    r->max_ticks = mx;
    r->sum_ticks = sum;
    __hip_atomic_store(&r->done_r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ void writer(uint32_t* w, int trials, uint64_t delay, uint32_t zero, Res* r)
{
    uint32_t* flag = w;
    uint32_t* go = w + 64;
    r->xcc_w = xcc_id();
    for (int t = 1; t <= trials; ++t) {
        const uint64_t t1 = now();   // the reader's go, for at most 10 s
        while ((int32_t)(rmw(go, zero) - (uint32_t)t) < 0 && now() - t1 < kBound) __builtin_amdgcn_s_sleep(1);
        if (now() - t1 >= kBound) break;
        const uint64_t t0 = now();
        while (now() - t0 < delay) __builtin_amdgcn_s_sleep(1);
        st_sys(flag, (uint32_t)t);
    }
    __hip_atomic_store(&r->done_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_pair(uint32_t* w, int trials, uint64_t limit, uint64_t delay, int wb, uint32_t zero, Res* r)
{
    if (threadIdx.x != 0) return;
    if (blockIdx.x == 0) reader(w, trials, limit, zero, r);
    else if ((int)blockIdx.x == wb) writer(w, trials, delay, zero, r);
}

__global__ void k_reader(uint32_t* w, int trials, uint64_t limit, uint32_t zero, Res* r)
{
    if (threadIdx.x == 0 && blockIdx.x == 0) reader(w, trials, limit, zero, r);
}

__global__ void k_writer(uint32_t* w, int trials, uint64_t delay, uint32_t zero, Res* r)
{
    if (threadIdx.x == 0 && blockIdx.x == 0) writer(w, trials, delay, zero, r);
}

static void* alloc(const char* mem, size_t bytes)
{
    void* p = nullptr;
    if (!strcmp(mem, "coarse")) CHECK(hipMalloc(&p, bytes));
    else if (!strcmp(mem, "finegrained")) CHECK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained));
    else CHECK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached));
    CHECK(hipMemset(p, 0, bytes));
    CHECK(hipDeviceSynchronize());
    return p;
}

static void report(const char* what, const char* mem, int trials, double limit_us, double delay_us, int wb, const Res* r)
{
    const double tick_us = 0.01;   // s_memrealtime: 100 MHz
    printf("{\"run\": \"%s\", \"mem\": \"%s\", \"trials\": %d, \"limit_us\": %.0f, \"delay_us\": %.1f, "
           "\"writer_block\": %d, \"xcc_reader\": %u, \"xcc_writer\": %u, \"seen\": %u, \"stale\": %u, "
           "\"missing\": %u, \"mean_us\": %.2f, \"max_us\": %.2f}\n",
           what, mem, trials, limit_us, delay_us, wb, r->xcc_r, r->xcc_w, r->seen, r->stale, r->missing,
           r->seen ? (double)r->sum_ticks / r->seen * tick_us : 0.0, (double)r->max_ticks * tick_us);
    fflush(stdout);
}

int main(int argc, char** argv)
{
    if (argc < 5) {
        fprintf(stderr, "usage: see the header of tools/flag_probe.hip\n");
        return 2;
    }
    Res* r = nullptr;
    CHECK(hipHostMalloc((void**)&r, sizeof(Res), hipHostMallocMapped));
    memset(r, 0, sizeof(Res));
    Res* rd = nullptr;
    CHECK(hipHostGetDevicePointer((void**)&rd, r, 0));
    const uint32_t zero = (uint32_t)(argc > 100);   // 0, opaque to the compiler
    if (!strcmp(argv[1], "ipc-owner") || !strcmp(argv[1], "ipc-peer")) {
        if (argc < 6) return 2;
        const char* file = argv[2];
        const int trials = atoi(argv[3]);
        const double limit_us = atof(argv[4]), delay_us = atof(argv[5]);
        const bool owner = !strcmp(argv[1], "ipc-owner");
        uint32_t* w = nullptr;
        if (owner) {
            w = (uint32_t*)alloc("uncached", 1 << 16);
            hipIpcMemHandle_t h;
            CHECK(hipIpcGetMemHandle(&h, w));
            char tmp[512];
            snprintf(tmp, sizeof(tmp), "%s.tmp", file);
            FILE* f = fopen(tmp, "wb");
            if (!f || fwrite(&h, sizeof(h), 1, f) != 1) return 3;
            fclose(f);
            rename(tmp, file);
            k_reader<<<1, 64>>>(w, trials, (uint64_t)(limit_us * 100), zero, rd);
        } else {
            hipIpcMemHandle_t h;
            FILE* f = nullptr;
            for (int i = 0; i < 600 && !(f = fopen(file, "rb")); ++i) usleep(100000);
            if (!f || fread(&h, sizeof(h), 1, f) != 1) return 3;
            fclose(f);
            CHECK(hipIpcOpenMemHandle((void**)&w, h, hipIpcMemLazyEnablePeerAccess));
            k_writer<<<1, 64>>>(w, trials, (uint64_t)(delay_us * 100), zero, rd);
        }
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        if (owner) report("ipc", "uncached", trials, limit_us, delay_us, -1, r);
        if (!owner) CHECK(hipIpcCloseMemHandle(w));
        else {
            sleep(1);   // the peer closes its mapping first
            CHECK(hipFree(w));
        }
        return 0;
    }
    const char* mem = argv[1];
    const int trials = atoi(argv[2]);
    const double limit_us = atof(argv[3]), delay_us = atof(argv[4]);
    const int wb = argc > 5 ? atoi(argv[5]) : 1;
    if (wb < 1 || wb > 15) return 2;
    uint32_t* w = (uint32_t*)alloc(mem, 1 << 16);
    k_pair<<<16, 64>>>(w, trials, (uint64_t)(limit_us * 100), (uint64_t)(delay_us * 100), wb, zero, rd);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    report("pair", mem, trials, limit_us, delay_us, wb, r);
    CHECK(hipFree(w));
    return 0;
}
