// inccl_ll.hip -- the small-bucket ("ll", low-latency) allreduce: one kernel per
// call on every rank, no host synchronisation, no RCCL.
//
// The reference aggregates 1 KiB packets as they arrive (nts.c:303-501): every
// packet is added into a slot and the slot is released once FAN_IN have
// arrived.  This kernel is that switch, one level up: workgroup b of every rank
//   1. quantises + sums its R local buckets over its quads (4 elements) into the
//      rank's own data buffer (library memory, shared with the peers over HIP
//      IPC),
//   2. raises its arrival flag in every peer's signal array (system-scope
//      release store over xGMI: the `arrival_state` bit of nts.c:363),
//   3. waits until every peer's workgroup b has raised its flag for this call
//      (the FAN_IN check, nts.c:365), then
//   4. sums the W ranks' quads -- W-1 of them read over xGMI -- and
//      dequantises them into dst (the broadcast, nts.c:367-372, fused with the
//      new back stage).
// Each rank reads the whole bucket from every peer ("one shot"), which is the
// right trade while a call is latency-bound, i.e. for buckets up to ~1 MiB.
//
// Buffer reuse.  The data slots alternate by call parity.  A rank writes the
// parity-p slot in call e only after its call e-1 saw every peer's flag for
// call e-1, which those peers raise only after their call e-2 kernel (the last
// reader of the parity-p slot) completed: kernels of one rank are ordered on
// its stream (the host side adds an event wait when the caller switches
// streams).  Flags carry the call number (epoch), so they never need resetting.
// The epoch lives on the device (read by every workgroup at its start, advanced
// by the last one to retire), so a captured hipGraph replays correctly.
//
// Termination.  Every wait is bounded by a wall-clock timeout; a rank whose
// peers never arrive sets a host-visible error word and finishes the kernel,
// so a missing peer costs a reported error, never a hung GPU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "inccl_kernels.h"
#include "inccl_stream.h"

namespace {

using namespace inccl_dev;

constexpr int kLLBlock = 256;
constexpr int kLLDefaultCap = 64;

struct LLArgs {
    SrcPtrs src;                    // R local fp32 buckets
    float* dst;
    int64_t n;                      // elements
    uint32_t* own_data;             // own data slot 0 (slot 1 at + slot_elems)
    const uint32_t* peer_data[kMaxR];   // every rank's slot 0 ([me] = own_data)
    int64_t slot_elems;
    uint32_t* peer_sig[kMaxR];      // every rank's signal array ([me] unused)
    const uint32_t* own_sig;
    uint32_t* ctr;                  // [0] calls completed on this rank, [1] workgroups retired
    uint32_t* err;                  // host-mapped error word
    int W, me;
    uint64_t timeout_ticks;         // s_memrealtime ticks
    Scale sc;
    int64_t rs_lo4, rs_hi4;         // rs_hi4 > 0: reduce-scatter, dst = quads [rs_lo4, rs_hi4) of the result
};

__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

// System-scope (sc0 sc1) access: write-through on store, L1-bypassing and
// coherent on load -- the WT protocol's data path needs no L2 writeback or
// invalidate.  16-B accesses: a 4-B sc1 store costs ~6x a 16-B one per byte
// (MI355X_MICROARCH.md, store flavours).
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
constexpr int kAuxSys = 1 | 16;   // buffer instruction cache policy: sc0 | sc1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
// 16-B system-scope store through a (wave-uniform) buffer resource.  A builtin,
// not inline asm: the compiler's hazard recognizer must see the store, or it may
// overwrite the data VGPRs of a >64-bit store before the store has read them.
__device__ __forceinline__ void st_sys16(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, u32x4 v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)byte_off, 0, kAuxSys);
}

// WT = false: plain data accesses ordered by a system-scope release (buffer_wbl2)
//             on the flag store and an acquire (buffer_inv) after the wait.
// WT = true:  data written through and read around the caches (sc0 sc1), so the
//             flag store only has to follow the data stores' completion.
template <int R, bool WT>
__global__ __launch_bounds__(kLLBlock) void k_ll_oneshot(LLArgs a, int vec_src, int vec_dst)
{
    const int k = resolve_k(a.sc);
    const float scale = pow2f(k);
    const float inv = deq_scale(a.sc, k);
    const int64_t nq = (a.n + 3) >> 2;
    const int64_t stride = (int64_t)gridDim.x * kLLBlock;
    const int tid = threadIdx.x;
    // this call's number, kept on the device so that graph replays advance it too
    const uint32_t epoch = __hip_atomic_load(a.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    const int64_t slot = (int64_t)(epoch & 1u) * a.slot_elems;

    // 1. quantise + local sum into the own data slot (padding lanes are 0)
    u32x4* own = reinterpret_cast<u32x4*>(a.own_data + slot);
    const __amdgpu_buffer_rsrc_t own_rs = rsrc(a.own_data + slot, (uint32_t)(nq * 16));
    for (int64_t q = (int64_t)blockIdx.x * kLLBlock + tid; q < nq; q += stride) {
        u32x4 acc = {0u, 0u, 0u, 0u};
        if (vec_src && 4 * q + 4 <= a.n) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const u32x4 x = reinterpret_cast<const u32x4*>(a.src.p[r])[q];
                acc.x += quant1(__uint_as_float(x.x), scale);
                acc.y += quant1(__uint_as_float(x.y), scale);
                acc.z += quant1(__uint_as_float(x.z), scale);
                acc.w += quant1(__uint_as_float(x.w), scale);
            }
        } else {
            uint32_t s[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t i = 4 * q + e;
                if (i < a.n)
#pragma unroll
                    for (int r = 0; r < R; ++r) s[e] += quant1(reinterpret_cast<const float*>(a.src.p[r])[i], scale);
            }
            acc.x = s[0];
            acc.y = s[1];
            acc.z = s[2];
            acc.w = s[3];
        }
        if constexpr (WT) {
            st_sys16(own_rs, (uint32_t)(q * 16), acc);
        } else {
            own[q] = acc;
        }
    }
    if constexpr (WT) __builtin_amdgcn_s_waitcnt(0);   // own stores acknowledged at system scope
    __syncthreads();   // every lane's stores issued and complete at workgroup scope

    // 2. arrival flag into every peer (release at system scope: L2 written back first)
    const int flag = a.me * INCCL_LL_MAX_BLOCKS + blockIdx.x;
    if (tid < a.W && tid != a.me) {
        if constexpr (WT) st_sys(a.peer_sig[tid] + flag, epoch);
        else __hip_atomic_store(a.peer_sig[tid] + flag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }

    // 3. wait for every peer's workgroup blockIdx.x (bounded)
    if (tid < a.W && tid != a.me) {
        const uint32_t* s = a.own_sig + tid * INCCL_LL_MAX_BLOCKS + blockIdx.x;
        const uint64_t t0 = now_ticks();
        while ((int32_t)(__hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
            if (now_ticks() - t0 > a.timeout_ticks) {
                __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if constexpr (!WT) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // system scope: invalidates stale lines
    }
    __syncthreads();
    if constexpr (!WT) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // every wave, before reading peer memory

    // 4. sum the W ranks' quads, dequantise into dst: all W loads of up to kU
    //    quads in flight before the first add.  Reduce-scatter: only the quads
    //    of this rank's shard, written from dst[0]
    constexpr int kU = 4;
    const bool rs = a.rs_hi4 > 0;
    const int64_t qlo = rs ? a.rs_lo4 : 0, qhi = rs ? a.rs_hi4 : nq;
    const int64_t out_n = rs ? 4 * (qhi - qlo) : a.n;
    __amdgpu_buffer_rsrc_t peer[kMaxR];
    if constexpr (WT) {
#pragma unroll
        for (int j = 0; j < kMaxR; ++j)
            if (j < a.W) peer[j] = rsrc(a.peer_data[j] + slot, (uint32_t)(nq * 16));
    }
    const __amdgpu_buffer_rsrc_t dst_rs = rsrc(a.dst, (uint32_t)(out_n * 4));
    for (int64_t q0 = (int64_t)blockIdx.x * kLLBlock + tid; q0 < nq; q0 += stride * kU) {
        u32x4 x[kU][kMaxR];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t q = q0 + u * stride;
#pragma unroll
            for (int j = 0; j < kMaxR; ++j) {
                if (j < a.W && q >= qlo && q < qhi) {
                    if constexpr (WT) x[u][j] = __builtin_amdgcn_raw_buffer_load_b128(peer[j], (int)(q * 16), 0, kAuxSys);
                    else x[u][j] = reinterpret_cast<const u32x4*>(a.peer_data[j] + slot)[q];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t q = q0 + u * stride;
            if (q >= nq) break;
            if (q < qlo || q >= qhi) continue;
            const int64_t qo = q - qlo;   // the output quad
            u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int j = 0; j < kMaxR; ++j)
                if (j < a.W) {
                    acc.x += x[u][j].x;
                    acc.y += x[u][j].y;
                    acc.z += x[u][j].z;
                    acc.w += x[u][j].w;
                }
            u32x4 o;
            o.x = __float_as_uint((float)(int32_t)acc.x * inv);
            o.y = __float_as_uint((float)(int32_t)acc.y * inv);
            o.z = __float_as_uint((float)(int32_t)acc.z * inv);
            o.w = __float_as_uint((float)(int32_t)acc.w * inv);
            if (vec_dst && 4 * qo + 4 <= out_n) {
                // write-through (sc1): nothing of dst stays dirty in this XCD's L2
                __builtin_amdgcn_raw_buffer_store_b128(o, dst_rs, (int)(qo * 16), 0, 16);
            } else {
                const uint32_t v[4] = {o.x, o.y, o.z, o.w};
                for (int e = 0; e < 4; ++e)
                    if (4 * qo + e < out_n) reinterpret_cast<uint32_t*>(a.dst)[4 * qo + e] = v[e];
            }
        }
    }

    // 5. retire: the last workgroup advances the call counter for the next call
    //    (every workgroup read it at its start, before retiring)
    if (tid == 0) {
        // relaxed: only atomicity matters, the next kernel is ordered by the kernel boundary
        const uint32_t done = __hip_atomic_fetch_add(a.ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done == gridDim.x - 1) {
            __hip_atomic_store(a.ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.ctr, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <int R>
hipError_t launch_R(const LLArgs& a, int grid, int vs, int vd, hipStream_t st)
{
    static int wt = -1;   // $INCCL_LL_PROTOCOL: "wt" (default) or "fence"; same on every rank
    if (wt < 0) {
        const char* e = getenv("INCCL_LL_PROTOCOL");
        wt = (e && e[0] == 'f') ? 0 : 1;
    }
    if (wt) hipLaunchKernelGGL((k_ll_oneshot<R, true>), dim3(grid), dim3(kLLBlock), 0, st, a, vs, vd);
    else hipLaunchKernelGGL((k_ll_oneshot<R, false>), dim3(grid), dim3(kLLBlock), 0, st, a, vs, vd);
    return hipGetLastError();
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace

// Workgroups per call: one per 256 quads up to a cap ($INCCL_LL_GRID_CAP, which
// must be the same on every rank).  Default 64: the cap sweep with two ranks
// on one MI355X (profiles/r01_ll_grid_cap_sweep.jsonl) gave 19 us per 1 MiB call
// at 32-64 workgroups vs 34 us at 256 -- every workgroup pays a system-scope
// release (L2 writeback) and polls its own flags.
extern "C" int inccl_k_ll_grid(size_t n)
{
    static int cap = -1;
    if (cap < 0) {
        const char* e = getenv("INCCL_LL_GRID_CAP");
        const int v = e ? atoi(e) : 0;
        cap = (v >= 1 && v <= INCCL_LL_MAX_BLOCKS) ? v : kLLDefaultCap;
    }
    const int64_t nq = ((int64_t)n + 3) >> 2;
    int64_t g = (nq + kLLBlock - 1) / kLLBlock;
    if (g > cap) g = cap;
    return g < 1 ? 1 : (int)g;
}

extern "C" int inccl_k_ll_oneshot(const struct inccl_ll_launch* l, void* stream)
{
    if (!l || l->R < 1 || l->R > kMaxR || l->W < 2 || l->W > kMaxR || l->me < 0 || l->me >= l->W ||
        (l->rs_n && ((l->rs_lo | l->rs_n) & 3u || l->rs_lo + l->rs_n > l->n)))
        return INCCL_ERR_ARG;
    LLArgs a{};
    for (int r = 0; r < l->R; ++r) a.src.p[r] = l->src[r];
    a.dst = l->dst;
    a.n = (int64_t)l->n;
    a.own_data = l->own_data;
    a.slot_elems = (int64_t)l->slot_elems;
    for (int j = 0; j < l->W; ++j) {
        a.peer_data[j] = l->peer_data[j];
        a.peer_sig[j] = l->peer_sig[j];
    }
    a.own_sig = l->own_sig;
    a.ctr = l->ctr;
    a.err = l->err;
    a.W = l->W;
    a.me = l->me;
    a.timeout_ticks = l->timeout_ticks;
    a.sc.k = l->scale_exp;
    a.sc.amax_bits = l->amax_bits;
    a.sc.scale_R = l->scale_R;
    a.sc.out_shift = l->out_shift;
    a.rs_lo4 = (int64_t)(l->rs_lo >> 2);
    a.rs_hi4 = l->rs_n ? (int64_t)((l->rs_lo + l->rs_n) >> 2) : 0;
    int vs = 1;
    for (int r = 0; r < l->R; ++r) vs &= aligned16(l->src[r]) ? 1 : 0;
    const int vd = aligned16(l->dst) ? 1 : 0;
    const int grid = inccl_k_ll_grid(l->n);
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    switch (l->R) {
        case 1: e = launch_R<1>(a, grid, vs, vd, st); break;
        case 2: e = launch_R<2>(a, grid, vs, vd, st); break;
        case 3: e = launch_R<3>(a, grid, vs, vd, st); break;
        case 4: e = launch_R<4>(a, grid, vs, vd, st); break;
        case 5: e = launch_R<5>(a, grid, vs, vd, st); break;
        case 6: e = launch_R<6>(a, grid, vs, vd, st); break;
        case 7: e = launch_R<7>(a, grid, vs, vd, st); break;
        default: e = launch_R<8>(a, grid, vs, vd, st); break;
    }
    return e == hipSuccess ? 0 : (int)e;
}
