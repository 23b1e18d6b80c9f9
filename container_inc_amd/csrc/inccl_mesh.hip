// inccl_mesh.hip -- the "mesh" engine: a whole large-bucket allreduce as ONE
// persistent kernel per rank, with no host synchronisation and no RCCL.
//
// Every GPU is the aggregation switch for its own shard of the bucket
// (non_termination_switch.c:303-501 keeps one switch per tree; on a fully
// connected xGMI mesh every rank can be one).  A shard is cut into chunks, and
// one call is three kinds of work item per chunk c:
//
//   push(c, j)   quantise + sum the R local buckets over chunk c of shard j and
//                write the int32 partial straight into rank j's inbox over xGMI
//                (the host's encode + RDMA WRITE of api.c:293-327), then raise
//                arrive[me][c] in rank j's signal array;
//   reduce(c)    wait until every rank's partial of chunk c of MY shard has
//                arrived (the switch's arrival bitmap, nts.c:361-365), sum the W
//                partials from local HBM, dequantise into my result shard, and
//                raise ready[me][c] in every rank's signal array (the broadcast,
//                nts.c:447-453);
//   gather(c, j) wait for ready[j][c], then pull rank j's result chunk over xGMI
//                into dst (the host's decode, api.c:428-430).
//
// "meshw" (push_res): reduce(c) also writes the result chunk into slot `me` of
// every rank's result inbox before raising ready, and gather(c, j) copies it
// from the local inbox -- every xGMI transfer of the call is then a write.  The
// inbox reuse argument below holds for the result inbox as it does for the
// partial inbox (rank j rewrites my slot j of chunk c only after my next
// push(c, j), i.e. after my previous call, gathers included, has finished).
//
// Scheduling.  Items are numbered in one global order that every rank shares:
// slot s holds push(s, *), reduce(s - lag) and gather(s - 2 lag, *).  Workgroups
// take tickets from a device counter, so items start in that order on every
// rank, and every item waits only for items of strictly earlier tickets on
// other ranks.  Hence the earliest unfinished item anywhere never waits, and
// the call always completes, whatever the grid size and residency (ranks on
// separate GPUs; ranks sharing one GPU are sized so their grids co-reside).
// A waiting workgroup holds its CU slot idle, so the host picks `lag` large
// (default: the whole shard -- every push is taken before the first reduce);
// the phases still overlap at their seams, quantisation overlaps the pushes'
// xGMI writes, and both link directions are busy while pushing and gathering.
//
// Coherence.  Data crossing GPUs is written with system-scope 16-B stores
// (`buffer_store_dwordx4 ... sc0 sc1`, write-through) and read with
// system-scope 16-B buffer loads (`sc0 sc1`), so neither side needs an L2
// writeback or invalidate; a flag is stored only after the workgroup's data
// stores are acknowledged (s_waitcnt + barrier).  Flags carry the call number
// (a device-resident counter, so a captured hipGraph replays correctly) and
// never need resetting.
//
// Buffer reuse without double buffering: rank j pushes call e+1's partial of
// chunk c into my inbox only after its call e finished, including its gather of
// my result chunk c, which I raised only after reading that inbox chunk.
// dst may alias srcs[0]: gather(c, j) waits for ready[j][c], which follows my
// own push(c, j) -- the last reader of that source range.
//
// Termination.  Every wait is bounded by a wall-clock timeout; on expiry the
// kernel sets a host-mapped error word and a local abort word, and every
// workgroup leaves its loop: a missing peer costs a reported error, never a
// hung GPU.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "inccl_kernels.h"
#include "inccl_stream.h"

namespace {

using namespace inccl_dev;

constexpr int kMeshBlock = 256;
constexpr int kMeshU = 4;   // quads per lane per pass (all loads in flight before the first add)
constexpr int kAuxSys = 1 | 16;   // buffer instruction cache policy: sc0 | sc1

struct MeshArgs {
    SrcPtrs src;
    float* dst;
    int64_t n;
    int64_t shard;                       // elements per rank's shard (multiple of 64)
    int64_t chunk;                       // elements per chunk (multiple of 64)
    int64_t inbox_stride;                // elements per source slot of an inbox
    uint32_t* peer_inbox[kMaxR];         // rank j's inbox; my slot at + me * inbox_stride
    const uint32_t* own_inbox;
    uint32_t* own_res;
    const uint32_t* peer_res[kMaxR];
    uint32_t* peer_resin[kMaxR];         // rank j's result inbox (push_res): slot i at + i * inbox_stride
    const uint32_t* own_resin;
    uint32_t* peer_sig[kMaxR];           // rank j's signal array ([me] = own)
    const uint32_t* own_sig;
    uint32_t* ctr;                       // [0] calls done, [1] retired, [2] ticket, [3] abort, [4] started,
                                         // [8 + j] pushes to rank j finished; 64-bit at [32]: call start,
                                         // [34 + 2 j]: last push flag store to rank j (s_memrealtime)
                                         // (this call)
    uint32_t* err;                       // host-mapped error words (16)
    uint64_t timeout_ticks;
    int nchunks, W, me, lag, vec_src, vec_dst, push_res;
    int rs;                              // reduce-scatter: gather(c, me) copies my result chunk into dst (the
                                         // shard), the other gathers only wait
    Scale sc;
    uint64_t src_bytes, dst_bytes, inbox_bytes, res_bytes, resin_bytes;   // region sizes (bounds check)
    uint32_t zero;                       // 0, opaque to the compiler (which turns an idempotent RMW into a load)
};

__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
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

__device__ __forceinline__ int arrive_idx(int j, int c) { return j * INCCL_MESH_MAX_CHUNKS + c; }
__device__ __forceinline__ int ready_idx(int j, int c) { return (kMaxR + j) * INCCL_MESH_MAX_CHUNKS + c; }

// Bounded wait for *f >= epoch (serial-number order).  false: timed out or aborted.
// A timeout reports which wait expired: err[0] = INCCL_MESH_ERR_TIMEOUT | item << 8
// | peer << 4 | chunk << 16 (item 3: a reduce's arrival flag, 6: a gather's ready
// flag), err[1] = the flag's last value, err[2] = the epoch waited for, err[3] =
// the tickets this rank's workgroups had taken, err[4] / err[5] = its workgroups
// started / retired, err[6 + j] = its pushes to rank j finished, err[13] = the
// call's chunks, err[14] = the flag re-read by a read-modify-write, err[15] /
// err[16] / err[17 + j] = the clock (/16) at the timeout, at the call's start,
// at the last push flag store to rank j.  (DESIGN.md "Mesh reduce-scatter
// route", liveness: what these told apart.)
__device__ bool wait_flag(const MeshArgs& a, const uint32_t* f, uint32_t epoch, uint32_t item, int peer, int c)
{
    const uint64_t t0 = now_ticks();
    uint32_t v;
    while ((int32_t)((v = ld_sys(f)) - epoch) < 0) {
        if (__hip_atomic_load(a.ctr + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
        if (now_ticks() - t0 > a.timeout_ticks) {
            __hip_atomic_store(a.err + 1, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(a.err + 2, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(a.err + 3, __hip_atomic_load(a.ctr + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);   // tickets taken so far
            // the rank's own progress: workgroups started and retired, pushes
            // finished per destination; and the flag re-read by a system-scope
            // read-modify-write (performed at the coherence point, never a
            // cached copy)
            __hip_atomic_store(a.err + 4, __hip_atomic_load(a.ctr + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(a.err + 5, __hip_atomic_load(a.ctr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            for (int j = 0; j < a.W; ++j)
                __hip_atomic_store(a.err + 6 + j, __hip_atomic_load(a.ctr + 8 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(a.err + 13, (uint32_t)a.nchunks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            // clock readings (s_memrealtime / 16, one GPU-wide 100 MHz clock):
            // this timeout, this call's first workgroup start, and the last
            // flag store of this rank's pushes to each rank
            const uint64_t* t64 = reinterpret_cast<const uint64_t*>(a.ctr + 32);
            __hip_atomic_store(a.err + 15, (uint32_t)(now_ticks() >> 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(a.err + 16,
                               (uint32_t)(__hip_atomic_load(t64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 4),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            for (int j = 0; j < a.W; ++j)
                __hip_atomic_store(a.err + 17 + j,
                                   (uint32_t)(__hip_atomic_load(t64 + 1 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 4),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(a.err + 14,
                               __hip_atomic_fetch_add(const_cast<uint32_t*>(f), a.zero, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_SYSTEM),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(a.err, INCCL_MESH_ERR_TIMEOUT | item << 8 | (uint32_t)peer << 4 | (uint32_t)c << 16,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(a.ctr + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return true;
}

// Per-item bounds check (wave-uniform, a few scalar instructions per item): the
// byte range [p, p + bytes) an item is about to build a buffer resource over, or
// read through plain loads, must lie inside its region [base, base + size).
// Otherwise the item reports where (*err = INCCL_MESH_ERR_BOUNDS | item << 8 |
// peer << 4, the first report wins) and the call aborts without the access --
// the evidence a fault would have destroyed (DESIGN.md "Mesh reduce-scatter
// route"; a later report may overwrite an earlier one).  item: 1 push src, 2 push inbox, 3 reduce inbox, 4 reduce res,
// 5 reduce resin, 6 gather src, 7 gather dst.
__device__ bool inside(const MeshArgs& a, const void* base, uint64_t size, const void* p, uint64_t bytes,
                       uint32_t item, int peer)
{
    const uint64_t b = reinterpret_cast<uint64_t>(base), q = reinterpret_cast<uint64_t>(p);
    if (base != nullptr && q >= b && bytes <= size && q - b <= size - bytes) return true;
    if (threadIdx.x == 0) {
        __hip_atomic_store(a.err, INCCL_MESH_ERR_BOUNDS | item << 8 | (uint32_t)peer << 4, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(a.ctr + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return false;
}

__device__ __forceinline__ int64_t chunk_len(const MeshArgs& a, int c)
{
    const int64_t rest = a.shard - (int64_t)c * a.chunk;
    return rest < a.chunk ? rest : a.chunk;
}

// push(c, j): partial sums of chunk c of shard j -> rank j's inbox, slot me.
// E = BF16 / F16: the sources are 2-byte (8 bytes per quad of elements); E = 0:
// fp32.  The partials are int32 either way.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int R, int E>
__device__ bool do_push(const MeshArgs& a, int c, int j, uint32_t epoch, float scale)
{
    const int64_t lo = (int64_t)j * a.shard + (int64_t)c * a.chunk;   // global element index
    const int64_t nq = chunk_len(a, c) >> 2;
    constexpr int SE = is16(E) ? 2 : 4;   // source element bytes
    if (lo < a.n) {
        const int64_t cnt = a.n - lo < 4 * nq ? a.n - lo : 4 * nq;
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (!inside(a, a.src.p[r], a.src_bytes, reinterpret_cast<const char*>(a.src.p[r]) + lo * SE,
                        (uint64_t)cnt * SE, 1, r))
                return false;
    }
    uint32_t* obase = a.peer_inbox[j] + (int64_t)a.me * a.inbox_stride + (int64_t)c * a.chunk;
    if (!inside(a, a.peer_inbox[j], a.inbox_bytes, obase, (uint64_t)nq * 16, 2, j)) return false;
    const __amdgpu_buffer_rsrc_t out = rsrc(obase, (uint32_t)(nq * 16));
    const bool full = a.vec_src && lo + 4 * nq <= a.n;
    for (int64_t q0 = threadIdx.x; q0 < nq; q0 += (int64_t)kMeshBlock * kMeshU) {
        u32x4 acc[kMeshU];
        if (full && is16(E)) {
            u32x2 x[kMeshU][R];
#pragma unroll
            for (int u = 0; u < kMeshU; ++u) {
                const int64_t q = q0 + (int64_t)u * kMeshBlock;
#pragma unroll
                for (int r = 0; r < R; ++r)
                    x[u][r] = q < nq ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(a.src.p[r]) + (lo >> 2) + q)
                                     : u32x2{0u, 0u};
            }
#pragma unroll
            for (int u = 0; u < kMeshU; ++u) {
                acc[u] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    acc[u].x += quant16<E>(x[u][r].x & 0xffffu, scale);
                    acc[u].y += quant16<E>(x[u][r].x >> 16, scale);
                    acc[u].z += quant16<E>(x[u][r].y & 0xffffu, scale);
                    acc[u].w += quant16<E>(x[u][r].y >> 16, scale);
                }
            }
        } else if (full) {
            u32x4 x[kMeshU][R];
#pragma unroll
            for (int u = 0; u < kMeshU; ++u) {
                const int64_t q = q0 + (int64_t)u * kMeshBlock;
#pragma unroll
                for (int r = 0; r < R; ++r)
                    x[u][r] = q < nq ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.src.p[r]) + (lo >> 2) + q)
                                     : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int u = 0; u < kMeshU; ++u) {
                acc[u] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    acc[u].x += quant1(__uint_as_float(x[u][r].x), scale);
                    acc[u].y += quant1(__uint_as_float(x[u][r].y), scale);
                    acc[u].z += quant1(__uint_as_float(x[u][r].z), scale);
                    acc[u].w += quant1(__uint_as_float(x[u][r].w), scale);
                }
            }
        } else {   // ragged end of the bucket / unaligned sources: element-granular, zero past n
#pragma unroll
            for (int u = 0; u < kMeshU; ++u) {
                const int64_t q = q0 + (int64_t)u * kMeshBlock;
                uint32_t s[4] = {0u, 0u, 0u, 0u};
                if (q < nq)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int64_t i = lo + 4 * q + e;
                        if (i < a.n)
#pragma unroll
                            for (int r = 0; r < R; ++r)
                                s[e] += is16(E) ? quant16<E>(reinterpret_cast<const uint16_t*>(a.src.p[r])[i], scale)
                                                : quant1(reinterpret_cast<const float*>(a.src.p[r])[i], scale);
                    }
                acc[u] = u32x4{s[0], s[1], s[2], s[3]};
            }
        }
#pragma unroll
        for (int u = 0; u < kMeshU; ++u) {
            const int64_t q = q0 + (int64_t)u * kMeshBlock;
            if (q < nq) st_sys16(out, (uint32_t)(q * 16), acc[u]);
        }
    }
    __builtin_amdgcn_s_waitcnt(0);   // this lane's stores acknowledged at system scope
    __syncthreads();                 // ... and every lane's
    if (threadIdx.x == 0) {
        st_sys(a.peer_sig[j] + arrive_idx(a.me, c), epoch);
        __hip_atomic_fetch_add(a.ctr + 8 + j, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // progress record
        __hip_atomic_fetch_max(reinterpret_cast<uint64_t*>(a.ctr + 32) + 1 + j, now_ticks(), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    return true;
}

// reduce(c): my shard's chunk c = dequant(sum over the W inbox slots); E = BF16 /
// F16: the result chunk is 2-byte (8 bytes per quad), at element offsets in
// 2-byte units
template <int E>
__device__ bool do_reduce(const MeshArgs& a, int c, uint32_t epoch, float inv)
{
    bool ok = true;
    if (threadIdx.x < a.W) ok = wait_flag(a, a.own_sig + arrive_idx(threadIdx.x, c), epoch, 3, threadIdx.x, c);
    if (!__syncthreads_and(ok)) return false;
    const int64_t nq = chunk_len(a, c) >> 2;
    const uint32_t bytes = (uint32_t)(nq * 16);
    for (int j = 0; j < a.W; ++j)
        if (!inside(a, a.own_inbox, a.inbox_bytes, a.own_inbox + (int64_t)j * a.inbox_stride + (int64_t)c * a.chunk,
                    bytes, 3, j))
            return false;
    __amdgpu_buffer_rsrc_t in[kMaxR];
#pragma unroll
    for (int j = 0; j < kMaxR; ++j)
        in[j] = rsrc(a.own_inbox + (int64_t)(j < a.W ? j : 0) * a.inbox_stride + (int64_t)c * a.chunk, bytes);
    constexpr int ES = is16(E) ? 2 : 4;   // result element bytes
    const uint32_t obytes = (uint32_t)(nq * 4 * ES);
    const bool push = a.push_res && !a.rs;
    // my result chunk, in every mode but meshw's allreduce the same store into
    // own_res (IPC memory); reduce-scatter copies it into dst in gather(c, me)
    const char* rbase = reinterpret_cast<const char*>(a.own_res) + (int64_t)c * a.chunk * ES;
    if (!push && !inside(a, a.own_res, a.res_bytes, rbase, obytes, 4, a.me)) return false;
    const __amdgpu_buffer_rsrc_t res = rsrc(rbase, obytes);
    __amdgpu_buffer_rsrc_t outs[kMaxR];   // push_res: my slot of every rank's result inbox
    if (push) {
        for (int j = 0; j < a.W; ++j)
            if (!inside(a, a.peer_resin[j], a.resin_bytes,
                        reinterpret_cast<const char*>(a.peer_resin[j]) +
                            ((int64_t)a.me * a.inbox_stride + (int64_t)c * a.chunk) * ES,
                        obytes, 5, j))
                return false;
#pragma unroll
        for (int j = 0; j < kMaxR; ++j)
            outs[j] = rsrc(reinterpret_cast<const char*>(a.peer_resin[j < a.W ? j : 0]) +
                               ((int64_t)a.me * a.inbox_stride + (int64_t)c * a.chunk) * ES,
                           obytes);
    }
    for (int64_t q0 = threadIdx.x; q0 < nq; q0 += (int64_t)kMeshBlock * 2) {
        u32x4 x[2][kMaxR];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int j = 0; j < kMaxR; ++j)   // out-of-range lanes read 0 (buffer range check)
                x[u][j] = j < a.W ? __builtin_amdgcn_raw_buffer_load_b128(in[j], (int)((q0 + u * kMeshBlock) * 16), 0, kAuxSys)
                                  : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int64_t q = q0 + (int64_t)u * kMeshBlock;
            if (q >= nq) break;
            u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int j = 0; j < kMaxR; ++j) {
                acc.x += x[u][j].x;
                acc.y += x[u][j].y;
                acc.z += x[u][j].z;
                acc.w += x[u][j].w;
            }
            if constexpr (is16(E)) {
                const u32x2 o = {deq16x2<E>(acc.x, acc.y, inv), deq16x2<E>(acc.z, acc.w, inv)};
                if (push) {
#pragma unroll
                    for (int j = 0; j < kMaxR; ++j)
                        if (j < a.W) __builtin_amdgcn_raw_buffer_store_b64(o, outs[j], (int)(q * 8), 0, kAuxSys);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b64(o, res, (int)(q * 8), 0, kAuxSys);
                }
            } else {
                u32x4 o;
                o.x = __float_as_uint((float)(int32_t)acc.x * inv);
                o.y = __float_as_uint((float)(int32_t)acc.y * inv);
                o.z = __float_as_uint((float)(int32_t)acc.z * inv);
                o.w = __float_as_uint((float)(int32_t)acc.w * inv);
                if (push) {
#pragma unroll
                    for (int j = 0; j < kMaxR; ++j)
                        if (j < a.W) st_sys16(outs[j], (uint32_t)(q * 16), o);
                } else {
                    st_sys16(res, (uint32_t)(q * 16), o);
                }
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x < a.W) st_sys(a.peer_sig[threadIdx.x] + ready_idx(a.me, c), epoch);
    return true;
}

// gather(c, j): rank j's result chunk c -> dst (clipped to n).
// Reduce-scatter: gather(c, me) copies my own result chunk into my shard (the
// pull path with j = me, as in the allreduce); gather(c, j != me) is the wait
// alone -- the call then ends only after every rank has reduced every chunk,
// i.e. read its inbox, which is what lets the next call push into it.  So a
// reduce-scatter issues no instruction the allreduce does not (DESIGN.md,
// "Mesh reduce-scatter route").
__device__ bool do_gather(const MeshArgs& a, int c, int j, uint32_t epoch)
{
    bool ok = true;
    if (threadIdx.x == 0) ok = wait_flag(a, a.own_sig + ready_idx(j, c), epoch, 6, j, c);
    if (!__syncthreads_and(ok)) return false;
    if (a.rs && j != a.me) return true;
    const int64_t lo = (int64_t)j * a.shard + (int64_t)c * a.chunk;
    if (lo >= a.n) return true;
    int64_t cnt = chunk_len(a, c);
    if (lo + cnt > a.n) cnt = a.n - lo;
    const int64_t nq = cnt >> 2;
    // pull rank j's result chunk over xGMI, or (push_res) copy what rank j pushed
    // into my result inbox; reduce-scatter: my own result chunk
    const bool inbox = a.push_res && !a.rs;
    const uint32_t* sbase = inbox ? a.own_resin + (int64_t)j * a.inbox_stride + (int64_t)c * a.chunk
                                  : a.peer_res[j] + (int64_t)c * a.chunk;
    if (!inside(a, inbox ? a.own_resin : a.peer_res[j], inbox ? a.resin_bytes : a.res_bytes, sbase,
                (uint64_t)chunk_len(a, c) * 4, 6, j))
        return false;
    const __amdgpu_buffer_rsrc_t src = rsrc(sbase, (uint32_t)(chunk_len(a, c) * 4));
    uint32_t* d = reinterpret_cast<uint32_t*>(a.dst) + (a.rs ? (int64_t)c * a.chunk : lo);
    if (!inside(a, a.dst, a.dst_bytes, d, (uint64_t)cnt * 4, 7, j)) return false;
    const __amdgpu_buffer_rsrc_t drs = rsrc(d, (uint32_t)(nq * 16));   // write-through dst stores (vec_dst)
    for (int64_t q0 = threadIdx.x; q0 < nq; q0 += (int64_t)kMeshBlock * kMeshU) {
        u32x4 v[kMeshU];
#pragma unroll
        for (int u = 0; u < kMeshU; ++u)
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(src, (int)((q0 + u * kMeshBlock) * 16), 0, kAuxSys);
#pragma unroll
        for (int u = 0; u < kMeshU; ++u) {
            const int64_t q = q0 + (int64_t)u * kMeshBlock;
            if (q < nq) {
                if (a.vec_dst) {
                    __builtin_amdgcn_raw_buffer_store_b128(v[u], drs, (int)(q * 16), 0, 16);   // sc1
                } else {
                    d[4 * q] = v[u].x;
                    d[4 * q + 1] = v[u].y;
                    d[4 * q + 2] = v[u].z;
                    d[4 * q + 3] = v[u].w;
                }
            }
        }
    }
    for (int64_t i = 4 * nq + threadIdx.x; i < cnt; i += kMeshBlock)   // ragged end of the bucket
        d[i] = __builtin_amdgcn_raw_buffer_load_b32(src, (int)(i * 4), 0, kAuxSys);
    return true;
}

// gather(c, j) of a 2-byte result: 8 elements per 16-B access, a ragged end of
// the bucket element by element
__device__ bool do_gather16(const MeshArgs& a, int c, int j, uint32_t epoch)
{
    bool ok = true;
    if (threadIdx.x == 0) ok = wait_flag(a, a.own_sig + ready_idx(j, c), epoch, 6, j, c);
    if (!__syncthreads_and(ok)) return false;
    if (a.rs && j != a.me) return true;   // reduce-scatter: as do_gather
    const int64_t lo = (int64_t)j * a.shard + (int64_t)c * a.chunk;
    if (lo >= a.n) return true;
    int64_t cnt = chunk_len(a, c);
    if (lo + cnt > a.n) cnt = a.n - lo;
    const int64_t n8 = cnt >> 3;
    const bool inbox = a.push_res && !a.rs;
    const uint16_t* sbase = inbox
                                ? reinterpret_cast<const uint16_t*>(a.own_resin) + (int64_t)j * a.inbox_stride + (int64_t)c * a.chunk
                                : reinterpret_cast<const uint16_t*>(a.peer_res[j]) + (int64_t)c * a.chunk;
    if (!inside(a, inbox ? a.own_resin : a.peer_res[j], inbox ? a.resin_bytes : a.res_bytes, sbase,
                (uint64_t)chunk_len(a, c) * 2, 6, j))
        return false;
    const __amdgpu_buffer_rsrc_t src = rsrc(sbase, (uint32_t)(chunk_len(a, c) * 2));
    uint16_t* d = reinterpret_cast<uint16_t*>(a.dst) + (a.rs ? (int64_t)c * a.chunk : lo);
    if (!inside(a, a.dst, a.dst_bytes, d, (uint64_t)cnt * 2, 7, j)) return false;
    const __amdgpu_buffer_rsrc_t drs = rsrc(d, (uint32_t)(n8 * 16));
    for (int64_t q0 = threadIdx.x; q0 < n8; q0 += (int64_t)kMeshBlock * kMeshU) {
        u32x4 v[kMeshU];
#pragma unroll
        for (int u = 0; u < kMeshU; ++u)
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(src, (int)((q0 + u * kMeshBlock) * 16), 0, kAuxSys);
#pragma unroll
        for (int u = 0; u < kMeshU; ++u) {
            const int64_t q = q0 + (int64_t)u * kMeshBlock;
            if (q < n8) {
                if (a.vec_dst) {
                    __builtin_amdgcn_raw_buffer_store_b128(v[u], drs, (int)(q * 16), 0, 16);   // sc1
                } else {
                    const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        d[8 * q + 2 * e] = (uint16_t)(w[e] & 0xffffu);
                        d[8 * q + 2 * e + 1] = (uint16_t)(w[e] >> 16);
                    }
                }
            }
        }
    }
    for (int64_t i = 8 * n8 + threadIdx.x; i < cnt; i += kMeshBlock)   // ragged end of the bucket
        d[i] = (uint16_t)__builtin_amdgcn_raw_buffer_load_b16(src, (int)(i * 2), 0, kAuxSys);
    return true;
}

template <int R, int E>
__global__ __launch_bounds__(kMeshBlock) void k_mesh(MeshArgs a)
{
    __shared__ int s_ticket;
    const int k = resolve_k(a.sc);
    const float scale = pow2f(k);
    const float inv = deq_scale(a.sc, k);
    // this call's number, kept on the device so that graph replays advance it too
    const uint32_t epoch = __hip_atomic_load(a.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    const int W = a.W;
    const int per_slot = 2 * W + 1;
    const int total = (a.nchunks + 2 * a.lag) * per_slot;
    if (threadIdx.x == 0 && __hip_atomic_fetch_add(a.ctr + 4, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
        __hip_atomic_store(reinterpret_cast<uint64_t*>(a.ctr + 32), now_ticks(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);   // this call's start (the first workgroup's)
    for (;;) {
        if (threadIdx.x == 0)
            s_ticket = (int)__hip_atomic_fetch_add(a.ctr + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const int t = s_ticket;
        __syncthreads();   // everyone has read s_ticket before it is rewritten
        if (t >= total) break;
        const int s = t / per_slot, pos = t - s * per_slot;
        if (pos < W) {
            if (s < a.nchunks && !do_push<R, E>(a, s, (a.me + 1 + pos) % W, epoch, scale)) break;
        } else if (pos == W) {
            const int c = s - a.lag;
            if (c >= 0 && c < a.nchunks && !do_reduce<E>(a, c, epoch, inv)) break;
        } else {
            const int c = s - 2 * a.lag;
            const int jj = (a.me + pos - W) % W;
            if (c >= 0 && c < a.nchunks && !(is16(E) ? do_gather16(a, c, jj, epoch) : do_gather(a, c, jj, epoch))) break;
        }
    }
    // retire: the last workgroup resets the ticket and advances the call counter
    if (threadIdx.x == 0) {
        const uint32_t done = __hip_atomic_fetch_add(a.ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done == gridDim.x - 1) {
            __hip_atomic_store(a.ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.ctr + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.ctr + 4, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (int j = 0; j < W; ++j) __hip_atomic_store(a.ctr + 8 + j, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.ctr, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace

extern "C" int inccl_k_mesh(const struct inccl_mesh_launch* l, void* stream)
{
    if (!l || l->R < 1 || l->R > kMaxR || l->W < 1 || l->W > kMaxR || l->me < 0 || l->me >= l->W || l->grid < 1 ||
        l->nchunks < 1 || l->nchunks > INCCL_MESH_MAX_CHUNKS || l->lag < 1 || (l->shard & 63) || (l->chunk & 63) ||
        l->chunk == 0 || (l->kind16 != 0 && l->kind16 != BF16 && l->kind16 != F16) || (size_t)l->nchunks * l->chunk < l->shard || l->shard > l->inbox_stride ||
        (size_t)l->W * l->shard < l->n || l->chunk > ((size_t)1 << 26))
        return INCCL_ERR_ARG;
    MeshArgs a{};
    for (int r = 0; r < l->R; ++r) a.src.p[r] = l->src[r];
    a.dst = l->dst;
    a.n = (int64_t)l->n;
    a.shard = (int64_t)l->shard;
    a.chunk = (int64_t)l->chunk;
    a.inbox_stride = (int64_t)l->inbox_stride;
    for (int j = 0; j < l->W; ++j) {
        a.peer_inbox[j] = l->peer_inbox[j];
        a.peer_res[j] = l->peer_res[j];
        a.peer_resin[j] = l->peer_resin[j];
        a.peer_sig[j] = l->peer_sig[j];
    }
    a.own_resin = l->own_resin;
    a.push_res = l->push_res ? 1 : 0;
    a.rs = l->rs ? 1 : 0;
    if (a.push_res && (l->own_resin == nullptr || l->peer_resin[0] == nullptr)) return INCCL_ERR_ARG;
    a.own_inbox = l->own_inbox;
    a.own_res = l->own_res;
    a.own_sig = l->own_sig;
    a.ctr = l->ctr;
    a.err = l->err;
    a.timeout_ticks = l->timeout_ticks;
    a.nchunks = l->nchunks;
    a.W = l->W;
    a.me = l->me;
    a.lag = l->lag;
    int vs = 1;
    for (int r = 0; r < l->R; ++r) vs &= aligned16(l->src[r]) ? 1 : 0;
    a.vec_src = vs;
    a.vec_dst = aligned16(l->dst) ? 1 : 0;
    a.sc.k = l->scale_exp;
    a.sc.amax_bits = l->amax_bits;
    a.sc.scale_R = l->scale_R;
    a.sc.out_shift = l->out_shift;
    a.src_bytes = l->src_bytes;
    a.dst_bytes = l->dst_bytes;
    a.inbox_bytes = l->inbox_bytes;
    a.res_bytes = l->res_bytes;
    a.resin_bytes = l->resin_bytes;
    a.zero = 0;
    hipStream_t st = (hipStream_t)stream;
    const dim3 g((unsigned)l->grid), b(kMeshBlock);
#define INCCL_MESH_CASE(RR)                                                  \
    case RR:                                                                 \
        if (l->kind16 == F16)                                                \
            hipLaunchKernelGGL((k_mesh<RR, F16>), g, b, 0, st, a);           \
        else if (l->kind16 == BF16)                                          \
            hipLaunchKernelGGL((k_mesh<RR, BF16>), g, b, 0, st, a);          \
        else                                                                 \
            hipLaunchKernelGGL((k_mesh<RR, 0>), g, b, 0, st, a);             \
        break;
    switch (l->R) {
        INCCL_MESH_CASE(1) INCCL_MESH_CASE(2) INCCL_MESH_CASE(3) INCCL_MESH_CASE(4) INCCL_MESH_CASE(5)
        INCCL_MESH_CASE(6) INCCL_MESH_CASE(7)
        default: INCCL_MESH_CASE(8)
    }
#undef INCCL_MESH_CASE
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}
