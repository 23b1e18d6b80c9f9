"""BASELINE config 3 pipeline shapes on this box (1 GiB pinned fp32, 64 MiB
buckets), all with the library's fused kernel:
  lib      inccl_allreduce_f32_host as built
  events   H2D / kernel / D2H streams joined by events (the library's shape, in torch)
  chainsK  K streams, each running whole H2D -> kernel (in place) -> D2H chains
  copies   H2D and D2H alone on two streams (the PCIe ceiling)
One JSON line per variant."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import container_inc_amd
    from container_inc_amd import inccl
    container_inc_amd.load()
    dev = torch.device("cuda:0")
    gib = int(os.environ.get("GIB", "1"))
    n = (gib << 30) // 4
    B = (int(os.environ.get("BUCKET_MIB", "64")) << 20) // 4
    x = torch.randn(n).pin_memory()
    y = torch.empty(n).pin_memory()
    pre = os.environ.get("PRE", "")   # bench-like process state before the pipeline runs
    if "dev" in pre:
        torch.cuda.set_device(0)
    early = [torch.randn((256 << 20) // 4, device=dev) for _ in range(3)] if "allocfirst" in pre else []
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1", device=0 if "dev" in pre else -1)
    comm = inccl.inccl_communicator_create(grp, 0)
    if "stagefirst" in pre:   # the library's staging buffers exist before the big allocations
        comm.allreduce_f32_host(x, y, scale_exp=25, bucket_bytes=B * 4)
    big = [torch.randn((256 << 20) // 4, device=dev) for _ in range(3)] if "alloc" in pre else []
    if "free" in pre:
        del big
        big = []
        torch.cuda.empty_cache()
    if "run" in pre:
        st = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()
        for _ in range(60):
            comm.allreduce_f32(big[:2], out=big[2], scale_exp=25, stream=st.cuda_stream)
        torch.cuda.synchronize()
    if "streams" in pre:
        extra = [torch.cuda.Stream(device=dev) for _ in range(6)]
        for e in extra:
            with torch.cuda.stream(e):
                torch.empty(1024, device=dev).fill_(1)
        torch.cuda.synchronize()
    variants = os.environ.get("VARIANTS", "lib,events,chains2,chains3,chains4,copies,lib").split(",")

    def timeit(fn, reps=4):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    def lib():
        comm.allreduce_f32_host(x, y, scale_exp=25, bucket_bytes=B * 4)

    sh, sk, sd = (torch.cuda.Stream(device=dev) for _ in range(3))
    din = [torch.empty(B, device=dev) for _ in range(2)]
    dout = [torch.empty(B, device=dev) for _ in range(2)]

    def events():
        eh = [None, None]
        ek = [None, None]
        ed = [None, None]
        for i, off in enumerate(range(0, n, B)):
            s = i & 1
            with torch.cuda.stream(sh):
                if ek[s] is not None:
                    sh.wait_event(ek[s])
                din[s].copy_(x[off:off + B], non_blocking=True)
                eh[s] = torch.cuda.Event()
                eh[s].record(sh)
            with torch.cuda.stream(sk):
                sk.wait_event(eh[s])
                if ed[s] is not None:
                    sk.wait_event(ed[s])
                inccl.reduce_f32([din[s]], 25, out=dout[s], stream=sk.cuda_stream)
                ek[s] = torch.cuda.Event()
                ek[s].record(sk)
            with torch.cuda.stream(sd):
                sd.wait_event(ek[s])
                y[off:off + B].copy_(dout[s], non_blocking=True)
                ed[s] = torch.cuda.Event()
                ed[s].record(sd)

    def chains(K):
        ss = [torch.cuda.Stream(device=dev) for _ in range(K)]
        bufs = [torch.empty(B, device=dev) for _ in range(K)]

        def run():
            for i, off in enumerate(range(0, n, B)):
                j = i % K
                with torch.cuda.stream(ss[j]):
                    bufs[j].copy_(x[off:off + B], non_blocking=True)
                    inccl.reduce_f32([bufs[j]], 25, out=bufs[j], stream=ss[j].cuda_stream)
                    y[off:off + B].copy_(bufs[j], non_blocking=True)
        return run

    def copies():
        for off in range(0, n, B):
            with torch.cuda.stream(sh):
                din[0].copy_(x[off:off + B], non_blocking=True)
            with torch.cuda.stream(sd):
                y[off:off + B].copy_(dout[0], non_blocking=True)

    import ctypes
    L = container_inc_amd.load()
    zst = torch.cuda.Stream(device=dev)

    def zc(bucket_elems):
        def run():
            for off in range(0, n, bucket_elems):
                cnt = min(bucket_elems, n - off)
                srcs = (ctypes.c_void_p * 1)(x.data_ptr() + 4 * off)
                rc = L.inccl_reduce_f32(srcs, 1, ctypes.c_void_p(y.data_ptr() + 4 * off), ctypes.c_size_t(cnt), 25,
                                        ctypes.c_void_p(zst.cuda_stream))
                assert rc == 0, rc
        return run

    state = {"comm": comm, "grp": grp}

    def lib_newcomm():
        if "fresh" not in state:
            state["comm"].destroy()
            state["grp"].destroy()
            state["grp"] = inccl.inccl_group_create(1, 0, "127.0.0.1")
            state["comm"] = inccl.inccl_communicator_create(state["grp"], 0)
            state["fresh"] = True
        state["comm"].allreduce_f32_host(x, y, scale_exp=25, bucket_bytes=B * 4)

    table = {"zc1": zc(n), "zc64": zc(B), "lib_newcomm": lib_newcomm, "lib": lambda: state["comm"].allreduce_f32_host(
        x, y, scale_exp=25, bucket_bytes=B * 4), "events": events, "chains2": chains(2), "chains3": chains(3), "chains4": chains(4),
             "copies": copies}
    for name in variants:
        dt = timeit(table[name])
        print(json.dumps({"pre": pre, "variant": name, "ms": round(dt * 1e3, 2),
                          "GBps": round((gib << 30) / dt / 1e9, 2)}), flush=True)
    state["comm"].destroy()
    state["grp"].destroy()


if __name__ == "__main__":
    main()
