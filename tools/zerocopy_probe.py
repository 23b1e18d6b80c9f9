"""BASELINE config 3 without staging copies: the fused stream kernel reading a
pinned host fp32 gradient and writing the pinned host result directly over
PCIe ("zero-copy"), per 64 MiB bucket or in one launch, vs the 3-stream
H2D / kernel / D2H pipeline.  A probe for the host path's design.

    python tools/zerocopy_probe.py
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import container_inc_amd
    from container_inc_amd import inccl
    from oracle import oracle as O
    L = container_inc_amd.load()
    torch.cuda.init()
    n = (1 << 30) // 4
    x = torch.randn(n, dtype=torch.float32).pin_memory()
    y = torch.empty(n, dtype=torch.float32).pin_memory()
    st = torch.cuda.Stream()
    k = 24

    def zc(bucket_elems):
        for off in range(0, n, bucket_elems):
            cnt = min(bucket_elems, n - off)
            srcs = (ctypes.c_void_p * 1)(x.data_ptr() + 4 * off)
            rc = L.inccl_reduce_f32(srcs, 1, ctypes.c_void_p(y.data_ptr() + 4 * off), ctypes.c_size_t(cnt), k,
                                    ctypes.c_void_p(st.cuda_stream))
            assert rc == 0, rc

    for name, be in (("zero-copy, one launch", n), ("zero-copy, 64 MiB buckets", 16 << 20),
                     ("zero-copy, 16 MiB buckets", 4 << 20)):
        zc(be)
        torch.cuda.synchronize()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            zc(be)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        print(json.dumps({"what": name, "ms": round(dt * 1e3, 3), "GBs_gradient": round((1 << 30) / dt / 1e9, 2)}),
              flush=True)
    # hybrid: H2D by the copy engine into a 2-slot device ring on one stream, the
    # kernel reads the slot and writes the pinned host result directly
    dev = torch.device("cuda:0")
    hs = torch.cuda.Stream()
    for be_mib in (64, 16):
        be = be_mib << 18
        ring = [torch.empty(be, device=dev) for _ in range(2)]
        ev_in = [torch.cuda.Event() for _ in range(2)]
        ev_used = [torch.cuda.Event() for _ in range(2)]

        def hybrid():
            for i, off in enumerate(range(0, n, be)):
                s = i & 1
                cnt = min(be, n - off)
                with torch.cuda.stream(hs):
                    if i >= 2:
                        hs.wait_event(ev_used[s])
                    ring[s][:cnt].copy_(x[off:off + cnt], non_blocking=True)
                    ev_in[s].record(hs)
                st.wait_event(ev_in[s])
                srcs = (ctypes.c_void_p * 1)(ring[s].data_ptr())
                rc = L.inccl_reduce_f32(srcs, 1, ctypes.c_void_p(y.data_ptr() + 4 * off), ctypes.c_size_t(cnt), k,
                                        ctypes.c_void_p(st.cuda_stream))
                assert rc == 0, rc
                ev_used[s].record(st)

        hybrid()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            hybrid()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        print(json.dumps({"what": f"hybrid: copy-engine H2D + kernel writing host, {be_mib} MiB buckets",
                          "ms": round(dt * 1e3, 3), "GBs_gradient": round((1 << 30) / dt / 1e9, 2)}), flush=True)
    m = 1 << 22
    want = O.reduce_f32([x[:m].numpy()], k)
    print(json.dumps({"what": "zero-copy bit-exact vs oracle (first 16 MiB)",
                      "ok": bool(np.array_equal(y[:m].numpy().view(np.uint32), want.view(np.uint32)))}), flush=True)
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    comm.allreduce_f32_host(x, y, scale_exp=k, bucket_bytes=64 << 20)
    t0 = time.perf_counter()
    for _ in range(5):
        comm.allreduce_f32_host(x, y, scale_exp=k, bucket_bytes=64 << 20)
    dt = (time.perf_counter() - t0) / 5
    print(json.dumps({"what": "3-stream pipeline, 64 MiB buckets", "ms": round(dt * 1e3, 3),
                      "GBs_gradient": round((1 << 30) / dt / 1e9, 2)}), flush=True)
    comm.destroy()
    grp.destroy()


if __name__ == "__main__":
    main()
