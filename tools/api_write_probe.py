"""inccl_allreduce_write (the reference's entry point) on a host int32 message at
world 1, registered and unregistered, in a fresh process or after bench-like
GPU activity (PRE=bench: resident buckets, fused launches on a side stream and
a config-3 pipeline first).  Also times the registered path's pieces alone:
H2D and D2H copies of the same chunks on the library's copy-stream priority
and a pure H2D+D2H ping-pong.  One JSON line per measurement.
    MIB=256 PRE=bench python tools/api_write_probe.py"""
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
    container_inc_amd.load()
    dev = torch.device("cuda:0")
    mib = int(os.environ.get("MIB", "256"))
    pre = os.environ.get("PRE", "")
    n = mib << 18
    torch.cuda.set_device(0)
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1", device=0)
    comm = inccl.inccl_communicator_create(grp, 0)
    if pre == "warm":   # GPU busy for ~0.5 s right before, nothing else
        xs = [torch.randn((256 << 20) // 4, device=dev) for _ in range(3)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5:
            for _ in range(20):
                inccl.reduce_f32(xs[:2], 25, out=xs[2])
            torch.cuda.synchronize()
        del xs
    if pre == "pinned":   # only the config-3 pinned host buffers first
        hx = torch.randn((1 << 30) // 4).pin_memory()
        hy = torch.empty_like(hx).pin_memory()
        comm.allreduce_f32_host(hx, hy, scale_exp=25, bucket_bytes=64 << 20)
    if pre == "bench":
        xs = [torch.randn((256 << 20) // 4, device=dev) for _ in range(3)]
        st = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()
        for _ in range(200):
            inccl.reduce_f32(xs[:2], 25, out=xs[2], stream=st.cuda_stream)
        torch.cuda.synchronize()
        hx = torch.randn((1 << 30) // 4).pin_memory()
        hy = torch.empty_like(hx).pin_memory()
        comm.allreduce_f32_host(hx, hy, scale_exp=25, bucket_bytes=64 << 20)
    rng = np.random.default_rng(9)
    src = rng.integers(-(2 ** 31), 2 ** 31 - 1, n, dtype=np.int64, endpoint=True).astype(np.int32)
    dst = np.empty_like(src)

    def emit(**kw):
        print(json.dumps(dict(pre=pre or "fresh", mib=mib, **kw)), flush=True)

    if os.environ.get("HOSTREF"):   # what the unregistered path is built from, alone
        dbuf = torch.empty(n, dtype=torch.int32, device=dev)
        ps, pd = torch.from_numpy(src), torch.from_numpy(dst)
        for label, fn in (("np_copyto_1thread", lambda: np.copyto(dst, src)),
                          ("hip_pageable_h2d", lambda: dbuf.copy_(ps)),
                          ("hip_pageable_d2h", lambda: pd.copy_(dbuf))):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 3
            emit(what=label, ms=round(dt * 1e3, 3), GBps=round(n * 4 / dt / 1e9, 2))
        del dbuf
    if os.environ.get("F32HOST"):   # config 3's entry point on pageable numpy buffers, 1 GiB, 64 MiB buckets
        from oracle import oracle as O
        xf = np.random.default_rng(3).standard_normal((1 << 30) // 4).astype(np.float32)
        yf = np.empty_like(xf)
        ms = []
        for _ in range(5):
            t0 = time.perf_counter()
            comm.allreduce_f32_host(xf, yf, scale_exp=25, bucket_bytes=64 << 20)
            ms.append(round((time.perf_counter() - t0) * 1e3, 2))
        ok = bool(np.array_equal(yf.view(np.uint32), O.reduce_f32([xf], 25).view(np.uint32)))
        emit(what="f32_host_pageable_1GiB", ms_per_call=ms, GBps_best=round((1 << 30) / min(ms) / 1e6, 2), correct=ok)
    if os.environ.get("SERIES"):   # per-call times over a long series: when does a slow phase end?
        for phase in ("first_registration", "second_registration_new_buffers"):
            s2 = src.copy() if phase.startswith("second") else src
            d2 = np.empty_like(dst) if phase.startswith("second") else dst
            comm.host_register(s2)
            comm.host_register(d2)
            t_start = time.perf_counter()
            ms = []
            for _ in range(int(os.environ["SERIES"])):
                t0 = time.perf_counter()
                comm.allreduce_write(s2, n, d2)
                ms.append(round((time.perf_counter() - t0) * 1e3, 2))
            emit(what="series_registered", phase=phase, ms_per_call=ms,
                 elapsed_s=round(time.perf_counter() - t_start, 3), correct=bool(np.array_equal(s2, d2)))
            comm.host_deregister(s2)
            comm.host_deregister(d2)
            # the same series unregistered (HIP pageable copies)
            ms = []
            for _ in range(int(os.environ["SERIES"])):
                t0 = time.perf_counter()
                comm.allreduce_write(s2, n, d2)
                ms.append(round((time.perf_counter() - t0) * 1e3, 2))
            emit(what="series_unregistered", phase=phase, ms_per_call=ms)
    modes = [m for m in os.environ.get("MODES", "unregistered,registered,registered,unregistered").split(",") if m]
    for mode in modes:
        if mode == "registered":
            comm.host_register(src)
            comm.host_register(dst)
        comm.allreduce_write(src, n, dst)
        t0 = time.perf_counter()
        for _ in range(3):
            comm.allreduce_write(src, n, dst)
        dt = (time.perf_counter() - t0) / 3
        emit(what="allreduce_write", mode=mode, copy_threads=os.environ.get("INCCL_COPY_THREADS", "4"), ms=round(dt * 1e3, 3), GBps=round(n * 4 / dt / 1e9, 2),
             correct=bool(np.array_equal(src, dst)))
        if mode == "registered":
            # the same DMA pattern through torch on pinned tensors: 16 MiB chunks, H2D on
            # one stream, D2H on another, chunk i's D2H beside chunk i+1's H2D
            ps, pd = torch.from_numpy(src), torch.from_numpy(dst)
            dbuf = torch.empty(2 * (4 << 20), dtype=torch.int32, device=dev)
            prio = torch.cuda.Stream(device=dev, priority=-1), torch.cuda.Stream(device=dev, priority=-1)
            for label, (s_h, s_d) in (("hi_prio_streams", prio),
                                      ("default_prio_streams", (torch.cuda.Stream(device=dev),
                                                                torch.cuda.Stream(device=dev)))):
                def run():
                    ch = 4 << 20
                    evs = []
                    for i in range(0, n, ch):
                        s = (i // ch) & 1
                        d = dbuf[s * ch:(s + 1) * ch]
                        c = min(ch, n - i)
                        with torch.cuda.stream(s_h):
                            if len(evs) >= 2:
                                s_h.wait_event(evs[-2])
                            d[:c].copy_(ps[i:i + c], non_blocking=True)
                            e = torch.cuda.Event()
                            e.record(s_h)
                        with torch.cuda.stream(s_d):
                            s_d.wait_event(e)
                            pd[i:i + c].copy_(d[:c], non_blocking=True)
                            e2 = torch.cuda.Event()
                            e2.record(s_d)
                            evs.append(e2)
                    torch.cuda.synchronize()
                run()
                t0 = time.perf_counter()
                for _ in range(3):
                    run()
                dt = (time.perf_counter() - t0) / 3
                emit(what="torch_h2d_d2h_pingpong_16MiB", streams=label, ms=round(dt * 1e3, 3),
                     GBps=round(n * 4 / dt / 1e9, 2))
            comm.host_deregister(src)
            comm.host_deregister(dst)
    comm.destroy()
    grp.destroy()


if __name__ == "__main__":
    main()
