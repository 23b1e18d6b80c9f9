"""Host-memory end-to-end rates (BASELINE config 3 and the reference API path).

* config 3: a 1 GiB fp32 gradient in pinned host memory, split into 64 MiB
  buckets, pipelined H2D / reduce / D2H on three HIP streams
  (inccl_allreduce_f32_host), vs the same work issued serially per bucket.
* reference API: inccl_allreduce_write on host int32 arrays (api.c:403-452
  replacement) at 4 / 64 / 256 MiB, world 1 (RCCL transport) and the
  in-process 2-rank transport (ranks = threads sharing the GPU).

Prints one JSON line per measurement.
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import container_inc_amd
    from container_inc_amd import inccl
    container_inc_amd.load()
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)

    total = int(os.environ.get("HOST_BENCH_GIB", "1")) << 30
    n = total // 4
    x = torch.randn(n, dtype=torch.float32).pin_memory()
    y = torch.empty(n, dtype=torch.float32).pin_memory()
    for bucket_mib in (64, 16, 256):
        bb = bucket_mib << 20
        comm.allreduce_f32_host(x, y, scale_exp=24, bucket_bytes=bb)   # warm
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            comm.allreduce_f32_host(x, y, scale_exp=24, bucket_bytes=bb)
        dt = (time.perf_counter() - t0) / reps
        print(json.dumps({"what": "config3 pipelined host fp32 allreduce (H2D/reduce/D2H, 3 streams)",
                          "gradient_gib": total >> 30, "bucket_mib": bucket_mib, "ms": round(dt * 1e3, 3),
                          "GBs_gradient": round(total / dt / 1e9, 2),
                          "GBs_pcie_both_directions": round(2 * total / dt / 1e9, 2)}), flush=True)
    # serial reference: one bucket at a time, H2D -> kernel -> D2H, synchronous
    dev = torch.device("cuda:0")
    bb = 64 << 20
    m = bb // 4
    din = torch.empty(m, device=dev)
    dout = torch.empty(m, device=dev)
    t0 = time.perf_counter()
    for off in range(0, n, m):
        din.copy_(x[off:off + m], non_blocking=False)
        comm.allreduce_f32([din], out=dout, scale_exp=24)
        y[off:off + m].copy_(dout, non_blocking=False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"what": "config3 serial per-bucket (no overlap)", "gradient_gib": total >> 30,
                      "bucket_mib": 64, "ms": round(dt * 1e3, 3), "GBs_gradient": round(total / dt / 1e9, 2)}),
          flush=True)
    # raw PCIe copy rates for context
    t0 = time.perf_counter()
    for off in range(0, n, m):
        din.copy_(x[off:off + m], non_blocking=True)
    torch.cuda.synchronize()
    h2d = total / (time.perf_counter() - t0) / 1e9
    t0 = time.perf_counter()
    for off in range(0, n, m):
        y[off:off + m].copy_(dout, non_blocking=True)
    torch.cuda.synchronize()
    d2h = total / (time.perf_counter() - t0) / 1e9
    print(json.dumps({"what": "pinned copy rates", "H2D_GBs": round(h2d, 2), "D2H_GBs": round(d2h, 2)}), flush=True)
    comm.destroy()
    grp.destroy()

    # reference API: inccl_allreduce_write on host int32
    for world, label in ((1, "rccl world 1"), (2, "local 2 ranks (threads, one GPU)")):
        for reg, mib in [(reg, mib) for reg in (False, True) for mib in (4, 64, 256)]:
            ne = (mib << 20) // 4
            srcs = [np.arange(ne, dtype=np.int32) * (r + 1) for r in range(world)]
            times = [0.0] * world
            hub = f"hb-{world}-{mib}-{int(reg)}"

            def rank(r):
                g = (inccl.inccl_group_create(1, 0, "127.0.0.1") if world == 1
                     else inccl.inccl_group_create_local(world, r, hub))
                c = inccl.inccl_communicator_create(g, 8 << 20)
                dst = np.empty(ne, np.int32)
                if reg:   # inccl_host_register: direct DMA, no staging copies
                    c.host_register(srcs[r])
                    c.host_register(dst)
                c.allreduce_write(srcs[r], ne, dst)   # warm
                t0 = time.perf_counter()
                reps = 3
                for _ in range(reps):
                    c.allreduce_write(srcs[r], ne, dst)
                times[r] = (time.perf_counter() - t0) / reps
                ok = bool(np.array_equal(dst, np.arange(ne, dtype=np.int64).astype(np.int32) * (world * (world + 1) // 2)))
                c.destroy()
                g.destroy()
                times[r] = (times[r], ok)

            th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            dt = max(t[0] for t in times)
            print(json.dumps({"what": "inccl_allreduce_write host int32", "transport": label, "bucket_mib": mib,
                              "registered": reg,
                              "ms": round(dt * 1e3, 3), "GBs_per_rank": round((mib << 20) / dt / 1e9, 3),
                              "correct": all(t[1] for t in times)}), flush=True)


if __name__ == "__main__":
    main()
