"""bench.py -- BASELINE.json metric: GB/s of device-resident fp32 gradient buckets
quantised + reduced (+ dequantised), 256 MiB per bucket, 1/2/4/8 GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Workload (one "step"): every rank holds R = 2 resident 256 MiB fp32 buckets
(the reference's FAN_IN = 2 children per switch, non_termination_switch.c:23)
and produces their allreduce over all ranks into a third buffer:
  N = 1   one fused HIP kernel: dequant(sum_r quant(x_r))          (config 2)
  N > 1   the exchange engine that is fastest during warmup among rccl
          (quant + local sum -> RCCL reduce-scatter int32 -> dequant shard ->
          RCCL all-gather), ar, a2a, p2p, mesh and meshw, all bit-identical
          (config 4; DESIGN.md "Multi-GPU"); then the config 5 size sweep
value = bucket bytes reduced per second over the whole job = N * R * 256 MiB / t.

Extra JSON fields: ``roofline`` for the dominant kernel (the fused / quant+sum
kernel, algorithmic bytes (R+1)*4*n per launch, timed with HIP events on its
own stream) and ``cpu_baseline`` (the C oracle on a bounded sample, rank 0 at
N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--bucket-mib", type=int, default=256)
    p.add_argument("--local-buckets", type=int, default=2)
    p.add_argument("--scale-exp", type=int, default=25)
    p.add_argument("--chunks", type=int, default=0, help="pipelined chunks for the rccl engine (0 = tune)")
    p.add_argument("--engine", default="auto", choices=["auto", "rccl", "ar", "a2a", "p2p", "mesh", "meshw"],
                   help="N>1 exchange engine; auto = time every candidate during warmup, keep the fastest")
    p.add_argument("--no-sweep", action="store_true", help="N>1: skip the bucket-size sweep (BASELINE config 5)")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--grid-cap", type=int, default=0)
    p.add_argument("--json-out", default="")
    return p.parse_args()


def cpu_baseline(n_elems: int, R: int, k: int, seconds: float) -> dict:
    """The C restatement (oracle/inccl_oracle.c, scalar, 1 core) on a bounded
    sample of the same workload: R buckets of 16 Mi elements (64 MiB each)."""
    import numpy as np

    from oracle import oracle as O
    O.build()
    m = min(n_elems, 1 << 24)
    rng = np.random.default_rng(1000)
    xs = [rng.standard_normal(m).astype(np.float32) for _ in range(R)]
    out = None
    t0 = time.perf_counter()
    iters = 0
    while True:
        out = O.reduce_f32(xs, k)
        iters += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    del out
    return {"value": round(iters * R * m * 4 / dt / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{iters} x fused quantise+sum+dequantise of R={R} x {m * 4 >> 20} MiB fp32 buckets "
                      f"(oracle/inccl_oracle.c orc_reduce_f32, 1 thread, {dt:.1f} s)"}


def cpu_baseline_allcores(n_elems: int, R: int, k: int, seconds: float) -> dict:
    """The same restatement on every host core: threads over disjoint 1 Mi-element
    chunks of the sample (ctypes releases the GIL inside the C loop)."""
    import threading

    import numpy as np

    from oracle import oracle as O
    # the GPU box exposes the whole machine's CPUs; our share is $OMP_NUM_THREADS (16)
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cores = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), 64))
    m = min(n_elems, 1 << 24)
    rng = np.random.default_rng(1000)
    xs = [rng.standard_normal(m).astype(np.float32) for _ in range(R)]
    out = np.empty(m, np.float32)
    chunk = 1 << 20
    jobs = [(o, min(m, o + chunk)) for o in range(0, m, chunk)]
    L = O.lib()

    def worker(tid, stop_at, counter):
        while time.perf_counter() < stop_at:
            for j in range(tid, len(jobs), cores):
                lo, hi = jobs[j]
                srcs = (O.ctypes.c_void_p * R)(*[x[lo:hi].ctypes.data for x in xs])
                L.orc_reduce_f32(srcs, R, out[lo:hi].ctypes.data, hi - lo, k)
                counter[tid] += hi - lo

    counter = [0] * cores
    t0 = time.perf_counter()
    th = [threading.Thread(target=worker, args=(t, t0 + seconds, counter)) for t in range(cores)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    return {"value": round(sum(counter) * R * 4 / dt / 1e9, 4), "unit": "GB/s", "cores": cores, "kind": "port",
            "sample": f"orc_reduce_f32 over 1 Mi-element chunks of R={R} x {m * 4 >> 20} MiB buckets on {cores} "
                      f"threads for {dt:.1f} s"}


def cpu_reference_pipeline(seconds: float) -> dict:
    """The reference's own per-element CPU path restated end to end, int32:
    encode (api.c:300-302) -> root switch add per 1 KiB packet (nts.c:361-363) ->
    egress frame build + ICRC per child (util.c:331-442) -> decode (api.c:428-430),
    two ranks in one thread (oracle orc_allreduce_write_loopback with framing)."""
    import numpy as np

    from oracle import oracle as O
    m = 1 << 20   # 4 MiB bucket per rank (BASELINE config 1)
    rng = np.random.default_rng(1)
    xs = [rng.integers(-2 ** 31, 2 ** 31 - 1, m, dtype=np.int64).astype(np.int32) for _ in range(2)]
    t0 = time.perf_counter()
    iters = 0
    while True:
        rc, _, _ = O.allreduce_write_loopback(xs, with_icrc=True)
        assert rc == m // 1024
        iters += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": round(iters * m * 4 / dt / 1e9, 4), "unit": "GB/s of one rank's int32 bucket", "cores": 1,
            "kind": "port", "sample": f"{iters} x loopback inccl_allreduce_write of 2 ranks x 4 MiB int32 with "
                                      f"switch aggregation and ICRC framing, {dt:.1f} s"}


def size_sweep(comm, dev, R: int, k: int, rank: int) -> list:
    """BASELINE config 5 at N > 1: bucket sizes 4 KiB (one reference message,
    api.h:39) to 256 MiB in x4 steps, per engine: host wall time per call over back-to-back
    calls (max over ranks), and whether the output is bit-identical to the
    first engine's.  Buckets up to the ll threshold (1 MiB) take the one-kernel
    ll engine; rccl / ar run everywhere for comparison."""
    import torch
    import torch.distributed as dist
    rows = []
    for b in [(4 << 10) << (2 * i) for i in range(9)]:   # 4 KiB .. 256 MiB in x4 steps (BASELINE config 5)
        n = b // 4
        gen = torch.Generator(device=dev)
        gen.manual_seed(7000 + rank)
        xs = [torch.randn(n, generator=gen, device=dev) for _ in range(R)]
        out = torch.empty(n, device=dev)
        st = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()   # inputs made on torch's stream; the calls run on st
        ref = None
        iters = 50 if b <= (1 << 20) else 10
        for eng in (("rccl", "ar", "ll") if b <= (1 << 20) else ("rccl", "ar", "p2p", "mesh", "meshw")):
            ok, dt, same = 1, float("inf"), True
            try:
                comm.set_engine(eng)
                for _ in range(3):
                    comm.allreduce_f32(xs, out=out, scale_exp=k, stream=st.cuda_stream)
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                else:
                    same = bool(torch.equal(ref, out))
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(iters):
                    comm.allreduce_f32(xs, out=out, scale_exp=k, stream=st.cuda_stream)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / iters
            except Exception as e:  # noqa: BLE001
                print(f"rank {rank}: sweep {b} B engine {eng} failed: {e}", file=sys.stderr, flush=True)
                ok = 0
            v = torch.tensor([dt if ok else float("inf"), 0.0 if ok else 1.0, 0.0 if same else 1.0],
                             dtype=torch.float64)
            dist.all_reduce(v, op=dist.ReduceOp.MAX)
            good = v[1].item() == 0.0
            rows.append({"bucket_bytes": b, "engine": eng, "ok": good,
                         "us": round(v[0].item() * 1e6, 2) if good else None,
                         "algbw_GBps": round(b / v[0].item() / 1e9, 2) if good else None,
                         "bit_identical": v[2].item() == 0.0})
        del xs, out
    return rows


def load_traffic(workload: str):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3
    PMC summary (profiles/pmc_traffic.json), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        return d.get(workload, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    a = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import container_inc_amd
    from container_inc_amd import inccl
    from container_inc_amd.plan import chunk_plan

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"warning: WORLD_SIZE={world} but --gpus={a.gpus}; using WORLD_SIZE", file=sys.stderr)
    # rehearsal hook: every rank on device 0 (a one-GPU box running N>1 over the
    # p2p engine; RCCL refuses two ranks on one GPU)
    if os.environ.get("INCCL_BENCH_SAME_DEVICE") == "1":
        local_rank = 0
    os.environ.setdefault("INCCL_BOOT_TIMEOUT", "120")
    if a.engine in ("p2p", "mesh", "meshw"):
        os.environ["INCCL_ENGINE"] = a.engine   # no eager RCCL communicator
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    container_inc_amd.load()
    if a.grid_cap:
        inccl.set_tuning(a.grid_cap, True)

    R, k = a.local_buckets, a.scale_exp
    n = a.bucket_mib * (1 << 20) // 4
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000 + rank)
    srcs = [torch.randn(n, generator=gen, device=dev, dtype=torch.float32) for _ in range(R)]
    out = torch.empty(n, device=dev, dtype=torch.float32)
    torch.cuda.synchronize()   # inputs made on torch's stream; the library runs on its own

    master = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500")) + 17
    grp = inccl.inccl_group_create(world, rank, master, port=port, device=local_rank)
    if grp is None:
        raise SystemExit("inccl_group_create failed: " + container_inc_amd.load().inccl_last_error().decode())
    comm = inccl.inccl_communicator_create(grp, 0)
    stream = torch.cuda.Stream(device=dev)

    def barrier():
        if world > 1:
            dist.barrier()

    # N>1: pick the exchange engine / chunking during warmup (untimed).  Every
    # candidate must produce a bit-identical result (integer sums are exact);
    # any failure or mismatch on any rank drops that candidate on all ranks.
    chosen = ("rccl", 1, {})
    tuning = []
    if world > 1:
        # (engine, rccl chunks, environment of the candidate): the mesh engines'
        # phase lag is a scheduling knob whose best value depends on the fabric
        # (DESIGN.md "Engine mesh"), so both the default and a short lag run
        cands = []
        if a.engine in ("auto", "rccl"):
            cands += [("rccl", c, {}) for c in ([a.chunks] if a.chunks else [1, 4])]
        if a.engine in ("auto", "ar"):
            cands.append(("ar", 1, {}))
        if a.engine in ("auto", "a2a"):
            cands.append(("a2a", 1, {}))
        if a.engine in ("auto", "p2p"):
            cands.append(("p2p", 1, {}))
        for eng in ("mesh", "meshw"):
            if a.engine in ("auto", eng):
                cands += [(eng, 1, {}), (eng, 1, {"INCCL_MESH_LAG": "32"})]
        ref = None
        best = None
        for eng, ch, env in cands:
            ok, dt = 1, float("inf")
            os.environ.update(env)
            try:
                comm.set_engine(eng)
                for _ in range(3):
                    comm.allreduce_f32(srcs, out=out, scale_exp=k, chunks=ch, stream=stream.cuda_stream)
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                elif not torch.equal(ref, out):
                    ok = 0
                barrier()
                t0 = time.perf_counter()
                for _ in range(5):
                    comm.allreduce_f32(srcs, out=out, scale_exp=k, chunks=ch, stream=stream.cuda_stream)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
            except Exception as e:  # noqa: BLE001
                print(f"rank {rank}: engine {eng} chunks {ch} {env} failed: {e}", file=sys.stderr, flush=True)
                ok = 0
            for key in env:
                os.environ.pop(key, None)
            v = torch.tensor([dt if ok else float("inf"), 0.0 if ok else 1.0], dtype=torch.float64)
            dist.all_reduce(v, op=dist.ReduceOp.MAX)
            good = v[1].item() == 0.0
            tuning.append({"engine": eng, "chunks": ch, "env": env or None, "ok": good,
                           "ms": round(v[0].item() * 200, 3) if good else None})
            if good and (best is None or v[0].item() < best[0]):
                best = (v[0].item(), eng, ch, env)
        if best is not None:
            chosen = (best[1], best[2], best[3])
        comm.set_engine(chosen[0])
        os.environ.update(chosen[2])
    chunks = chosen[1]

    def step():
        comm.allreduce_f32(srcs, out=out, scale_exp=k, chunks=chunks, stream=stream.cuda_stream)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(a.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    dev_ms = ev0.elapsed_time(ev1)
    t = torch.tensor([wall], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t.item())
    ms_per_step = wall * 1e3 / a.steps

    # dominant kernel alone: fused (N=1) or quant + local sum (N>1), HIP events on its stream
    kstream = torch.cuda.Stream(device=dev)
    qbuf = torch.empty(n, device=dev, dtype=torch.int32) if world > 1 else None

    def kernel():
        if world == 1:
            inccl.reduce_f32(srcs, k, out=out, stream=kstream.cuda_stream)
        else:
            inccl.quant_sum(srcs, k, out=qbuf, stream=kstream.cuda_stream)

    for _ in range(3):
        kernel()
    kev0, kev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kiters = max(a.steps, 20)
    kev0.record(kstream)
    for _ in range(kiters):
        kernel()
    kev1.record(kstream)
    torch.cuda.synchronize()
    k_ms = kev0.elapsed_time(kev1) / kiters
    alg_bytes = (R + 1) * 4 * n
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    per_rank = f"R={R} resident {a.bucket_mib} MiB fp32 buckets per rank: "
    workload = (f"fused quantise+sum+dequantise of R={R} resident {a.bucket_mib} MiB fp32 buckets, 1 GPU"
                if world == 1 else per_rank + {
                    "rccl": f"quant+local sum -> RCCL reduce-scatter int32 -> dequant shard -> RCCL all-gather fp32, "
                            f"{chunks} pipelined chunks",
                    "ar": "quant+local sum -> RCCL all-reduce int32 in place -> dequant",
                    "a2a": "quant+local sum -> RCCL all-to-all of int32 shards -> fused sum+dequant (HIP) -> RCCL "
                           "all-gather fp32",
                    "p2p": "quant+local sum -> p2p pull of every peer's shard over xGMI with fused sum+dequant -> p2p "
                           "gather of every result shard",
                    "mesh": "one persistent HIP kernel: per-chunk quant+local sum pushed into the owner's inbox over "
                            "xGMI -> owner's sum+dequant on arrival flags -> pull of every result chunk",
                    "meshw": "one persistent HIP kernel: per-chunk quant+local sum pushed into the owner's inbox over "
                             "xGMI -> owner's sum+dequant on arrival flags, result chunk pushed into every rank's "
                             "inbox (all xGMI transfers are writes) -> local copy into dst",
                }.get(comm.engine, comm.engine))
    kname = "k_stream_vec<F32,F32,R>" if world == 1 else "k_stream_vec<F32,Q32,R>"
    traffic = load_traffic(kname + f" R={R} n={n}")

    value = world * R * n * 4 / (ms_per_step * 1e-3) / 1e9
    res = {
        "metric": "GB/s device-resident fp32 bucket quantise+reduce, 256 MiB, 1/2/4/8 GPUs",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "device_ms_per_step_rank0": round(dev_ms / a.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic N(0,1) fp32 buckets, torch.Generator seed 1000+rank",
        "config": {
            "workload": workload,
            "bucket_mib": a.bucket_mib,
            "local_buckets": R,
            "scale_exp": k,
            "numerics": f"fp32 in/out; quantised to int32 fixed point 2^-{k}; int32 wrap-around sum (exact)",
            "parallelism": f"dp{world}",
            "chunks": chunks,
            "engine": comm.engine if world > 1 else "fused",
            "engine_env": (chosen[2] or None) if world > 1 else None,
            "engine_tuning": tuning or None,
            "shard_elems": chunk_plan(n, world, chunks)[0][2] if world > 1 else n,
        },
        "roofline": {
            "kernel": kname,
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "alg_bytes_per_launch": alg_bytes,
            "kernel_ms": round(k_ms, 5),
        },
        "cpu_baseline": None,
    }
    if world > 1:
        # nccl-tests convention (BASELINE config 4): algbw = one rank's bucket bytes
        # / step time; busbw = algbw * 2(W-1)/W, the per-GPU link traffic of RS + AG
        algbw = n * 4 / (ms_per_step * 1e-3) / 1e9
        res["collective"] = {"algbw_GBps": round(algbw, 2), "busbw_GBps": round(algbw * 2 * (world - 1) / world, 2),
                             "bytes_per_rank": n * 4}
    if world > 1 and not a.no_sweep:
        for key in chosen[2]:   # the sweep runs every engine with its defaults
            os.environ.pop(key, None)
        res["sweep"] = size_sweep(comm, dev, R, k, rank)
        comm.set_engine(chosen[0])
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(n, R, k, a.cpu_seconds)
        res["cpu_baseline_allcores"] = cpu_baseline_allcores(n, R, k, min(a.cpu_seconds, 5.0))
        res["cpu_reference_pipeline"] = cpu_reference_pipeline(min(a.cpu_seconds, 5.0))
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    comm.destroy()
    grp.destroy()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
