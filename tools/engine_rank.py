"""One rank of an N > 1 engine run, as its own process, so that each rank can be
started under its own profiler from a shell (no launcher process that would
fork/exec children after the profiler initialised the GPU):

    for r in 0 1; do rocprofv3 --kernel-trace --stats -d out/r$r -o run -- \\
        python tools/engine_rank.py $r 2 PORT p2p 256 & done; wait

Every rank sits on device 0 (a one-GPU rehearsal).  R = 2 resident buckets of
MIB MiB, k = 25; warmup calls, then ITERS timed calls on one stream; rank 0
prints one JSON line (ms per call, max over ranks through the group barrier
order).  The first call's output is checked against the oracle."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port, engine = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    mib = float(sys.argv[5]) if len(sys.argv) > 5 else 256.0   # fractions: 0.00390625 = 4 KiB
    iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
    k = 0x7FFFFFFF if os.environ.get("SCALE") == "auto" else 25   # SCALE=auto: inccl SCALE_AUTO
    os.environ.setdefault("INCCL_ENGINE", engine if engine in ("p2p", "mesh", "meshw") else "p2p")
    import numpy as np
    import torch
    import container_inc_amd
    from container_inc_amd import inccl
    container_inc_amd.load()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    n = max(64, int(mib * (1 << 18)))
    grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port, device=0)
    if grp is None:
        raise SystemExit("group create failed")
    comm = inccl.inccl_communicator_create(grp, 0)
    comm.set_engine(engine)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000 + rank)
    xs = [torch.randn(n, generator=gen, device=dev) for _ in range(2)]
    out = torch.empty(n, device=dev)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    comm.allreduce_f32(xs, out=out, scale_exp=k, stream=st.cuda_stream)
    torch.cuda.synchronize()
    ok = None
    if mib <= 64:   # oracle check of the first call (every rank's inputs regenerated here)
        from oracle import oracle as O
        every = []
        for r in range(world):
            g = torch.Generator(device=dev)
            g.manual_seed(1000 + r)
            every += [torch.randn(n, generator=g, device=dev).cpu().numpy() for _ in range(2)]
        kk = O.choose_scale(O.absmax(every), 2 * world) if k != 25 else 25
        ok = bool(np.array_equal(out.cpu().numpy().view(np.uint32), O.reduce_f32(every, kk).view(np.uint32)))
    for _ in range(5):
        comm.allreduce_f32(xs, out=out, scale_exp=k, stream=st.cuda_stream)
    torch.cuda.synchronize()
    comm.barrier()
    per_call = []
    t0 = time.perf_counter()
    for _ in range(iters):
        t1 = time.perf_counter()
        comm.allreduce_f32(xs, out=out, scale_exp=k, stream=st.cuda_stream)
        if os.environ.get("PER_CALL"):   # host time of each call, synchronised
            torch.cuda.synchronize()
            per_call.append(round((time.perf_counter() - t1) * 1e3, 3))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    comm.barrier()
    print(json.dumps({"rank": rank, "world": world, "engine": engine, "bucket_mib": mib, "R": 2,
                      "scale": "auto" if k != 25 else 25, "host_max_tcp": os.environ.get("INCCL_HOST_MAX_TCP"),
                      "ms_per_call": round(dt * 1e3, 4), "oracle_ok": ok,
                      **({"per_call_ms": per_call} if per_call else {})}), flush=True)
    comm.destroy()
    grp.destroy()


if __name__ == "__main__":
    main()
