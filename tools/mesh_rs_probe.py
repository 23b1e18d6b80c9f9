"""Reduce-scatter through the IPC engines with W processes on one GPU, at
shard sizes up to the bench's 256 MiB buckets, checked exactly without the
oracle: rank r's bucket is (r + 1) * b, with b[i] = ((i % 4093) - 2046) * 2^-12,
so every partial sum is exact in fixed point at k = 20 and the reduced bucket
is W (W + 1) / 2 * b.  Prints one JSON line per rank-0 case: how many of the
shard's elements differ, and the first differing chunks (the mesh engines'
chunk size), for the first call and for a later one.

    python tools/mesh_rs_probe.py W engine [--pre16] shard_log2 [shard_log2 ...]
    python tools/mesh_rs_probe.py --rank R PORT W engine [--pre16] shard_log2 ...

The --rank form runs ONE rank in this process and prints its JSON line, so
that each rank can be started under its own rocprofv3 from a shell
(tools/gpu_mesh_rs.sh): no launcher that forks after the profiler initialised
the GPU.

--pre16: a bf16 allreduce of the same bucket size on the same communicator
before the reduce-scatter calls (the bench's order: its bf16 / f16 phases run
the mesh engine's 16-bit allreduce before its reduce-scatter phase).  Rank 0
prints a progress line per case to stderr."""
import json
import multiprocessing as mp
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank(rank, world, port, engine, logs, pre16, q):
    try:
        os.environ["INCCL_ENGINE"] = engine
        os.environ["INCCL_DEVICE"] = "0"
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        os.environ["INCCL_MESH_RS"] = "1"   # the mesh engines' own route (the default since round 6)
        sys.path.insert(0, ROOT)
        import torch
        from container_inc_amd import inccl
        dev = torch.device("cuda", 0)
        grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port, device=0)
        comm = inccl.inccl_communicator_create(grp, 0)
        res = []
        for lg in logs:
            shard = 1 << lg
            n = world * shard
            i = torch.arange(n, device=dev, dtype=torch.int64)
            b = ((i % 4093) - 2046).to(torch.float32) * 2.0 ** -12
            x = b * float(rank + 1)
            want = (b * float(world * (world + 1) // 2))[rank * shard:(rank + 1) * shard]
            torch.cuda.synchronize()   # x is made on torch's stream; the calls run on comm.stream
            chunk = None
            if pre16:
                h = torch.randn(n, device=dev).to(torch.bfloat16)
                comm.allreduce_bf16([h], out=torch.empty_like(h), scale_exp=20, stream=comm.stream)
                torch.cuda.synchronize()
                del h
            for call in range(3):
                out = comm.reduce_scatter([x], scale_exp=20, stream=comm.stream)
                torch.cuda.synchronize()
                bad = (out != want).nonzero().flatten()
                row = {"shard_log2": lg, "call": call, "rank": rank, "bad": int(bad.numel())}
                if bad.numel():
                    sz = max(4096, ((shard + 255) // 256 + 4095) // 4096 * 4096) if chunk is None else chunk
                    sz = min(sz, 65536)
                    row["first_bad"] = [int(v) for v in bad[:8].tolist()]
                    row["bad_chunks_of_%d" % sz] = sorted(set(int(v) // sz for v in bad[:4096].tolist()))[:32]
                res.append(row)
                if rank == 0:
                    print(f"world {world} {engine} shard 2^{lg} call {call}: {row['bad']} bad", file=sys.stderr, flush=True)
            del i, b, x, want
        comm.destroy()
        grp.destroy()
        q.put((rank, res, None))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


class _Print:
    def put(self, item):
        rank, res, err = item
        print(json.dumps({"rank": rank, "rows": res, "error": err}), flush=True)


def main():
    if sys.argv[1] == "--rank":
        rank, port, world, engine = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
        rest = sys.argv[6:]
        pre16 = "--pre16" in rest
        logs = [int(v) for v in rest if v != "--pre16"] or [18, 23]
        _rank(rank, world, port, engine, logs, pre16, _Print())
        return
    world, engine = int(sys.argv[1]), sys.argv[2]
    pre16 = "--pre16" in sys.argv[3:]
    logs = [int(v) for v in sys.argv[3:] if v != "--pre16"] or [18, 23]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, port, engine, logs, pre16, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(world):
        r, res, err = q.get(timeout=600)
        out[r] = res if err is None else err
    for p in ps:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    print(json.dumps({"world": world, "engine": engine, "pre16": pre16, "ranks": out}), flush=True)


if __name__ == "__main__":
    main()
