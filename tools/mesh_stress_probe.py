"""One rank of a mesh-engine stress run: W processes on one GPU, many calls of
one mode sequence, every call checked exactly, a timed-out wait reported with
the wait it was (inccl_mesh.hip wait_flag).  Started per rank from a shell
(tools/gpu_mesh_stress.sh), so no launcher forks after GPU init.

    python tools/mesh_stress_probe.py RANK PORT W MODE CALLS LOG2 [LOG2 ...] [--concurrent]

--concurrent: while each call's kernel runs, W + 1 elementwise torch kernels
over the bucket on torch's stream (what the tests' expected-value code does).

MODE: ar (mesh allreduce fp32), rs (mesh reduce-scatter fp32), mix (the two
alternating), w (meshw allreduce).  Rank r's bucket in call i is (r + 1) * m * b
with m = 1 + i % 3 and b a multiple of 2^-12 below 1/2: exact at k = 20, and
different from the previous call's.  One JSON line per rank: calls
made, wrong calls, and the first error (a timeout names its wait)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, port, world, mode, calls = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4],
                                      int(sys.argv[5]))
    concurrent = "--concurrent" in sys.argv
    logs = [int(v) for v in sys.argv[6:] if not v.startswith("--")] or [20]
    os.environ["INCCL_ENGINE"] = "meshw" if mode == "w" else "mesh"
    os.environ["INCCL_DEVICE"] = "0"
    os.environ.setdefault("INCCL_BOOT_TIMEOUT", "120")
    os.environ.setdefault("INCCL_LL_TIMEOUT_MS", "10000")
    import torch
    from container_inc_amd import inccl
    dev = torch.device("cuda", 0)
    grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port, device=0)
    comm = inccl.inccl_communicator_create(grp, 0)
    made, wrong, err = 0, 0, None
    try:
        for lg in logs:
            shard = 1 << lg
            n = world * shard
            i = torch.arange(n, device=dev, dtype=torch.int64)
            b = ((i % 4093) - 2046).to(torch.float32) * 2.0 ** -12
            # three buckets that differ call to call (m = 1, 2, 3), so a partial
            # read stale from the previous call cannot pass as the right one
            xs = [b * float((rank + 1) * m) for m in (1, 2, 3)]
            fulls = [b * float(world * (world + 1) // 2 * m) for m in (1, 2, 3)]
            torch.cuda.synchronize()
            for call in range(calls):
                rs = mode == "rs" or (mode == "mix" and call % 2 == 1)
                x, full = xs[call % 3], fulls[call % 3]
                if rs:
                    out = comm.reduce_scatter([x], scale_exp=20, stream=comm.stream)
                else:
                    out = comm.allreduce_f32([x], scale_exp=20, stream=comm.stream)
                if concurrent:   # torch work on its own stream while the mesh kernel runs (as the tests' checks)
                    acc = torch.zeros_like(x)
                    for r in range(world):
                        acc += b * float(r + 1)
                    del acc
                torch.cuda.synchronize()
                made += 1
                wrong += 0 if torch.equal(out, full[rank * shard:(rank + 1) * shard] if rs else full) else 1
            del i, b, xs, fulls
        if comm.clear_error():   # a timeout of the last call is reported here
            err = "the last call timed out"
    except Exception as e:  # noqa: BLE001
        err = repr(e)[:400]
    print(json.dumps({"rank": rank, "mode": mode, "calls": made, "wrong": wrong, "error": err}), flush=True)
    try:
        comm.destroy()
        grp.destroy()
    except Exception:  # noqa: BLE001
        pass


if __name__ == "__main__":
    main()
