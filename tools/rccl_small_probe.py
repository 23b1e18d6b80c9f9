"""The rccl engine's small-bucket route (INCCL_RCCL_AR_BYTES) on a one-rank
RCCL communicator: per-call device time of an fp32 allreduce through one
ncclAllReduce (the route) against reduce-scatter + all-gather (the route off),
with the sharded path forced at world 1 (INCCL_FORCE_SHARDED).  One rank moves
no bytes between GPUs, so this measures what the route saves in launches and
RCCL's per-collective work, not link time.  Prints one JSON line.

    python tools/rccl_small_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    os.environ.update(INCCL_FORCE_RCCL="1", INCCL_FORCE_SHARDED="1", INCCL_MASTER_PORT="0")
    import torch

    from container_inc_amd import inccl
    dev = torch.device("cuda:0")
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comms = {}
    for label, val in (("one_allreduce", None), ("rs_ag", "0")):
        if val is None:
            os.environ.pop("INCCL_RCCL_AR_BYTES", None)
        else:
            os.environ["INCCL_RCCL_AR_BYTES"] = val
        comms[label] = inccl.inccl_communicator_create(grp, 0)
    rows = []
    for nbytes in (4 << 10, 64 << 10, 256 << 10, 1 << 20):
        n = nbytes // 4
        xs = [torch.randn(n, device=dev) for _ in range(2)]
        out = torch.empty(n, device=dev)
        row = {"bucket_bytes": nbytes}
        for label, comm in comms.items():
            st = torch.cuda.ExternalStream(comm.stream)
            for _ in range(20):
                comm.allreduce_f32(xs, out=out, scale_exp=24, stream=comm.stream)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            iters = 200
            e0.record(st)
            for _ in range(iters):
                comm.allreduce_f32(xs, out=out, scale_exp=24, stream=comm.stream)
            e1.record(st)
            torch.cuda.synchronize()
            row[label + "_us"] = round(e0.elapsed_time(e1) * 1e3 / iters, 2)
        rows.append(row)
    print(json.dumps({"what": "fp32 allreduce, R = 2, rccl engine, one rank (INCCL_FORCE_SHARDED): "
                              "one ncclAllReduce(int32) vs reduce-scatter + all-gather, us per call (HIP events)",
                      "rows": rows}))
    for c in comms.values():
        c.destroy()
    grp.destroy()


if __name__ == "__main__":
    main()
