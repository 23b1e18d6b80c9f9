"""Small-bucket latency, two processes sharing one GPU (BASELINE config 5, the
N=2 rehearsal; the 8-GPU sweep is the driver's): per bucket size, microseconds
per allreduce_f32 call for the sharded p2p exchange (two host barriers per call)
and for the ll engine (one kernel, device-side arrival flags).  Bit-equality of
the two engines' outputs is checked at every size.  One JSON line per size.

    python tools/ll_sweep.py [--out gpurun_out/ll_sweep.jsonl]
"""
import argparse
import json
import multiprocessing as mp
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZES = [4 << 10, 16 << 10, 64 << 10, 256 << 10, 1 << 20]


def rank_main(rank, port, q):
    os.environ["INCCL_DEVICE"] = "0"
    os.environ["INCCL_ENGINE"] = "p2p"
    sys.path.insert(0, ROOT)
    import torch
    from container_inc_amd import inccl
    dev = torch.device("cuda:0")
    grp = inccl.inccl_group_create(2, rank, "127.0.0.1", port=port)
    os.environ["INCCL_LL_MAX_BYTES"] = "0"          # read at creation: the sharded exchange only
    comms = {"p2p": inccl.inccl_communicator_create(grp, 0)}
    os.environ["INCCL_LL_MAX_BYTES"] = str(1 << 20)
    os.environ["INCCL_ENGINE"] = "ll"
    comms["ll"] = inccl.inccl_communicator_create(grp, 0)
    st = torch.cuda.Stream(device=dev)
    rows = []
    for b in SIZES:
        n = b // 4
        g = torch.Generator(device=dev).manual_seed(77 + rank)
        srcs = [torch.randn(n, generator=g, device=dev) for _ in range(2)]
        res = {}
        outs = {}
        for eng, comm in comms.items():
            out = torch.empty(n, device=dev)
            iters = 300
            for _ in range(20):
                comm.allreduce_f32(srcs, out=out, scale_exp=25, stream=st.cuda_stream)
            torch.cuda.synchronize()
            comm.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(iters):
                comm.allreduce_f32(srcs, out=out, scale_exp=25, stream=st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            res[eng] = round(e0.elapsed_time(e1) * 1e3 / iters, 2)
            outs[eng] = out.clone()
            if eng == "ll":   # the same calls captured in a hipGraph and replayed
                per = 20
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=st):
                    for _ in range(per):
                        comm.allreduce_f32(srcs, out=out, scale_exp=25, stream=st.cuda_stream)
                with torch.cuda.stream(st):   # replay() launches on the current stream
                    graph.replay()
                    torch.cuda.synchronize()
                    comm.barrier()
                    e0.record(st)
                    for _ in range(iters // per):
                        graph.replay()
                    e1.record(st)
                torch.cuda.synchronize()
                res["ll_graph"] = round(e0.elapsed_time(e1) * 1e3 / (iters // per * per), 2)
                outs["ll_graph"] = out.clone()
                del graph
        rows.append({"bucket_bytes": b, "us_per_call_p2p": res["p2p"], "us_per_call_ll": res["ll"],
                     "us_per_call_ll_graph": res["ll_graph"],
                     "bit_equal": bool(torch.equal(outs["p2p"], outs["ll"]) and torch.equal(outs["p2p"], outs["ll_graph"]))})
    for comm in comms.values():
        comm.destroy()
    grp.destroy()
    q.put((rank, rows))
    q.close()
    q.join_thread()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--grid-cap", type=int, default=0, help="INCCL_LL_GRID_CAP for the ll kernel")
    a = ap.parse_args()
    if a.grid_cap:
        os.environ["INCCL_LL_GRID_CAP"] = str(a.grid_cap)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    lines = []
    for row0, row1 in zip(got[0], got[1]):
        row = dict(row0)
        row["us_per_call_p2p"] = max(row0["us_per_call_p2p"], row1["us_per_call_p2p"])
        row["us_per_call_ll"] = max(row0["us_per_call_ll"], row1["us_per_call_ll"])
        row["us_per_call_ll_graph"] = max(row0["us_per_call_ll_graph"], row1["us_per_call_ll_graph"])
        row["bit_equal"] = row0["bit_equal"] and row1["bit_equal"]
        row["setup"] = "2 processes sharing one MI355X (IPC on one device), R=2 fp32 buckets, k=25"
        row["ll_grid_cap"] = a.grid_cap or 64
        lines.append(json.dumps(row))
        print(lines[-1], flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")
    ok = all(json.loads(x)["bit_equal"] for x in lines)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
