"""Two processes on one GPU, p2p engine: back-to-back calls per stream kind and host-sync pattern."""
import multiprocessing as mp
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rank_main(rank, port, variant, q):
    os.environ["INCCL_ENGINE"] = "p2p"
    os.environ["INCCL_DEVICE"] = "0"
    sys.path.insert(0, ROOT)
    import torch
    from container_inc_amd import inccl
    dev = torch.device("cuda:0")
    grp = inccl.inccl_group_create(2, rank, "127.0.0.1", port=port)
    comm = inccl.inccl_communicator_create(grp, 0)
    n = 1 << 22
    srcs = [torch.randn(n, device=dev) for _ in range(2)]
    out = torch.empty(n, device=dev)
    ts = torch.cuda.Stream(device=dev)
    stream = comm.stream if variant["stream"] == "comm" else ts.cuda_stream
    err = None
    i = 0
    try:
        for i in range(variant["calls"]):
            comm.allreduce_f32(srcs, out=out, scale_exp=25, stream=stream)
            if variant["sync_every"] and (i + 1) % variant["sync_every"] == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001
        err = f"call {i}: {e}"
    q.put((rank, err, comm.engine))
    q.close()
    q.join_thread()   # flush the queue's feeder thread before the hard exit
    os._exit(0)


def main():
    variants = [
        {"stream": "comm", "sync_every": 0, "calls": 30},
        {"stream": "torch", "sync_every": 1, "calls": 30},
        {"stream": "torch", "sync_every": 0, "calls": 30},
    ]
    ctx = mp.get_context("spawn")
    for v in variants:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        q = ctx.Queue()
        ps = [ctx.Process(target=rank_main, args=(r, port, v, q)) for r in range(2)]
        for p in ps:
            p.start()
        res = [q.get(timeout=120) for _ in range(2)]
        for p in ps:
            p.join(timeout=30)
        print(v, sorted(res), flush=True)


if __name__ == "__main__":
    main()
