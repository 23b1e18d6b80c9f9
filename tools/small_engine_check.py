"""Two ranks on one GPU replay the bench sweep's small-bucket sequence (per
size: ll verified calls, an ll hipGraph capture + replays, then p2p verified
calls) and check EVERY output against the oracle, to tell which engine is wrong
when the sweep reports a mismatch.  Prints one line per wrong call."""
import multiprocessing as mp
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_main(rank, world, port, q, graph):
    os.environ["INCCL_DEVICE"] = "0"
    os.environ["INCCL_BOOT_TIMEOUT"] = "120"
    os.environ["INCCL_LL_TIMEOUT_MS"] = "2000"
    import numpy as np
    import torch
    from container_inc_amd import inccl
    from oracle import oracle as O
    dev = torch.device("cuda:0")
    grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port)
    comm = inccl.inccl_communicator_create(grp, 0)   # RCCL refuses a shared GPU: p2p engine
    lines = []
    R, k = 2, 25
    for b in [(4 << 10) << (2 * i) for i in range(5)]:
        n = b // 4
        sets, wants = [], []
        for seed in (7000, 8000):
            every = []
            for r in range(world):
                g = torch.Generator(device=dev)
                g.manual_seed(seed + r)
                xs = [torch.randn(n, generator=g, device=dev) for _ in range(R)]
                every += [x.cpu().numpy() for x in xs]
                if r == rank:
                    sets.append(xs)
            wants.append(O.reduce_f32(every, k).view(np.uint32))
        out = torch.empty(n, device=dev)
        st = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()
        for eng in ("ll", "p2p"):
            comm.set_engine(eng)
            for call, which in enumerate((0, 1, 0, 1, 0)):
                out.fill_(float("nan"))
                torch.cuda.synchronize()
                comm.allreduce_f32(sets[which], out=out, scale_exp=k, stream=st.cuda_stream)
                torch.cuda.synchronize()
                got = out.cpu().numpy().view(np.uint32)
                bad = np.flatnonzero(got != wants[which])
                if bad.size:
                    lines.append(f"{b} B {eng} call {call} set {which}: {bad.size} wrong lanes, first {bad[:4].tolist()}")
            if eng == "ll" and graph:
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, stream=st):
                    for _ in range(20):
                        comm.allreduce_f32(sets[0], out=out, scale_exp=k, stream=st.cuda_stream)
                for _ in range(11):
                    gr.replay()
                torch.cuda.synchronize()
                got = out.cpu().numpy().view(np.uint32)
                if not np.array_equal(got, wants[0]):
                    lines.append(f"{b} B ll graph replay wrong")
                del gr
    comm.destroy()
    grp.destroy()
    q.put((rank, lines))


def main():
    graph = len(sys.argv) > 1 and sys.argv[1] == "graph"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, 2, port, q, graph)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
    bad = 0
    for r, lines in sorted(res):
        print(f"rank {r}: {len(lines)} wrong", flush=True)
        for ln in lines:
            print("   ", ln, flush=True)
        bad += len(lines)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
