"""Debugging aid: stress the ll engine's size transition seen to fail in the
bench sweep (hipGraph replays at 16 KiB, then eager calls at 64 KiB alternating
two input sets), two ranks on one GPU, every output checked against the
oracle.  argv: iterations, nan (fill dst with NaN before each call) or keep."""
import multiprocessing as mp
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_main(rank, port, q, iters, fill):
    try:
        _rank_main(rank, port, q, iters, fill)
    except BaseException as e:  # noqa: BLE001
        q.put((rank, [f"crash: {e!r}"]))


def _rank_main(rank, port, q, iters, fill):
    os.environ["INCCL_DEVICE"] = "0"
    os.environ["INCCL_LL_TIMEOUT_MS"] = "2000"
    os.environ["INCCL_ENGINE"] = "ll"
    import numpy as np
    import torch
    from container_inc_amd import inccl
    from oracle import oracle as O
    dev = torch.device("cuda:0")
    grp = inccl.inccl_group_create(2, rank, "127.0.0.1", port=port)
    comm = inccl.inccl_communicator_create(grp, 0)
    k = 25
    data = {}
    for n in (4096, 16384):
        for which, seed in enumerate((7000, 8000)):
            every, mine = [], None
            for r in range(2):
                g = torch.Generator(device=dev)
                g.manual_seed(seed + r + n)
                xs = [torch.randn(n, generator=g, device=dev) for _ in range(2)]
                every += [x.cpu().numpy() for x in xs]
                if r == rank:
                    mine = xs
            data[(n, which)] = (mine, O.reduce_f32(every, k).view(np.uint32))
    st = torch.cuda.Stream(device=dev)
    outs = {n: torch.empty(n, device=dev) for n in (4096, 16384)}
    torch.cuda.synchronize()
    comm.allreduce_f32(data[(4096, 0)][0], out=outs[4096], scale_exp=k, stream=st.cuda_stream)   # collective setup
    torch.cuda.synchronize()
    lines = []
    for it in range(iters):
        # graph replays at the small size
        xs, _ = data[(4096, 0)]
        out = outs[4096]
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=st):
            for _ in range(20):
                comm.allreduce_f32(xs, out=out, scale_exp=k, stream=st.cuda_stream)
        for _ in range(11):
            gr.replay()
        torch.cuda.synchronize()
        del gr
        # eager calls at the larger size, alternating sets
        out = outs[16384]
        for call, which in enumerate((0, 1, 0, 1)):
            xs, want = data[(16384, which)]
            if fill:
                out.fill_(float("nan"))
                torch.cuda.synchronize()
            comm.allreduce_f32(xs, out=out, scale_exp=k, stream=st.cuda_stream)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            wrong = np.flatnonzero(got != want)
            if wrong.size:
                qs = np.unique(wrong // 4)
                other = data[(16384, 1 - which)][1]
                nan = int(np.count_nonzero(np.isnan(got[wrong].view(np.float32))))
                lines.append(f"iter {it} call {call}: {wrong.size} wrong, quads {int(qs.min())}..{int(qs.max())}, "
                             f"equal to other set {int(np.count_nonzero(got[wrong] == other[wrong]))}, nan {nan}")
    comm.destroy()
    grp.destroy()
    q.put((rank, lines))


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    fill = len(sys.argv) > 2 and sys.argv[2] == "nan"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, port, q, iters, fill)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
    for r, lines in sorted(res):
        print(f"rank {r} ({'nan fill' if fill else 'no fill'}): {len(lines)} wrong calls", flush=True)
        for ln in lines[:12]:
            print("   ", ln, flush=True)


if __name__ == "__main__":
    main()
