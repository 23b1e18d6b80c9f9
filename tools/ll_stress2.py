"""Debugging aid: the bench sweep's verification pattern in a loop -- ll calls
on a side stream alternating two input sets, torch.cuda.synchronize(), a clone
of dst on torch's stream -- then p2p calls on the same buffers, two ranks on
one GPU; every clone AND a direct host read of dst checked against the
oracle.  argv: iterations [rccl] (rccl: also attempt the RCCL engine, which
fails on a shared GPU, before each ll round, as the sweep does).
STRESS_RACE=1: demonstrate the verification race of bench.run_verified before
its fix -- a delayed clone of dst on torch's stream, not waited for, is
overwritten by the next call on the side stream."""
import multiprocessing as mp
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_main(rank, port, q, iters, rccl):
    try:
        _rank_main(rank, port, q, iters, rccl)
    except BaseException as e:  # noqa: BLE001
        q.put((rank, [f"crash: {e!r}"]))


def _rank_main(rank, port, q, iters, rccl):
    os.environ["INCCL_DEVICE"] = "0"
    os.environ["INCCL_LL_TIMEOUT_MS"] = "2000"
    import numpy as np
    import torch
    from container_inc_amd import inccl
    from oracle import oracle as O
    dev = torch.device("cuda:0")
    grp = inccl.inccl_group_create(2, rank, "127.0.0.1", port=port)
    comm = inccl.inccl_communicator_create(grp, 0)
    k, n = 25, int(os.environ.get("STRESS_N", "16384"))
    race = os.environ.get("STRESS_RACE") == "1"
    sets, wants = [], []
    for seed in (7000, 8000):
        every, mine = [], None
        for r in range(2):
            g = torch.Generator(device=dev)
            g.manual_seed(seed + r)
            xs = [torch.randn(n, generator=g, device=dev) for _ in range(2)]
            every += [x.cpu().numpy() for x in xs]
            if r == rank:
                mine = xs
        sets.append(mine)
        wants.append(O.reduce_f32(every, k).view(np.uint32))
    out = torch.empty(n, device=dev)
    lines = []
    for it in range(iters):
        st = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()
        if rccl:
            comm.set_engine("rccl")
            try:
                comm.allreduce_f32(sets[0], out=out, scale_exp=k, stream=st.cuda_stream)
            except Exception:  # noqa: BLE001
                pass
        for eng in ("ll", "p2p"):
            comm.set_engine(eng)
            if race:
                # the round-2 bench bug, made deterministic: the clone on torch's
                # stream is delayed and NOT waited for before the next call on st
                clones = []
                for which in (0, 1, 0):
                    comm.allreduce_f32(sets[which], out=out, scale_exp=k, stream=st.cuda_stream)
                    torch.cuda.synchronize()
                    torch.cuda._sleep(20_000_000)
                    clones.append(out.clone())
                torch.cuda.synchronize()
                for call, (which, c) in enumerate(zip((0, 1, 0), clones)):
                    cl = c.cpu().numpy().view(np.uint32)
                    wrong = np.flatnonzero(cl != wants[which])
                    if wrong.size:
                        other = int(np.count_nonzero(cl[wrong] == wants[1 - which][wrong]))
                        lines.append(f"iter {it} {eng} call {call} (racing clone): {wrong.size} wrong, "
                                     f"{other} = the next call's set")
                continue
            for call, which in enumerate((0, 1, 0)):
                comm.allreduce_f32(sets[which], out=out, scale_exp=k, stream=st.cuda_stream)
                torch.cuda.synchronize()
                c = out.clone()
                direct = out.cpu().numpy().view(np.uint32)
                cl = c.cpu().numpy().view(np.uint32)
                bc, bd = int(np.count_nonzero(cl != wants[which])), int(np.count_nonzero(direct != wants[which]))
                if bc or bd:
                    wrong = np.flatnonzero(cl != wants[which])
                    other = int(np.count_nonzero(cl[wrong] == wants[1 - which][wrong])) if wrong.size else 0
                    lines.append(f"iter {it} {eng} call {call}: clone {bc} wrong ({other} = other set), direct {bd}")
    comm.destroy()
    grp.destroy()
    q.put((rank, lines))


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    rccl = len(sys.argv) > 2 and sys.argv[2] == "rccl"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, port, q, iters, rccl)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=170) for _ in range(2)]
    for p in ps:
        p.join(timeout=30)
    for r, lines in sorted(res):
        print(f"rank {r}: {len(lines)} wrong", flush=True)
        for ln in lines[:10]:
            print("   ", ln, flush=True)


if __name__ == "__main__":
    main()
