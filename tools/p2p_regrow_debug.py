"""Multi-process IPC engine on ONE GPU, W ranks, replaying the GPU test's call
pattern (tests/test_gpu_p2p.py P2P_CASES: repeated calls alternating two
streams, then 12 back-to-back calls) and reporting, per call, which result
shards of dst differ from the oracle -- so a stale peer mapping (one rank wrong
on shard j) is told apart from a wrong reduction (every rank wrong on shard j).
A debugging aid.

    python tools/p2p_regrow_debug.py [W] [engine]
"""
import multiprocessing as mp
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _rank(rank, world, port, engine, q):
    try:
        os.environ["INCCL_ENGINE"] = engine
        os.environ["INCCL_LL_MAX_BYTES"] = "0"
        os.environ["INCCL_DEVICE"] = "0"
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        import numpy as np
        import torch
        import test_gpu_p2p as T
        from container_inc_amd import inccl
        from oracle import oracle as O
        dev = torch.device("cuda:0")
        grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port)
        comm = inccl.inccl_communicator_create(grp, 0)
        side = torch.cuda.Stream(device=dev)
        lines = []
        for case in T.P2P_CASES:
            R, n, k, seed = case[:4]
            shift = case[4] if len(case) > 4 else 0
            xs = T._inputs(world, R, n, seed)
            every = [x for per in xs for x in per]
            kk = O.choose_scale(O.absmax(every), world * R) if k == "auto" else k
            want = O.reduce_f32(every, kk).view(np.uint32)
            shard = (((n + world - 1) // world) + 63) // 64 * 64
            srcs = [torch.from_numpy(np.concatenate([np.zeros(shift, np.float32), x])).to(dev)[shift:]
                    for x in xs[rank]]
            kx = inccl.SCALE_AUTO if k == "auto" else k

            def report(tag, out):
                got = out.cpu().numpy().view(np.uint32)
                bad = [j for j in range(world)
                       if not np.array_equal(got[j * shard:(j + 1) * shard], want[j * shard:(j + 1) * shard])]
                if bad:
                    nan = [j for j in bad if np.isnan(got[j * shard:(j + 1) * shard].view(np.float32)).any()]
                    lines.append(f"case n={n} R={R} k={k} {tag}: bad_shards={bad} nan={nan}")

            out = torch.full((n + shift,), float("nan"), device=dev)[shift:]
            torch.cuda.synchronize()
            for it in range(4):
                comm.allreduce_f32(srcs, out=out, scale_exp=kx, stream=comm.stream if it % 2 == 0 else side.cuda_stream)
                torch.cuda.synchronize()
                report(f"it={it}", out)
            outs = [torch.full((n + shift,), float("nan"), device=dev)[shift:] for _ in range(12)]
            torch.cuda.synchronize()
            for o in outs:
                comm.allreduce_f32(srcs, out=o, scale_exp=kx, stream=comm.stream)
            torch.cuda.synchronize()
            for i, o in enumerate(outs):
                report(f"b2b={i}", o)
        comm.destroy()
        grp.destroy()
        q.put((rank, lines, None))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    engine = sys.argv[2] if len(sys.argv) > 2 else "p2p"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, port, engine, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, lines, err = q.get(timeout=300)
            res[r] = (lines, err)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    bad = 0
    for r in sorted(res):
        lines, err = res[r]
        print(f"rank {r}: err={err} wrong_calls={len(lines or [])}")
        bad += (err is not None) + len(lines or [])
        for ln in (lines or [])[:20]:
            print("   ", ln)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
