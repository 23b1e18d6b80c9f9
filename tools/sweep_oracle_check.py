"""Debugging aid: bench.py's N>1 size sweep (small buckets, the same engine
order, the same verification and hipGraph replays, the same gloo agreement
calls) with every output ALSO checked against the oracle.  Launch like the
bench:  INCCL_BENCH_SAME_DEVICE=1 torchrun --nproc-per-node 2 tools/sweep_oracle_check.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    import bench
    import container_inc_amd
    from container_inc_amd import inccl
    from oracle import oracle as O
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    os.environ.setdefault("INCCL_LL_TIMEOUT_MS", "2000")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    container_inc_amd.load()
    grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=int(os.environ["MASTER_PORT"]) + 17, device=0)
    comm = inccl.inccl_communicator_create(grp, 0)
    R, k = 2, 25
    bad = []

    def checked(comm_, eng, ch, inputs, out, k_, stream, refs):
        # bench.run_verified, plus a direct host read of `out` beside its clone
        direct = []
        got = []
        for xs in (inputs[0], inputs[1], inputs[0]):
            comm_.allreduce_f32(xs, out=out, scale_exp=k_, chunks=ch, stream=stream.cuda_stream)
            torch.cuda.synchronize()
            got.append(out.clone())
            direct.append(out.cpu().numpy().view(np.uint32).copy())
        if refs is None:
            same = bool(torch.equal(got[0], got[2]))
        else:
            same = all(bool(torch.equal(g_, refs[i_ % 2])) for i_, g_ in enumerate(got))
        n = out.numel()
        for i, which in enumerate((0, 1, 0)):
            dn = int(np.count_nonzero(direct[i] != wants[(n, which)]))
            if dn:
                bad.append(f"{n * 4} B {eng} call {i}: direct host read of out has {dn} wrong lanes")
            every = []
            for r in range(world):
                for seed_x in range(R):
                    pass
            want = wants[(n, which)]
            g = got[i].cpu().numpy().view(np.uint32)
            wrong = np.flatnonzero(g != want)
            if wrong.size:
                qs = np.unique(wrong // 4)
                # what the wrong lanes hold: the result of some mix of the two
                # ranks' partial sums of sets A / B (0 = mine, 1 = the peer's)?
                mixes = []
                for mine_set in (0, 1):
                    for peer_set in (0, 1):
                        cand = mix[(n, mine_set, peer_set)]
                        mixes.append(f"mine={'AB'[mine_set]},peer={'AB'[peer_set]}:"
                                     f"{int(np.count_nonzero(g[wrong] == cand[wrong]))}")
                nan = int(np.count_nonzero(np.isnan(g[wrong].view(np.float32))))
                bad.append(f"{n * 4} B {eng} call {i} (set {'AB'[which]}, clone): {wrong.size} wrong lanes in quads "
                           f"{int(qs.min())}..{int(qs.max())} ({qs.size} quads); lanes equal to {' '.join(mixes)}; "
                           f"nan {nan}")
        return got, same

    wants, mix = {}, {}
    assert world == 2
    for b in bench.SWEEP_BYTES[:5]:
        n = b // 4
        part = {}
        for which, seed in enumerate((7000, 8000)):
            every = []
            for r in range(world):
                gen = torch.Generator(device=dev)
                gen.manual_seed(seed + r)
                xs = [torch.randn(n, generator=gen, device=dev).cpu().numpy() for _ in range(R)]
                every += xs
                part[(r, which)] = O.quant_sum(xs, k)
            wants[(n, which)] = O.reduce_f32(every, k).view(np.uint32)
        for a_ in (0, 1):
            for b_ in (0, 1):
                s_ = O.sum_q32([part[(rank, a_)], part[(1 - rank, b_)]])
                mix[(n, a_, b_)] = O.dequantise(s_, k).view(np.uint32)
    bench.run_verified = checked
    bench.SWEEP_BYTES = bench.SWEEP_BYTES[:5]
    rows = bench.size_sweep(comm, dev, R, k, rank, world)
    for r in rows:
        if rank == 0 and r["ok"]:
            print({key: r[key] for key in ("bucket_bytes", "engine", "bit_identical", "us", "graph_us") if key in r},
                  flush=True)
    print(f"rank {rank}: {len(bad)} wrong outputs", flush=True)
    for ln in bad:
        print(f"rank {rank}:   {ln}", flush=True)
    comm.destroy()
    grp.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
