"""Host logic on CPU: TCP rendezvous of a group (api.c:34-144 replacement) and
the multi-rank reduce-scatter / all-gather decomposition over gloo with
world_size 2 (the oracle computes, gloo exchanges)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _boot_rank(rank, world, port, q):
    os.environ["INCCL_BOOTSTRAP_ONLY"] = "1"
    os.environ["INCCL_BOOT_TIMEOUT"] = "60"
    import sys
    sys.path.insert(0, ROOT)
    from container_inc_amd import inccl
    g = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port)
    if g is None:
        q.put((rank, None))
        return
    q.put((rank, (g.rank, g.world_size, g.transport)))
    g.destroy()


@pytest.mark.parametrize("world", [2, 3])
def test_tcp_rendezvous(lib, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_boot_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert res[r] == (r, world, "rccl"), res


def test_tcp_rendezvous_port_briefly_in_use(lib):
    """Rank 0's port is held by another socket for the first 1.5 s (as a port
    from the ephemeral range can be, as the local end of some connection): the
    bind is retried until the boot deadline and the group still forms."""
    import time
    port = _free_port()
    holder = socket.socket()
    holder.bind(("0.0.0.0", port))
    holder.listen(1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_boot_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    time.sleep(1.5)
    holder.close()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    for r in range(2):
        assert res[r] == (r, 2, "rccl"), res


def test_rendezvous_timeout_returns_null(lib):
    env = dict(os.environ, INCCL_BOOTSTRAP_ONLY="1", INCCL_BOOT_TIMEOUT="1")
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from container_inc_amd import inccl\n"
            "g = inccl.inccl_group_create(2, 1, '127.0.0.1', port=%d)\n"
            "print('NULL' if g is None else 'GROUP')\n") % (ROOT, _free_port())
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=60)
    assert out.stdout.strip() == "NULL"


def test_chunk_plan_covers_bucket():
    from container_inc_amd.plan import chunk_plan, shard_elems
    for n in (1, 63, 64, 1000, 4096, 1 << 20, (1 << 20) + 17):
        for W in (1, 2, 3, 8):
            for chunks in (1, 2, 7):
                plan = chunk_plan(n, W, chunks)
                assert sum(c for _, c, _ in plan) == n
                assert plan[0][0] == 0
                for (o, c, s) in plan:
                    assert s * W >= c and s % 64 == 0 and o % (64 * W) == 0
                    assert s == shard_elems(c, W)


def _gloo_rank(rank, world, port, n, R, k, chunks, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from container_inc_amd.plan import chunk_plan
    from oracle import oracle as O
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    rng = np.random.default_rng(1000 + rank)
    xs = [rng.standard_normal(n).astype(np.float32) for _ in range(R)]
    out = np.empty(n, np.float32)
    for off, cnt, shard in chunk_plan(n, world, chunks):
        total = shard * world
        part = np.zeros(total, np.int32)
        part[:cnt] = O.quant_sum([x[off:off + cnt] for x in xs], k)          # local quant + sum
        gathered = [torch.zeros(total, dtype=torch.int32) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(part))                   # reduce-scatter by exchange
        mine = O.sum_q32([g[rank * shard:(rank + 1) * shard].numpy() for g in gathered])
        deq = O.dequantise(mine, k)                                          # dequantise own shard
        shards = [torch.zeros(shard, dtype=torch.float32) for _ in range(world)]
        dist.all_gather(shards, torch.from_numpy(deq))                       # all-gather
        out[off:off + cnt] = torch.cat(shards).numpy()[:cnt]
    allx = [None] * world
    dist.all_gather_object(allx, [x.tobytes() for x in xs])
    every = [np.frombuffer(b, np.float32) for per in allx for b in per]
    want = O.reduce_f32(every, k)
    q.put((rank, bool(np.array_equal(out.view(np.uint32), want.view(np.uint32)))))
    dist.destroy_process_group()


@pytest.mark.parametrize("n,chunks", [(4096, 1), (10_000 + 3, 3)])
def test_gloo_world2_decomposition(orc, n, chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world, R, k = 2, 2, 25
    ps = [ctx.Process(target=_gloo_rank, args=(r, world, port, n, R, k, chunks, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def _oracle_check_rank(rank, world, port, q):
    import os
    import sys

    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from oracle import oracle as O
    n, R, k = 3000, 2, 25
    xs = [np.random.default_rng(100 * r + j).standard_normal(n).astype(np.float32)
          for r in range(world) for j in range(R)]
    want = O.reduce_f32(xs, k)
    mine = [torch.from_numpy(xs[rank * R + j]) for j in range(R)]
    out = torch.from_numpy(want.copy())
    lanes = bench.oracle_lanes(n, world, 1, 200)
    good = bench.oracle_check(mine, out, lanes, k, rank, world)
    if rank == 1:
        out[lanes[3]] = -out[lanes[3]] + 1.0
    bad = bench.oracle_check(mine, out, lanes, k, rank, world)
    # bf16 buckets: 16-bit patterns, which gloo only gathers widened
    hb = [O.f32_to_bf16(x[:300]) for x in xs]
    wb = O.reduce_bf16(hb, k)
    mb = [torch.from_numpy(hb[rank * R + j].view(np.int16)).view(torch.bfloat16) for j in range(R)]
    ob = torch.from_numpy(wb.view(np.int16).copy()).view(torch.bfloat16)
    gb = bench.oracle_check(mb, ob, bench.oracle_lanes(300, world, 1, 50), k, rank, world, fmt="bf16")
    # reduce-scatter: each rank holds only its shard of the result
    shard = n // world
    rs_out = torch.from_numpy(want[rank * shard:(rank + 1) * shard].copy())
    rs_good = bench.rs_oracle_check(mine, rs_out, lanes, k, rank, world)
    if rank == 1:   # a wrong lane inside rank 1's shard
        inside = [l for l in lanes if shard <= l < 2 * shard][2] - shard
        rs_out[inside] = rs_out[inside] + 1.0
    rs_bad = bench.rs_oracle_check(mine, rs_out, lanes, k, rank, world)
    q.put((rank, good["mismatches"], bad["mismatches"], gb["mismatches"], rs_good["mismatches"],
           rs_bad["mismatches"]))
    dist.destroy_process_group()


def test_bench_oracle_check_gloo_world2():
    """bench.py's N>1 parity check: every rank's inputs and output at the
    sampled lanes are gathered to rank 0 over gloo and checked against the
    oracle's sum over all W*R buckets; a wrong lane on rank 1 is counted."""
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_oracle_check_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((t[0], t[1:]) for t in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(timeout=60)
    # rank 0 reports: clean, one bad lane, clean bf16; reduce-scatter clean, one bad lane in rank 1's shard
    assert res[0] == (0, 1, 0, 0, 1)
    assert res[1] == (None,) * 5           # other ranks only contribute
