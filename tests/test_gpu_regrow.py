"""IPC buffer regrowth (gpu): the p2p and mesh engines allocate their HIP-IPC
buffers collectively and regrow them when a larger bucket arrives
(make-before-break: DESIGN.md "IPC buffer lifecycle").  Three processes on
GPU 0 make the call sequence small -> 256 MiB -> small -> 256 MiB -> 512 MiB
(two regrowths, and small calls running inside the grown buffers), every call
on fresh inputs and every lane checked against the oracle."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SIZES_MIB = [1, 256, 1, 256, 512]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, engine, q):
    try:
        os.environ["INCCL_ENGINE"] = engine
        os.environ["INCCL_DEVICE"] = "0"
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        import sys
        sys.path.insert(0, ROOT)
        import torch
        from container_inc_amd import inccl
        from oracle import oracle as O
        dev = torch.device("cuda:0")
        grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port)
        comm = inccl.inccl_communicator_create(grp, 0)
        assert comm.engine == engine
        results = []
        for call, mib in enumerate(SIZES_MIB):
            n = (mib << 20) // 4 + 7 * call          # ragged: shards differ from call to call
            xs = []
            for r in range(world):                   # every rank's input, regenerated on this GPU
                g = torch.Generator(device=dev)
                g.manual_seed(10_000 * call + r)
                xs.append(torch.randn(n, generator=g, device=dev))
            out = torch.full((n,), float("nan"), device=dev)
            torch.cuda.synchronize()
            comm.allreduce_f32([xs[rank]], out=out, scale_exp=24, stream=comm.stream)
            torch.cuda.synchronize()
            want = O.reduce_f32([x.cpu().numpy() for x in xs], 24)
            results.append((mib, bool(np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32)))))
            del xs, out, want
        comm.destroy()
        grp.destroy()
        q.put((rank, results, None))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("engine", ["p2p", "mesh"])
def test_regrow_small_large_small_large(gpu, engine):
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, engine, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, ok, err = q.get(timeout=280)
            res[r] = (ok, err)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        ok, err = res[r]
        assert err is None, f"rank {r}: {err}"
        assert all(v for _, v in ok), f"rank {r}: {ok}"
