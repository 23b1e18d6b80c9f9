"""Multi-process groups on the GPU (gpu): one process per rank, TCP bootstrap
(api.c:34-144 replacement), the p2p engine (HIP IPC buffers, each rank pulls its
shard from every peer with the fused sum+dequantise kernel, then gathers every
result shard).  On a one-GPU box all ranks share device 0 -- IPC between
processes on one device exercises the same code as across xGMI.  RCCL itself
refuses two ranks on one GPU, so its multi-rank calls are covered by the
world-1 RCCL test and by the identical piece logic over the local transport."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(world, R, n, seed):
    out = []
    for r in range(world):
        rng = np.random.default_rng(seed + r)
        out.append([(rng.standard_normal(n) * 2).astype(np.float32) for _ in range(R)])
    return out


def _rank_main(rank, world, port, cases, q):
    try:
        os.environ["INCCL_ENGINE"] = "p2p"
        os.environ["INCCL_DEVICE"] = "0"
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        import sys
        sys.path.insert(0, ROOT)
        import torch
        from container_inc_amd import inccl
        from oracle import oracle as O
        dev = torch.device("cuda:0")
        grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port)
        assert grp is not None, "group create failed"
        comm = inccl.inccl_communicator_create(grp, 0)
        assert comm is not None and comm.engine == "p2p"
        results = []
        for (R, n, k, seed) in cases:
            xs = _inputs(world, R, n, seed)
            every = [x for per in xs for x in per]
            kk = O.choose_scale(O.absmax(every), world * R) if k == "auto" else k
            want = O.reduce_f32(every, kk)
            srcs = [torch.from_numpy(x).to(dev) for x in xs[rank]]
            out = torch.full((n,), float("nan"), device=dev)
            for _ in range(4):   # repeated: buffer reuse across calls
                comm.allreduce_f32(srcs, out=out, scale_exp=inccl.SCALE_AUTO if k == "auto" else k,
                                   stream=comm.stream)
                torch.cuda.synchronize()
                got = out.cpu().numpy()
                results.append(bool(np.array_equal(got.view(np.uint32), want.view(np.uint32))))
            # back to back with no host synchronisation in between (the bench's timed loop)
            outs = [torch.full((n,), float("nan"), device=dev) for _ in range(12)]
            for o in outs:
                comm.allreduce_f32(srcs, out=o, scale_exp=inccl.SCALE_AUTO if k == "auto" else k,
                                   stream=comm.stream)
            torch.cuda.synchronize()
            for o in outs:
                results.append(bool(np.array_equal(o.cpu().numpy().view(np.uint32), want.view(np.uint32))))
        comm.destroy()
        grp.destroy()
        q.put((rank, results, None))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_p2p_engine_multiprocess(gpu, world):
    cases = [(2, 1 << 20, 25, 11), (1, 100_003, 20, 12), (2, 65_536 * 3 + 5, "auto", 13), (2, 4 << 20, 24, 14)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, cases, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, ok, err = q.get(timeout=240)
            res[r] = (ok, err)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        ok, err = res[r]
        assert err is None, f"rank {r}: {err}"
        assert all(ok), f"rank {r}: {ok}"
