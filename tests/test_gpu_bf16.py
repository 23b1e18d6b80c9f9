"""bfloat16 buckets on the GPU (gpu): the k_stream16 kernels (BF16->BF16,
BF16->Q32, Q32->BF16), the bf16 absmax, and inccl_allreduce_bf16 over the
in-process transport (reduce-scatter int32 + all-gather bf16), RCCL at world 1
and the p2p engine with one process per rank -- all bit-exact against the
oracle's bf16 restatement (tests/test_oracle_bf16.py pins it)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from conftest import ROOT
from test_gpu_comm import _run_ranks

pytestmark = pytest.mark.gpu


def _bf16(rng, n, scale=2.0):
    import torch
    x = (rng.standard_normal(n) * scale).astype(np.float32)
    return torch.from_numpy(x).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)


def _dev(h, dev, shift=0):
    """uint16 bit patterns -> a bf16 CUDA tensor, optionally `shift` elements past a 16-B boundary."""
    import torch
    t = torch.from_numpy(np.concatenate([np.zeros(shift, np.uint16), h]).view(np.int16)).to(dev)
    return t.view(torch.bfloat16)[shift:]


def _host(t):
    import torch
    return t.view(torch.int16).cpu().numpy().view(np.uint16)


@pytest.mark.parametrize("R,n,k,shift", [(1, 8, 20, 0), (2, 1000, 22, 0), (2, 1 << 20, 25, 0),
                                         (3, (1 << 20) + 13, "auto", 0), (8, 3_000_001, "auto", 0),
                                         (2, 100_003, 24, 1), (3, 40_000, 40, 0), (2, 4099, 40, 1),
                                         (3, 50_001, "auto", 3)])
def test_reduce_bf16_kernel(gpu, orc, R, n, k, shift):
    """k = 40 saturates most lanes (|x| * 2^40 > 2^31) and wraps their sums."""
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(R * 1000 + n % 997)
    hs = [_bf16(rng, n) for _ in range(R)]
    hs[0][: min(n, 3)] = [0x7FC0, 0xFF80, 0x7F80][: min(n, 3)]   # NaN -> 0, -Inf / +Inf saturate
    kk = orc.choose_scale(orc.absmax_bf16(hs), R) if k == "auto" else k
    want = orc.reduce_bf16(hs, kk)
    srcs = [_dev(h, gpu, shift) for h in hs]
    out = _dev(np.full(n, 0x7FC0, np.uint16), gpu, shift)
    torch.cuda.synchronize()
    inccl.reduce_bf16(srcs, kk, out=out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(out), want)
    if k == "auto":
        assert inccl.absmax_bf16(srcs) == orc.absmax_bf16(hs)


@pytest.mark.parametrize("n", [64, 1 << 16, 777_777])
def test_bf16_kinds(gpu, orc, n):
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(n)
    hs = [_bf16(rng, n) for _ in range(3)]
    q = inccl.stream_op(inccl.KIND_BF16, inccl.KIND_Q32, [_dev(h, gpu) for h in hs], scale_exp=23)
    torch.cuda.synchronize()
    want_q = orc.quant_sum_bf16(hs, 23)
    np.testing.assert_array_equal(q.cpu().numpy(), want_q)
    qs = [q, q.clone()]
    y = inccl.stream_op(inccl.KIND_Q32, inccl.KIND_BF16, qs, scale_exp=23)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(y), orc.sum_dequant_bf16([want_q, want_q], 23))


def test_allreduce_bf16_dst_aliases_src(gpu, orc):
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(5)
    n = (1 << 18) + 5
    hs = [_bf16(rng, n) for _ in range(2)]
    grp = inccl.inccl_group_create_local(1, 0, "bf16-alias")
    comm = inccl.inccl_communicator_create(grp, 0)
    srcs = [_dev(h, gpu) for h in hs]
    torch.cuda.synchronize()
    comm.allreduce_bf16(srcs, out=srcs[0], scale_exp=inccl.SCALE_AUTO, stream=comm.stream)
    torch.cuda.synchronize()
    kk = orc.choose_scale(orc.absmax_bf16(hs), 2)
    np.testing.assert_array_equal(_host(srcs[0]), orc.reduce_bf16(hs, kk))
    comm.destroy()
    grp.destroy()


@pytest.mark.parametrize("world,R,n,k", [(2, 2, 1 << 20, 25), (3, 1, 100_001, "auto"), (4, 2, (1 << 18) + 3, 22),
                                         (8, 1, 65_536, "auto")])
def test_allreduce_bf16_local(gpu, orc, world, R, n, k):
    """reduce-scatter (int32) -> dequantise own shard to bf16 -> all-gather (bf16)."""
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(world * 10 + R)
    hs = [[_bf16(rng, n) for _ in range(R)] for _ in range(world)]
    every = [h for per in hs for h in per]
    kk = orc.choose_scale(orc.absmax_bf16(every), world * R) if k == "auto" else k
    want = orc.reduce_bf16(every, kk)
    dev_in = [[_dev(h, gpu) for h in per] for per in hs]
    torch.cuda.synchronize()
    hub = f"bf16-{world}-{R}-{n}"

    def rank(r):
        grp = inccl.inccl_group_create_local(world, r, hub)
        comm = inccl.inccl_communicator_create(grp, 0)
        out = torch.empty(n, dtype=torch.bfloat16, device=gpu)
        res = []
        for _ in range(2):   # buffer reuse
            comm.allreduce_bf16(dev_in[r], out=out, scale_exp=inccl.SCALE_AUTO if k == "auto" else k,
                                stream=comm.stream)
            torch.cuda.synchronize()
            res.append(_host(out))
        comm.barrier()
        comm.destroy()
        grp.destroy()
        return res

    for res in _run_ranks(world, rank):
        for got in res:
            np.testing.assert_array_equal(got, want)


def test_allreduce_bf16_rccl_world1(gpu, orc, monkeypatch):
    """RCCL transport at world 1 through the sharded path: ncclReduceScatter and
    the bf16 ncclAllGather are real RCCL calls on a one-rank communicator."""
    import torch
    from container_inc_amd import inccl
    monkeypatch.setenv("INCCL_FORCE_RCCL", "1")
    monkeypatch.setenv("INCCL_FORCE_SHARDED", "1")
    monkeypatch.setenv("INCCL_MASTER_PORT", "0")
    rng = np.random.default_rng(9)
    n = (1 << 20) + 7
    hs = [_bf16(rng, n) for _ in range(2)]
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    assert grp.transport == "rccl"
    out = torch.empty(n, dtype=torch.bfloat16, device=gpu)
    srcs = [_dev(h, gpu) for h in hs]
    torch.cuda.synchronize()
    for eng in ("rccl", "ar"):
        comm.set_engine(eng)
        out.fill_(float("nan"))
        torch.cuda.synchronize()
        comm.allreduce_bf16(srcs, out=out, scale_exp=24, stream=comm.stream)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_host(out), orc.reduce_bf16(hs, 24), err_msg=eng)
    comm.destroy()
    grp.destroy()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _p2p_rank(rank, world, port, q, engine="p2p"):
    try:
        os.environ["INCCL_ENGINE"] = engine
        os.environ["INCCL_DEVICE"] = "0"
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        import sys
        sys.path.insert(0, ROOT)
        import torch
        from container_inc_amd import inccl
        from oracle import oracle as O
        dev = torch.device("cuda", 0)
        grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port, device=0)
        comm = inccl.inccl_communicator_create(grp, 0)
        ok = []
        for R, n, k, seed in ((2, 1 << 20, 25, 1), (1, 300_001, "auto", 2), (2, 4099, 23, 3)):
            hs = []
            for r in range(world):
                rng = np.random.default_rng(seed * 100 + r)
                hs.append([_bf16(rng, n) for _ in range(R)])
            every = [h for per in hs for h in per]
            kk = O.choose_scale(O.absmax_bf16(every), world * R) if k == "auto" else k
            want = O.reduce_bf16(every, kk)
            srcs = [_dev(h, dev) for h in hs[rank]]
            out = torch.empty(n, dtype=torch.bfloat16, device=dev)
            torch.cuda.synchronize()
            comm.allreduce_bf16(srcs, out=out, scale_exp=inccl.SCALE_AUTO if k == "auto" else k, stream=comm.stream)
            torch.cuda.synchronize()
            ok.append(bool(np.array_equal(_host(out), want)))
            odd = torch.empty(n + 1, dtype=torch.bfloat16, device=dev)[1:]   # 2-B aligned: the int32-allreduce path
            torch.cuda.synchronize()
            comm.allreduce_bf16(srcs, out=odd, scale_exp=inccl.SCALE_AUTO if k == "auto" else k, stream=comm.stream)
            torch.cuda.synchronize()
            ok.append(bool(np.array_equal(_host(odd), want)))
            comm.allreduce_bf16(srcs, out=srcs[0], scale_exp=inccl.SCALE_AUTO if k == "auto" else k,
                                stream=comm.stream)   # in place
            torch.cuda.synchronize()
            ok.append(bool(np.array_equal(_host(srcs[0]), want)))
            if k != "auto":   # prepared (inccl_op_create_allreduce16), run twice on fresh inputs
                srcs = [_dev(h, dev) for h in hs[rank]]
                out.fill_(float("nan"))
                torch.cuda.synchronize()   # inputs and out made on torch's stream; op() runs on comm.stream
                op = comm.prepare_allreduce_bf16(srcs, out=out, scale_exp=k, stream=comm.stream)
                for _ in range(2):
                    op()
                    torch.cuda.synchronize()
                    ok.append(bool(np.array_equal(_host(out), want)))
                op.destroy()
        comm.destroy()
        grp.destroy()
        q.put((rank, ok, None))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("world,engine", [(2, "p2p"), (3, "p2p"), (8, "p2p"), (2, "mesh"), (3, "mesh"), (4, "meshw"),
                                          (8, "mesh")])
def test_allreduce_bf16_p2p_multiprocess(gpu, world, engine):
    """The IPC engines' bf16 paths: p2p (bf16 result shards gathered, odd element
    counts through the gather's 2-byte tail; a 2-byte-aligned dst takes the int32
    allreduce) and mesh / meshw (the persistent kernel with bf16 sources and
    results, any dst alignment), each also in place."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_p2p_rank, args=(r, world, port, q, engine)) for r in range(world)]
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


@pytest.mark.parametrize("engine,average", [("rccl", False), ("ar", True)])
def test_allreduce_bf16_graph_capture_world1(gpu, orc, monkeypatch, engine, average):
    """inccl_allreduce_bf16 captured into a hipGraph on the RCCL engines (world 1,
    sharded path forced): three captured calls replayed with fresh inputs,
    bit-exact vs the oracle (set_average at world 1 is the identity)."""
    import torch
    from container_inc_amd import inccl
    monkeypatch.setenv("INCCL_FORCE_RCCL", "1")
    monkeypatch.setenv("INCCL_FORCE_SHARDED", "1")
    monkeypatch.setenv("INCCL_MASTER_PORT", "0")
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    comm.set_engine(engine)
    comm.set_average(average)
    n = (1 << 18) + 64
    bufs = [torch.empty(n, device=gpu, dtype=torch.bfloat16) for _ in range(2)]
    outs = [torch.empty(n, device=gpu, dtype=torch.bfloat16) for _ in range(3)]
    st = torch.cuda.Stream(device=gpu)
    comm.allreduce_bf16(bufs, out=outs[0], scale_exp=24, stream=st.cuda_stream)   # workspaces sized eagerly
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=st):
        for o in outs:
            comm.allreduce_bf16(bufs, out=o, scale_exp=24, stream=st.cuda_stream)
    rng = np.random.default_rng(78)
    for _ in range(3):
        hs = [_bf16(rng, n) for _ in range(2)]
        for b, h in zip(bufs, hs):
            b.copy_(_dev(h, gpu))
        for o in outs:
            o.fill_(float("nan"))
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        want = orc.reduce_bf16(hs, 24)
        for o in outs:
            np.testing.assert_array_equal(_host(o), want)
    del graph
    comm.destroy()
    grp.destroy()
