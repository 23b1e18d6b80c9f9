"""IEEE fp16 buckets on the GPU (gpu): the k_stream16 kernels with F16
(F16->F16, F16->Q32, Q32->F16), the fp16 absmax, and inccl_allreduce_f16 over
the in-process transport (reduce-scatter int32 + 2-byte all-gather), RCCL at
world 1, and the IPC engines with one process per rank (p2p / mesh / meshw:
2-byte result exchange; ll: int32 exchange), plain and prepared -- all
bit-exact against the oracle's fp16 restatement (tests/test_oracle_f16.py pins
it to numpy's IEEE binary16)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from conftest import ROOT
from test_gpu_comm import _run_ranks

pytestmark = pytest.mark.gpu


def _f16(rng, n, scale=2.0):
    return (rng.standard_normal(n) * scale).astype(np.float16).view(np.uint16)


def _dev(h, dev, shift=0):
    """uint16 bit patterns -> an fp16 CUDA tensor, optionally `shift` elements past a 16-B boundary."""
    import torch
    t = torch.from_numpy(np.concatenate([np.zeros(shift, np.uint16), h]).view(np.int16)).to(dev)
    return t.view(torch.float16)[shift:]


def _host(t):
    import torch
    return t.view(torch.int16).cpu().numpy().view(np.uint16)


@pytest.mark.parametrize("R,n,k,shift", [(1, 8, 20, 0), (2, 1000, 22, 0), (2, 1 << 20, 25, 0),
                                         (3, (1 << 20) + 13, "auto", 0), (8, 3_000_001, "auto", 0),
                                         (2, 100_003, 24, 1), (3, 40_000, 40, 0), (2, 4099, 40, 1),
                                         (3, 50_001, "auto", 3), (2, 70_001, 30, 0), (2, 70_001, 2, 0)])
def test_reduce_f16_kernel(gpu, orc, R, n, k, shift):
    """k = 40 saturates most lanes and wraps their sums (the dequantised sums then
    reach the fp16 subnormal range); k = 30 puts many results there; k = 2 makes
    sums past 65504, which narrow to +-Inf."""
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(R * 1000 + n % 997 + (k if isinstance(k, int) else 0))
    hs = [_f16(rng, n, scale=2.0 if k != 2 else 30000.0) for _ in range(R)]
    hs[0][: min(n, 4)] = [0x7E00, 0xFC00, 0x7C00, 0x0001][: min(n, 4)]   # NaN -> 0, -Inf / +Inf, a subnormal
    kk = orc.choose_scale(orc.absmax_f16(hs), R) if k == "auto" else k
    want = orc.reduce_f16(hs, kk)
    srcs = [_dev(h, gpu, shift) for h in hs]
    out = _dev(np.full(n, 0x7E00, np.uint16), gpu, shift)
    torch.cuda.synchronize()
    inccl.reduce_f16(srcs, kk, out=out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(out), want)
    if k == "auto":
        assert inccl.absmax_f16(srcs) == orc.absmax_f16(hs)
    if k == 2:
        assert (want == 0x7C00).any() and (want == 0xFC00).any()


@pytest.mark.parametrize("n", [64, 1 << 16, 777_777])
def test_f16_kinds(gpu, orc, n):
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(n)
    hs = [_f16(rng, n) for _ in range(3)]
    q = inccl.stream_op(inccl.KIND_F16, inccl.KIND_Q32, [_dev(h, gpu) for h in hs], scale_exp=23)
    torch.cuda.synchronize()
    want_q = orc.quant_sum_f16(hs, 23)
    np.testing.assert_array_equal(q.cpu().numpy(), want_q)
    qs = [q, q.clone()]
    y = inccl.stream_op(inccl.KIND_Q32, inccl.KIND_F16, qs, scale_exp=23)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(y), orc.sum_dequant_f16([want_q, want_q], 23))


@pytest.mark.parametrize("world,R,n,k", [(1, 2, (1 << 18) + 5, "auto"), (2, 2, 1 << 20, 25), (3, 1, 100_001, "auto"),
                                         (8, 1, 65_536, "auto")])
def test_allreduce_f16_local(gpu, orc, world, R, n, k):
    """world 1: the fused kernel, in place; world > 1: reduce-scatter (int32) ->
    dequantise own shard to fp16 -> all-gather (2 bytes)."""
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(world * 10 + R + 7)
    hs = [[_f16(rng, n) for _ in range(R)] for _ in range(world)]
    every = [h for per in hs for h in per]
    kk = orc.choose_scale(orc.absmax_f16(every), world * R) if k == "auto" else k
    want = orc.reduce_f16(every, kk)
    dev_in = [[_dev(h, gpu) for h in per] for per in hs]
    torch.cuda.synchronize()
    hub = f"f16-{world}-{R}-{n}"

    def rank(r):
        grp = inccl.inccl_group_create_local(world, r, hub)
        comm = inccl.inccl_communicator_create(grp, 0)
        out = torch.empty(n, dtype=torch.float16, device=gpu)
        res = []
        for _ in range(2):   # buffer reuse
            comm.allreduce_f16(dev_in[r], out=out, scale_exp=inccl.SCALE_AUTO if k == "auto" else k,
                               stream=comm.stream)
            torch.cuda.synchronize()
            res.append(_host(out))
        if world == 1:   # in place, dst = srcs[0]
            comm.allreduce_f16(dev_in[r], out=dev_in[r][0], scale_exp=inccl.SCALE_AUTO if k == "auto" else k,
                               stream=comm.stream)
            torch.cuda.synchronize()
            res.append(_host(dev_in[r][0]))
        comm.barrier()
        comm.destroy()
        grp.destroy()
        return res

    for res in _run_ranks(world, rank):
        for got in res:
            np.testing.assert_array_equal(got, want)


def test_allreduce_f16_rccl_world1(gpu, orc, monkeypatch):
    """RCCL transport at world 1 through the sharded path: ncclReduceScatter and
    the 2-byte ncclAllGather are real RCCL calls on a one-rank communicator."""
    import torch
    from container_inc_amd import inccl
    monkeypatch.setenv("INCCL_FORCE_RCCL", "1")
    monkeypatch.setenv("INCCL_FORCE_SHARDED", "1")
    monkeypatch.setenv("INCCL_MASTER_PORT", "0")
    rng = np.random.default_rng(19)
    n = (1 << 20) + 7
    hs = [_f16(rng, n) for _ in range(2)]
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    assert grp.transport == "rccl"
    out = torch.empty(n, dtype=torch.float16, device=gpu)
    srcs = [_dev(h, gpu) for h in hs]
    torch.cuda.synchronize()
    for eng in ("rccl", "ar", "a2a"):
        comm.set_engine(eng)
        out.fill_(float("nan"))
        torch.cuda.synchronize()
        comm.allreduce_f16(srcs, out=out, scale_exp=24, stream=comm.stream)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_host(out), orc.reduce_f16(hs, 24), err_msg=eng)
    comm.destroy()
    grp.destroy()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ipc_rank(rank, world, port, q, engine):
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
                rng = np.random.default_rng(seed * 100 + r + 5)
                hs.append([_f16(rng, n) for _ in range(R)])
            every = [h for per in hs for h in per]
            kk = O.choose_scale(O.absmax_f16(every), world * R) if k == "auto" else k
            want = O.reduce_f16(every, kk)
            srcs = [_dev(h, dev) for h in hs[rank]]
            out = torch.empty(n, dtype=torch.float16, device=dev)
            torch.cuda.synchronize()
            comm.allreduce_f16(srcs, out=out, scale_exp=inccl.SCALE_AUTO if k == "auto" else k, stream=comm.stream)
            torch.cuda.synchronize()
            ok.append(bool(np.array_equal(_host(out), want)))
            odd = torch.empty(n + 1, dtype=torch.float16, device=dev)[1:]   # 2-B aligned: the int32-allreduce path
            torch.cuda.synchronize()
            comm.allreduce_f16(srcs, out=odd, scale_exp=inccl.SCALE_AUTO if k == "auto" else k, stream=comm.stream)
            torch.cuda.synchronize()
            ok.append(bool(np.array_equal(_host(odd), want)))
            comm.allreduce_f16(srcs, out=srcs[0], scale_exp=inccl.SCALE_AUTO if k == "auto" else k,
                               stream=comm.stream)   # in place
            torch.cuda.synchronize()
            ok.append(bool(np.array_equal(_host(srcs[0]), want)))
            if k != "auto":   # prepared (inccl_op_create_allreduce16), run twice on fresh inputs
                srcs = [_dev(h, dev) for h in hs[rank]]
                out.fill_(float("nan"))
                torch.cuda.synchronize()   # inputs and out made on torch's stream; op() runs on comm.stream
                op = comm.prepare_allreduce_f16(srcs, out=out, scale_exp=k, stream=comm.stream)
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


@pytest.mark.parametrize("world,engine", [(2, "p2p"), (3, "p2p"), (2, "mesh"), (3, "mesh"), (4, "meshw"), (2, "ll")])
def test_allreduce_f16_ipc_multiprocess(gpu, world, engine):
    """The IPC engines with fp16 buckets, one process per rank on GPU 0: p2p,
    mesh and meshw narrow to fp16 in their reduce kernel and exchange 2-byte
    results; ll runs its int32 allreduce and dequantises to fp16 after it."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ipc_rank, args=(r, world, port, q, engine)) for r in range(world)]
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
