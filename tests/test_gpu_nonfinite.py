"""Non-finite gradients under INCCL_NONFINITE_NAN (gpu): the absmax kernels'
flag word (INCCL_ABSMAX_FLAG_NONFINITE) against the oracle's restatement, and
every route of an auto-scaled allreduce -- the fused world-1 kernel, the
reduce-scatter / all-gather path (local transport and RCCL at world 1), the
IPC engines' host-agreed scale (p2p, mesh, ll; one process per rank) -- for
fp32, bf16 and fp16 buckets: a NaN or +-Inf anywhere makes every result NaN on
every rank, and finite buckets keep the oracle's bit-exact result (the mode
changes nothing else, and the flag does not stick to the next call)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from conftest import ROOT
from test_gpu_comm import _run_ranks

pytestmark = pytest.mark.gpu

KINDS = ("f32", "bf16", "f16")


def _bucket(rng, n, kind):
    x = rng.standard_normal(n).astype(np.float32) * 2.0
    if kind == "f32":
        return x
    if kind == "bf16":
        return (x.view(np.uint32) >> 16).astype(np.uint16)
    return x.astype(np.float16).view(np.uint16)


def _poison(h, kind, where, what):
    """h with element `where` set to NaN / +Inf / -Inf"""
    h = h.copy()
    val = {"nan": np.float32(np.nan), "inf": np.float32(np.inf), "-inf": np.float32(-np.inf)}[what]
    if kind == "f32":
        h[where] = val
    elif kind == "bf16":
        h[where] = np.uint16(np.array([val], np.float32).view(np.uint32)[0] >> 16)
    else:
        h[where] = np.array([val], np.float16).view(np.uint16)[0]
    return h


def _dev(h, dev, kind):
    import torch
    if kind == "f32":
        return torch.from_numpy(h).to(dev)
    t = torch.from_numpy(h.view(np.int16)).to(dev)
    return t.view(torch.bfloat16 if kind == "bf16" else torch.float16)


def _host(t, kind):
    import torch
    if kind == "f32":
        return t.cpu().numpy()
    return t.view(torch.int16).cpu().numpy().view(np.uint16)


def _isnan(h, kind):
    from oracle import oracle as O
    return np.isnan(O.widened_bits(h, kind).view(np.float32))


def _want(orc, every, kind, W_R):
    k = orc.choose_scale({"f32": orc.absmax, "bf16": orc.absmax_bf16, "f16": orc.absmax_f16}[kind](every), W_R)
    return {"f32": orc.reduce_f32, "bf16": orc.reduce_bf16, "f16": orc.reduce_f16}[kind](every, k)


def _allreduce(comm, kind, srcs, out):
    from container_inc_amd import inccl
    fn = {"f32": comm.allreduce_f32, "bf16": comm.allreduce_bf16, "f16": comm.allreduce_f16}[kind]
    fn(srcs, out=out, scale_exp=inccl.SCALE_AUTO, stream=comm.stream)


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("what", ["none", "inf", "-inf", "nan"])
def test_absmax_flag_word(gpu, orc, kind, what):
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(len(kind) * 7 + len(what))
    n = 100_003
    hs = [_bucket(rng, n, kind) for _ in range(2)]
    if what != "none":
        hs[1] = _poison(hs[1], kind, 77_777, what)
    srcs = [_dev(h, gpu, kind) for h in hs]
    torch.cuda.synchronize()
    plain = inccl.absmax_bits(srcs)
    flagged = inccl.absmax_bits(srcs, nonfinite_flag=True)
    want = orc.absmax_word_flagged(hs, kind)
    assert (flagged >> 31) == (what != "none")
    if what != "nan":   # (a NaN's payload bits may widen differently; bit 31 is the contract)
        assert flagged == want
    if what == "none":
        assert flagged == plain


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("world", [1, 3])
def test_nonfinite_local(gpu, orc, kind, world):
    """world 1: the fused kernel; world 3: reduce-scatter -> dequantise -> all-gather."""
    import torch
    from container_inc_amd import inccl
    n, R = 65_541, 2
    rng = np.random.default_rng(world * 31 + len(kind))
    hs = [[_bucket(rng, n, kind) for _ in range(R)] for _ in range(world)]
    bad = [[h.copy() for h in per] for per in hs]
    bad[world - 1][1] = _poison(bad[world - 1][1], kind, n - 3, "nan" if kind != "bf16" else "-inf")
    want = _want(orc, [h for per in hs for h in per], kind, world * R)
    hub = f"nonfinite-{kind}-{world}"

    def rank(r):
        grp = inccl.inccl_group_create_local(world, r, hub)
        comm = inccl.inccl_communicator_create(grp, 0)
        comm.set_nonfinite(True)
        good_in = [_dev(h, gpu, kind) for h in hs[r]]
        bad_in = [_dev(h, gpu, kind) for h in bad[r]]
        out = torch.empty_like(good_in[0])
        res = []
        for ins in (good_in, bad_in, good_in):   # the flag must not stick to the next call
            _allreduce(comm, kind, ins, out)
            torch.cuda.synchronize()
            res.append(_host(out, kind))
        rs = comm.reduce_scatter(bad_in, stream=comm.stream)   # the reduce-scatter's shard alike
        torch.cuda.synchronize()
        res.append(_host(rs, kind))
        comm.set_nonfinite(False)   # the quantiser's spec again: finite, whatever the input
        _allreduce(comm, kind, bad_in, out)
        torch.cuda.synchronize()
        res.append(_host(out, kind))
        comm.barrier()
        comm.destroy()
        grp.destroy()
        return res

    assert n % world == 0
    for good, poisoned, again, rs, spec in _run_ranks(world, rank):
        np.testing.assert_array_equal(good, want)
        assert _isnan(poisoned, kind).all()
        assert rs.size == n // world and _isnan(rs, kind).all()
        np.testing.assert_array_equal(again, want)
        assert not _isnan(spec, kind).any()


def test_nonfinite_rccl_world1(gpu, orc, monkeypatch):
    """RCCL transport at world 1 through the sharded path (real RCCL calls)."""
    import torch
    from container_inc_amd import inccl
    monkeypatch.setenv("INCCL_FORCE_RCCL", "1")
    monkeypatch.setenv("INCCL_FORCE_SHARDED", "1")
    monkeypatch.setenv("INCCL_MASTER_PORT", "0")
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    assert grp.transport == "rccl"
    comm.set_nonfinite(True)
    rng = np.random.default_rng(5)
    for kind in KINDS:
        hs = [_bucket(rng, 40_000, kind) for _ in range(2)]
        want = _want(orc, hs, kind, 2)
        for eng in ("rccl", "ar", "a2a"):
            comm.set_engine(eng)
            out = torch.empty_like(_dev(hs[0], gpu, kind))
            _allreduce(comm, kind, [_dev(h, gpu, kind) for h in hs], out)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(_host(out, kind), want, err_msg=f"{kind} {eng}")
            bad = [hs[0], _poison(hs[1], kind, 3, "inf")]
            _allreduce(comm, kind, [_dev(h, gpu, kind) for h in bad], out)
            torch.cuda.synchronize()
            assert _isnan(_host(out, kind), kind).all(), f"{kind} {eng}"
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
        comm.set_nonfinite(True)
        ok = []
        n = 50_000 if engine == "ll" else 300_001
        for kind in KINDS:
            hs = [_bucket(np.random.default_rng(100 + r), n, kind) for r in range(world)]
            want = _want(O, hs, kind, world)
            bad = [h.copy() for h in hs]
            bad[world - 1] = _poison(bad[world - 1], kind, n // 2, "nan" if kind == "f32" else "inf")
            out = torch.empty_like(_dev(hs[rank], dev, kind))
            for ins, expect in ((hs, "want"), (bad, "nan"), (hs, "want")):
                _allreduce(comm, kind, [_dev(ins[rank], dev, kind)], out)
                torch.cuda.synchronize()
                got = _host(out, kind)
                ok.append(bool(np.array_equal(got, want)) if expect == "want" else bool(_isnan(got, kind).all()))
        comm.destroy()
        grp.destroy()
        q.put((rank, ok, None))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("world,engine", [(2, "p2p"), (3, "mesh"), (2, "meshw"), (2, "ll")])
def test_nonfinite_ipc_multiprocess(gpu, world, engine):
    """The IPC engines agree the scale on the host; a flagged max goes back to
    the device so every rank's kernels write NaN.  One process per rank."""
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
