"""DDP comm hook (container_inc_amd/ddp.py) on CPU: world 2 over gloo with the
engine's contract restated by the oracle (tests/_ddp_rank.py GlooStandIn), so
the hook's plumbing -- several buckets, in-place result, averaging, the
completed future DDP copies back into ``.grad`` -- is tested without a GPU.
The same worker runs against the real library in tests/test_gpu_ddp.py."""
import multiprocessing as mp
import socket

import pytest


def _free_ports(n):
    """n distinct free ports, all held until every one is chosen.  (The GPU
    variant once derived the bootstrap's port as gloo's + 1, unchecked: gloo's
    own peer sockets sit in the same ephemeral range, and one took it.)"""
    socks = []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
    ports = [s.getsockname()[1] for s in socks]
    for s in socks:
        s.close()
    return ports


def run_world(world, mode, timeout, dtype="f32", as_view=False, engine="p2p", poison=None):
    import _ddp_rank
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port, boot_port = _free_ports(2)
    ps = [ctx.Process(target=_ddp_rank.run, args=(r, world, port, q, mode, 2, dtype, as_view, engine, boot_port,
                                                  poison))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=timeout) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("world,dtype,as_view", [(2, "f32", False), (2, "bf16", False), (2, "f16", False),
                                                 (2, "f32", True)])
def test_ddp_hook_plumbing_gloo(orc, world, dtype, as_view):
    res = run_world(world, "cpu", 300, dtype, as_view)
    for r, rep in res.items():
        assert "error" not in rep, rep.get("tb")
        # DDP's first iteration sends everything in one bucket; after its bucket
        # rebuild the small cap splits the model
        assert rep["buckets"][-1] >= 2, rep
        assert rep["calls"] == sum(rep["buckets"])
        assert rep["bit_exact"], rep
        assert rep["grad_err"] <= 1.0, rep


@pytest.mark.parametrize("dtype", ["f32", "f16"])
def test_ddp_hook_nonfinite_gloo(orc, dtype):
    """One rank's gradients overflow.  The hook propagates it: every rank's
    averaged gradients are all NaN, so a loss scaler skips the step on every
    rank alike.  Without propagation (the quantiser's spec) an fp32 bucket's
    other rank sees finite gradients -- the divergence the default prevents.
    (An fp16 bucket's saturated sum overflows fp16 on narrowing, so there the
    spec happens to yield Inf too.)"""
    res = run_world(2, "cpu", 300, dtype, poison="propagate")
    for r, rep in res.items():
        assert "error" not in rep, rep.get("tb")
        assert rep["found_inf"] and rep["all_nan"], (r, rep)
    if dtype != "f32":
        return
    res = run_world(2, "cpu", 300, dtype, poison="saturate")
    assert "error" not in res[0], res[0].get("tb")
    assert not res[0]["found_inf"], res[0]


def test_ddp_hook_refuses_other_formats():
    import torch

    from container_inc_amd import ddp
    from container_inc_amd._lib import IncclError

    class Bucket:
        def buffer(self):
            return torch.zeros(8, dtype=torch.float64)   # neither fp32, bf16 nor fp16

    with pytest.raises(IncclError):
        ddp.allreduce_hook(ddp.HookState(comm=None), Bucket())
