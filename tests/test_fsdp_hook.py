"""FSDP comm hooks (container_inc_amd/fsdp.py) on CPU: world 2 over gloo, the
engine's contract restated by the oracle (tests/_ddp_rank.py GlooStandIn), so
the hooks' plumbing inside FullyShardedDataParallel -- the padded flat gradient,
this rank's shard, the average -- is tested without a GPU.  The same worker runs
against the real library in tests/test_gpu_fsdp.py."""
import multiprocessing as mp

import pytest

from test_ddp_hook import _free_ports


def run_world(world, mode, timeout, sharded=True, engine="p2p", dtype="f32"):
    import _fsdp_rank
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port, boot_port = _free_ports(2)
    ps = [ctx.Process(target=_fsdp_rank.run, args=(r, world, port, q, mode, sharded, engine, boot_port, dtype))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=timeout) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("sharded", [True, False])
def test_fsdp_hooks_gloo(orc, sharded):
    res = run_world(2, "cpu", 300, sharded)
    for r, rep in res.items():
        assert "error" not in rep, rep.get("tb")
        assert rep["calls"] >= 2 and rep["checked"] == rep["calls"], rep
        assert rep["bit_exact"], rep


def test_fsdp_hook_refuses_bad_shapes():
    import torch

    from container_inc_amd import fsdp
    from container_inc_amd._lib import IncclError
    import types
    comm = types.SimpleNamespace(group=types.SimpleNamespace(world_size=2))
    st = fsdp.HookState(comm=comm)
    with pytest.raises(IncclError):
        fsdp.reduce_scatter_hook(st, torch.zeros(10), torch.zeros(4))   # 10 != 2 x 4
    with pytest.raises(IncclError):
        fsdp.reduce_scatter_hook(st, torch.zeros(8, dtype=torch.float64), torch.zeros(4, dtype=torch.float64))
    with pytest.raises(IncclError):   # a strided output shard would be written through a copy
        fsdp.reduce_scatter_hook(st, torch.zeros(8), torch.zeros(8)[::2])
    with pytest.raises(IncclError):
        fsdp.allreduce_hook(st, torch.zeros(4, 4).t())
