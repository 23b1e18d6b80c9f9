"""FSDP comm hooks on the GPU (gpu): FullyShardedDataParallel (FULL_SHARD and
NO_SHARD) with ``container_inc_amd.fsdp`` hooks, the real library underneath
(p2p engine; every rank on cuda:0 of a one-GPU box, FSDP's own parameter
all-gathers over gloo).  Every hooked call's shard must equal the oracle's
reduce of all ranks' gradients, sliced and divided by W, bit for bit
(tests/_fsdp_rank.py)."""
import pytest

from test_fsdp_hook import run_world

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sharded,dtype", [(True, "f32"), (False, "f32"), (True, "bf16")])
def test_fsdp_hooks_gpu(gpu, orc, sharded, dtype):
    res = run_world(2, "gpu", 240, sharded, "p2p", dtype)
    for r, rep in res.items():
        assert "error" not in rep, rep.get("tb")
        assert rep["calls"] >= 2 and rep["checked"] == rep["calls"], rep
        assert rep["bit_exact"], rep
