"""Per-stage timing (gpu): inccl_comm_set_stage_timing / inccl_comm_stage_times
on the sharded allreduce (quant + local sum -> int32 reduce-scatter -> dequantise
the own shard -> all-gather, api.c allreduce_piece and its pipelined form) and
the reduce-scatter.  The stages must be recorded with plausible times, the
pipelined call must report its chunks' stages, and timing must not change a
result (bit-exact vs the oracle with timing on)."""
import numpy as np
import pytest

from test_gpu_comm import _run_ranks

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("chunks", [1, 4])
def test_stage_times_allreduce_local(gpu, orc, chunks):
    import torch
    from container_inc_amd import inccl
    world, n, k = 2, (1 << 22) + 192, 25
    rng = np.random.default_rng(chunks)
    hs = [[rng.standard_normal(n).astype(np.float32) for _ in range(2)] for _ in range(world)]
    want = orc.reduce_f32([h for per in hs for h in per], k)

    def rank(r):
        grp = inccl.inccl_group_create_local(world, r, f"stage-{chunks}")
        comm = inccl.inccl_communicator_create(grp, 0)
        xs = [torch.from_numpy(h).to(gpu) for h in hs[r]]
        comm.allreduce_f32(xs, scale_exp=k, chunks=chunks, stream=comm.stream)   # workspaces, untimed
        torch.cuda.synchronize()
        assert comm.stage_times()["stages"] == 0   # timing is off by default
        comm.set_stage_timing(True)
        out = comm.allreduce_f32(xs, scale_exp=k, chunks=chunks, stream=comm.stream)
        torch.cuda.synchronize()
        st = comm.stage_times()
        rs = comm.reduce_scatter(xs, scale_exp=k, stream=comm.stream)
        torch.cuda.synchronize()
        st_rs = comm.stage_times()
        comm.set_stage_timing(False)
        res = out.cpu().numpy(), rs.cpu().numpy(), st, st_rs
        comm.barrier()
        comm.destroy()
        grp.destroy()
        return res

    shard = n // world
    for r, (got, got_rs, st, st_rs) in enumerate(_run_ranks(world, rank)):
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
        np.testing.assert_array_equal(got_rs.view(np.uint32), want[r * shard:(r + 1) * shard].view(np.uint32))
        for name in ("quant", "reduce_scatter", "dequant", "all_gather"):
            assert st.get(name, 0.0) > 0.0, (name, st)
        # 4 stages per chunk (+ the copy-out of a ragged bucket), + the pipelined form's anchor
        assert st["stages"] >= 4 * chunks + (1 if chunks > 1 else 0), st
        assert st["wall_us"] > 0.0
        assert sum(v for key, v in st.items() if key in inccl.Communicator.STAGE_NAMES) >= 0.5 * st["wall_us"]
        for name in ("quant", "reduce_scatter", "dequant"):
            assert st_rs.get(name, 0.0) > 0.0, (name, st_rs)


@pytest.mark.parametrize("chunks", [1, 4])
def test_stage_times_rccl_world1(gpu, orc, monkeypatch, chunks):
    """The rccl engine's own stages around real RCCL collectives (world 1, the
    sharded route forced: ncclReduceScatter and ncclAllGather are launched)."""
    import torch
    from container_inc_amd import inccl
    monkeypatch.setenv("INCCL_FORCE_RCCL", "1")
    monkeypatch.setenv("INCCL_FORCE_SHARDED", "1")
    monkeypatch.setenv("INCCL_MASTER_PORT", "0")
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    comm.set_engine("rccl")
    n, k = 1 << 22, 25
    rng = np.random.default_rng(5 + chunks)
    hs = [rng.standard_normal(n).astype(np.float32) for _ in range(2)]
    xs = [torch.from_numpy(h).to(gpu) for h in hs]
    comm.allreduce_f32(xs, scale_exp=k, chunks=chunks, stream=comm.stream)
    torch.cuda.synchronize()
    comm.set_stage_timing(True)
    out = comm.allreduce_f32(xs, scale_exp=k, chunks=chunks, stream=comm.stream)
    torch.cuda.synchronize()
    st = comm.stage_times()
    comm.set_stage_timing(False)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), orc.reduce_f32(hs, k).view(np.uint32))
    for name in ("quant", "reduce_scatter", "dequant", "all_gather"):
        assert st.get(name, 0.0) > 0.0, (name, st)
    assert st["stages"] >= 4 * chunks, st
    comm.destroy()
    grp.destroy()
