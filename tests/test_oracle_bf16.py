"""The bfloat16 restatement (oracle/inccl_oracle.c orc_*_bf16) on CPU, pinned
two ways: its fp32 -> bf16 narrowing against PyTorch's own conversion (an
independent round-to-nearest-even implementation), and every bf16 function
against the fp32 functions applied to the exactly widened values.  The bf16
format has no reference counterpart (the reference moves int32 only); its spec
is DESIGN.md "Numerics"."""
import numpy as np
import pytest


def _bf16_bits(x32: np.ndarray) -> np.ndarray:
    """torch's fp32 -> bf16 (round to nearest even), as uint16 bit patterns."""
    import torch
    return torch.from_numpy(np.ascontiguousarray(x32, np.float32)).to(torch.bfloat16).view(torch.int16).numpy() \
        .view(np.uint16)


def _random_bf16(rng, n, scale=1.0):
    return _bf16_bits((rng.standard_normal(n) * scale).astype(np.float32))


def test_narrowing_matches_torch(orc):
    rng = np.random.default_rng(7)
    bits = rng.integers(0, 2 ** 32, 100_000, dtype=np.uint64).astype(np.uint32)
    x = bits.view(np.float32)
    x = x[np.isfinite(x)]
    # ties to even at both parities, around 1.0 and near the top of the range
    ties = np.array([0x3F808000, 0x3F818000, 0x3F807FFF, 0x3F808001, 0x7F7F7FFF, 0x7F7F8000, 0x00008000,
                     0x80018000, 0x00000001], np.uint32).view(np.float32)
    x = np.concatenate([x, ties])
    np.testing.assert_array_equal(orc.f32_to_bf16(x), _bf16_bits(x))


@pytest.mark.parametrize("R,k", [(1, 20), (2, 25), (3, "auto"), (8, "auto")])
def test_bf16_functions_are_the_fp32_ones_on_widened_values(orc, R, k):
    rng = np.random.default_rng(100 + R)
    n = 20_011
    hs = [_random_bf16(rng, n, 3.0) for _ in range(R)]
    hs[0][:4] = [0x7FC0, 0xFF80, 0x7F80, 0x0000]   # NaN -> 0, -Inf / +Inf saturate, +0
    ws = [orc.bf16_to_f32(h) for h in hs]
    assert orc.absmax_bf16(hs) == orc.absmax(ws)
    kk = orc.choose_scale(orc.absmax_bf16(hs), R) if k == "auto" else k
    np.testing.assert_array_equal(orc.quant_sum_bf16(hs, kk), orc.quant_sum(ws, kk))
    want = _bf16_bits(orc.reduce_f32(ws, kk))
    np.testing.assert_array_equal(orc.reduce_bf16(hs, kk), want)
    q = orc.quant_sum(ws, kk)
    np.testing.assert_array_equal(orc.sum_dequant_bf16([q], kk), _bf16_bits(orc.dequantise(q, kk)))


def test_bf16_known_answers(orc):
    # exact cases: 1.5 + 2.25 = 3.75 at k = 4; -0.5 + 0.5 = 0; a sum that needs
    # rounding: 1 + 2^-8 (bf16 has 8 significant bits) -> ties to even -> 1.0
    one, a, b = 0x3F80, 0x3FC0, 0x4010                   # 1.0, 1.5, 2.25
    half, mhalf = 0x3F00, 0xBF00
    tiny = _bf16_bits(np.array([2.0 ** -8], np.float32))[0]
    srcs = [np.array([a, mhalf, one], np.uint16), np.array([b, half, tiny], np.uint16)]
    got = orc.reduce_bf16(srcs, 10)
    np.testing.assert_array_equal(orc.bf16_to_f32(got), np.array([3.75, 0.0, 1.0], np.float32))


def _gloo_bf16_rank(rank, world, port, n, R, k, q):
    """inccl_allreduce_bf16's "rccl" decomposition over gloo: quant + local sum ->
    reduce-scatter int32 (by exchange) -> dequantise own shard to bf16 ->
    all-gather bf16, against reduce_bf16 of every rank's buckets."""
    try:
        _gloo_bf16_body(rank, world, port, n, R, k, q)
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def _gloo_bf16_body(rank, world, port, n, R, k, q):
    import sys

    from conftest import ROOT
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from container_inc_amd.plan import shard_elems
    from oracle import oracle as O
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    rng = np.random.default_rng(500 + rank)
    hs = [_random_bf16(rng, n, 2.0) for _ in range(R)]
    shard = shard_elems(n, world)
    part = np.zeros(shard * world, np.int32)
    part[:n] = O.quant_sum_bf16(hs, k)
    got = [torch.zeros(shard * world, dtype=torch.int32) for _ in range(world)]
    dist.all_gather(got, torch.from_numpy(part))
    mine = O.sum_dequant_bf16([g[rank * shard:(rank + 1) * shard].numpy() for g in got], k)
    # gloo has no 16-bit integer type: the bf16 bit patterns travel widened
    shards = [torch.zeros(shard, dtype=torch.int32) for _ in range(world)]
    dist.all_gather(shards, torch.from_numpy(mine.astype(np.int32)))
    out = torch.cat(shards).numpy().astype(np.uint16)[:n]
    allh = [None] * world
    dist.all_gather_object(allh, [h.tobytes() for h in hs])
    every = [np.frombuffer(b, np.uint16) for per in allh for b in per]
    q.put((rank, bool(np.array_equal(out, O.reduce_bf16(every, k)))))
    dist.destroy_process_group()


def test_gloo_world2_bf16_decomposition(orc):
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_bf16_rank, args=(r, 2, port, 10_007, 2, 24, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
