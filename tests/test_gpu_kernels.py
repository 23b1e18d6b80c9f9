"""HIP kernels vs the CPU oracle, bit-exact (gpu).  Every call goes through
libinccl_amd.so's C ABI; the oracle only checks."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

INT32_MIN, INT32_MAX = -(2 ** 31), 2 ** 31 - 1
SIZES = [1, 3, 4, 5, 255, 1024, 4099, 100_003]


def _t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _np(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _grads(rng, n, scale=1.0):
    x = (rng.standard_normal(n) * scale).astype(np.float32)
    if n >= 8:
        x[:8] = [np.nan, np.inf, -np.inf, 0.0, -0.0, 1e-45, 3e38, -3e38]
    return x


def _bits_equal(a, b):
    np.testing.assert_array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("k", [0, 25, -8, 64])
def test_quantise(gpu, orc, n, k):
    from container_inc_amd import inccl
    rng = np.random.default_rng(abs(n + 7 * k))
    x = _grads(rng, n, 2.0 ** (-k // 2) if k > 0 else 8.0)
    for be in (False, True):
        q = _np(inccl.quantise(_t(x, gpu), k, wire_be=be))
        want = orc.quantise(x, k)
        if be:
            want = orc.encode_be32(want).view(np.int32)
        np.testing.assert_array_equal(q, want)


def test_quantise_unaligned(gpu, orc):
    """Sub-tensor starting 4 bytes into an allocation: element-granular path."""
    from container_inc_amd import inccl
    rng = np.random.default_rng(1)
    x = _grads(rng, 10_001)
    xt = _t(x, gpu)[1:]
    q = _np(inccl.quantise(xt, 20))
    np.testing.assert_array_equal(q, orc.quantise(x[1:], 20))


def test_quant_known_answers(gpu):
    from container_inc_amd import inccl
    g = json.load(open(os.path.join(GOLDEN, "quant_kat.json")))
    by_k = {}
    for c in g["cases"]:
        by_k.setdefault(c["k"], []).append(c)
    for k, cases in by_k.items():
        x = np.array([c["bits"] for c in cases], np.uint32).view(np.float32)
        q = _np(inccl.quantise(_t(x, gpu), k))
        np.testing.assert_array_equal(q, np.array([c["q"] for c in cases], np.int64).astype(np.int32), err_msg=f"k={k}")


@pytest.mark.parametrize("n", SIZES)
def test_dequantise(gpu, orc, n):
    from container_inc_amd import inccl
    rng = np.random.default_rng(n)
    q = rng.integers(INT32_MIN, INT32_MAX, n, dtype=np.int64, endpoint=True).astype(np.int32)
    q[: min(n, 4)] = [INT32_MIN, INT32_MAX, 0, -1][: min(n, 4)]
    for k in (0, 25, -3, 64):
        _bits_equal(_np(inccl.dequantise(_t(q, gpu), k)), orc.dequantise(q, k))
        be = orc.encode_be32(q).view(np.int32)
        _bits_equal(_np(inccl.dequantise(_t(be, gpu), k, wire_be=True)), orc.dequantise(q, k))


@pytest.mark.parametrize("R", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("n", [1, 1023, 65_536 + 13])
def test_fused_reduce(gpu, orc, R, n):
    from container_inc_amd import inccl
    rng = np.random.default_rng(1000 * R + n)
    xs = [_grads(rng, n) for _ in range(R)]
    k = 25
    out = _np(inccl.reduce_f32([_t(x, gpu) for x in xs], k))
    _bits_equal(out, orc.reduce_f32(xs, k))


@pytest.mark.parametrize("R", [1, 2, 8])
def test_quant_sum_and_wire(gpu, orc, R):
    from container_inc_amd import inccl
    rng = np.random.default_rng(R)
    n = 50_001
    xs = [_grads(rng, n, 100.0) for _ in range(R)]
    ts = [_t(x, gpu) for x in xs]
    np.testing.assert_array_equal(_np(inccl.quant_sum(ts, 20)), orc.quant_sum(xs, 20))
    be = _np(inccl.quant_sum(ts, 20, wire_be=True))
    np.testing.assert_array_equal(be.view(np.uint32), orc.encode_be32(orc.quant_sum(xs, 20)))


def test_switch_sum_edge_lanes(gpu, orc):
    """Golden wrap-edge sums (non_termination_switch.c:361-363) in every wire order."""
    from container_inc_amd import inccl
    g = np.load(os.path.join(GOLDEN, "sum_edge.npz"))
    for R in range(2, 9):
        x = g[f"in_R{R}"]
        want = g[f"sum_R{R}"]
        ts = [_t(r, gpu) for r in x]
        np.testing.assert_array_equal(_np(inccl.sum_q32(ts)), want)
        wire = [_t(orc.encode_be32(r).view(np.int32), gpu) for r in x]
        got = _np(inccl.sum_q32(wire, in_be=True, out_be=True))
        np.testing.assert_array_equal(orc.decode_be32(got.view(np.uint32)), want)


@pytest.mark.parametrize("R", [1, 2, 8])
def test_sum_dequant(gpu, orc, R):
    from container_inc_amd import inccl
    rng = np.random.default_rng(40 + R)
    n = 12_345
    qs = [rng.integers(-2 ** 27, 2 ** 27, n, dtype=np.int64).astype(np.int32) for _ in range(R)]
    out = _np(inccl.sum_dequant([_t(q, gpu) for q in qs], 25))
    _bits_equal(out, orc.dequantise(orc.sum_q32(qs), 25))


@pytest.mark.parametrize("R,shift", [(1, 0), (2, 0), (8, 0), (2, 1), (3, 3)])
def test_absmax_and_auto_scale(gpu, orc, R, shift):
    """shift > 0: buckets that start `shift` elements past a 16-B boundary (the
    absmax then reads elements only, the reduce takes the element kernel)."""
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(77 + R)
    n = 100_003
    xs = [(rng.standard_normal(n) * 3).astype(np.float32) for _ in range(R)]
    xs[0][17] = np.nan
    xs[-1][n - 1] = -7.5   # the largest magnitude, in the ragged tail
    ts = [torch.from_numpy(np.concatenate([np.zeros(shift, np.float32), x])).to(gpu)[shift:] for x in xs]
    amax = inccl.absmax(ts)
    assert amax == orc.absmax(xs)
    k = orc.choose_scale(amax, R)
    _bits_equal(_np(inccl.reduce_f32_auto(ts)), orc.reduce_f32(xs, k))


@pytest.mark.parametrize("n", [1, 4, 1000, 1 << 20])
def test_checksum(gpu, orc, n):
    from container_inc_amd import inccl
    rng = np.random.default_rng(n)
    q = rng.integers(INT32_MIN, INT32_MAX, n, dtype=np.int64, endpoint=True).astype(np.int32)
    assert inccl.checksum_q32(_t(q, gpu)) == orc.checksum_q32(q)
    assert inccl.checksum_q32(_t(q, gpu), 12345) == orc.checksum_q32(q, 12345)


def test_in_place_dst_aliases_src(gpu, orc):
    from container_inc_amd import inccl
    rng = np.random.default_rng(9)
    xs = [_grads(rng, 33_333) for _ in range(2)]
    ts = [_t(x, gpu) for x in xs]
    inccl.reduce_f32(ts, 25, out=ts[0])
    _bits_equal(_np(ts[0]), orc.reduce_f32(xs, 25))


def test_rejects_bad_args(gpu):
    from container_inc_amd import inccl
    import torch
    x = torch.zeros(16, device=gpu)
    with pytest.raises(ValueError):
        inccl.reduce_f32([x] * 9, 25)
    with pytest.raises(ValueError):
        inccl.quantise(x, 65)
    with pytest.raises(TypeError):
        inccl.quantise(x.to(torch.float64), 3)


def test_full_bucket_256mib(gpu, orc):
    """BASELINE config 2 shape: two 256 MiB fp32 buckets, bit-exact vs the oracle,
    plus the size-independent linearity property sum(checksum(q_r)) == checksum(sum q_r)."""
    import torch
    from container_inc_amd import inccl
    n = 1 << 26
    gen = torch.Generator(device="cpu").manual_seed(1000)
    xs = [torch.randn(n, generator=gen, dtype=torch.float32) for _ in range(2)]
    ts = [x.to(gpu) for x in xs]
    k = 25
    out = inccl.reduce_f32(ts, k)
    _bits_equal(_np(out), orc.reduce_f32([x.numpy() for x in xs], k))
    qs = [inccl.quantise(t, k) for t in ts]
    s = inccl.quant_sum(ts, k)
    cs = sum(inccl.checksum_q32(q) for q in qs) % 2 ** 32
    assert inccl.checksum_q32(s) == cs
