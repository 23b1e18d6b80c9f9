"""The oracle's IEEE binary16 restatement (oracle/inccl_oracle.c: orc_f16_to_f32,
orc_f32_to_f16 and the fp16 bucket functions), pinned against numpy's float16
conversions -- IEEE 754 binary16 with round to nearest even -- exhaustively for
widening and on every rounding class for narrowing.  CPU only.  The reference
has no floating point at all: fp16 buckets are a caller-side
format of the engine, like bf16 (tests/test_oracle_bf16.py)."""
import numpy as np
import pytest

INT32_MIN, INT32_MAX = -(2 ** 31), 2 ** 31 - 1


def test_widening_exhaustive(orc):
    h = np.arange(1 << 16, dtype=np.uint32).astype(np.uint16)
    got = orc.f16_to_f32(h)
    want = h.view(np.float16).astype(np.float32)
    nan = np.isnan(want)
    assert np.array_equal(np.isnan(got), nan)
    np.testing.assert_array_equal(got[~nan].view(np.uint32), want[~nan].view(np.uint32))


def test_narrowing_every_rounding_class(orc):
    rng = np.random.default_rng(16)
    # every half's neighbourhood: the value itself, the exact midpoints to its
    # neighbours (ties to even), and one fp32 ulp either side of them
    h = np.arange(0, 0x7C00, dtype=np.uint32).astype(np.uint16)   # finite non-negative halves
    v = h.view(np.float16).astype(np.float64)
    nxt = np.append(v[1:], 65536.0)
    mid = ((v + nxt) / 2).astype(np.float32)
    cands = [v.astype(np.float32), mid, np.nextafter(mid, np.float32(np.inf)), np.nextafter(mid, np.float32(0))]
    x = np.concatenate(cands + [rng.standard_normal(1 << 20).astype(np.float32) * s for s in (1e-6, 1e-3, 1.0, 1e4)])
    x = np.concatenate([x, -x, np.float32([65504, 65519.99, 65520, 65536, 1e30, np.inf, -np.inf, 2.0 ** -25,
                                           2.0 ** -24, 1.5 * 2.0 ** -25, 2.0 ** -14, 0.0, -0.0])])
    got = orc.f32_to_f16(x)
    with np.errstate(over="ignore"):
        want = x.astype(np.float16).view(np.uint16)
    np.testing.assert_array_equal(got, want)
    nan = orc.f32_to_f16(np.float32([np.nan]))
    assert (int(nan[0]) & 0x7C00) == 0x7C00 and (int(nan[0]) & 0x3FF) != 0


@pytest.mark.parametrize("R,k", [(1, 10), (2, 14), (3, 22), (8, 18)])
def test_f16_functions_are_the_fp32_ones_on_widened_values(orc, R, k):
    rng = np.random.default_rng(R * 31 + k)
    n = 4097
    hs = [(rng.standard_normal(n) * 4).astype(np.float16).view(np.uint16) for _ in range(R)]
    hs[0][:4] = [0x7E00, 0xFC00, 0x7C00, 0x0001]   # NaN -> 0, -Inf / +Inf saturate, the smallest subnormal
    widened = [orc.f16_to_f32(h) for h in hs]
    q = orc.quant_sum(widened, k)
    np.testing.assert_array_equal(orc.quant_sum_f16(hs, k), q)
    deq = orc.dequantise(q, k)
    with np.errstate(over="ignore"):
        want = deq.astype(np.float16).view(np.uint16)
    np.testing.assert_array_equal(orc.reduce_f16(hs, k), want)
    np.testing.assert_array_equal(orc.sum_dequant_f16([q], k), want)
    a = np.abs(np.concatenate(widened))
    assert orc.absmax_f16(hs) == float(np.max(a[~np.isnan(a)]))


def test_f16_known_answers(orc):
    one = np.uint16(0x3C00)
    # 1.0 + 1.0 at k = 10 -> 2048 -> 2.0
    assert int(orc.reduce_f16([np.array([one]), np.array([one])], 10)[0]) == 0x4000
    # 65504 + 65504 at k = 0: 131008, past the largest half -> +Inf
    big = np.array([0x7BFF], np.uint16)
    assert int(orc.reduce_f16([big, big], 0)[0]) == 0x7C00
    # a sum that dequantises below the smallest subnormal: 3 * 2^-26 = 0.75 * 2^-24 rounds up to it
    q = np.array([3], np.int32)
    assert int(orc.sum_dequant_f16([q], 26)[0]) == 0x0001


def test_absmax_word_flagged(orc):
    """The INCCL_ABSMAX_FLAG_NONFINITE word's restatement: finite buckets give
    the plain absmax bits; an Inf gives bit 31 | 0x7f800000; a NaN sets bit 31."""
    import numpy as np
    x = np.array([1.5, -3.25, 0.0], np.float32)
    assert orc.absmax_word_flagged([x]) == int(np.float32(3.25).view(np.uint32))
    assert orc.absmax_word_flagged([x, np.array([np.inf], np.float32)]) == 0x80000000 | 0x7F800000
    assert orc.absmax_word_flagged([np.array([np.nan, 1.0], np.float32)]) >> 31 == 1
    h = np.array([1.0, -2.0], np.float16).view(np.uint16)
    assert orc.absmax_word_flagged([h], "f16") == int(np.float32(2.0).view(np.uint32))
    assert orc.any_nonfinite([np.array([np.inf], np.float16).view(np.uint16)], "f16")
    b = np.array([0x3F80, 0xFF80], np.uint16)   # bf16 1.0, -Inf
    assert orc.absmax_word_flagged([b], "bf16") == 0x80000000 | 0x7F800000
    assert not orc.any_nonfinite([np.array([0x3F80], np.uint16)], "bf16")
