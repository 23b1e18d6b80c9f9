"""The CPU oracle (oracle/inccl_oracle.c) pinned against the reference's own
known answers and the spec's known-answer vectors.  CPU only."""
import json
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN

INT32_MIN, INT32_MAX = -(2 ** 31), 2 ** 31 - 1


def _bits_f32(b):
    return struct.unpack("<f", struct.pack("<I", b))[0]


# ---------------- reference golden vectors ----------------
def test_host_known_answer_loopback(orc):
    """host.c:20-25,47,51-55 through api.c:403-452 + nts.c:303-501 restated."""
    g = np.load(os.path.join(GOLDEN, "host_known_answer.npz"))
    rc, dsts, frames = orc.allreduce_write_loopback(list(g["inputs"]))
    assert rc == g["inputs"].shape[1] // 1024
    for d in dsts:
        np.testing.assert_array_equal(d, g["expected"])
    # 4 messages x 4 packets x FAN_IN egress copies
    assert frames == 4 * 4 * 2


def test_icrc_matches_captured_frame(orc):
    """test.c:4-22: the ICRC the soft-RoCE stack wrote (test.c:21)."""
    g = json.load(open(os.path.join(GOLDEN, "icrc_test_c.json")))
    frame = bytes.fromhex(g["frame_hex"])
    assert orc.icrc(frame) == g["icrc_u32"]
    assert orc.icrc(frame).to_bytes(4, "little").hex() == g["icrc_bytes_hex"]


def test_ipv4_checksum_matches_captured_frame(orc):
    g = json.load(open(os.path.join(GOLDEN, "icrc_test_c.json")))
    frame = np.frombuffer(bytes.fromhex(g["frame_hex"]), np.uint8).copy()
    L = orc.lib()
    import ctypes
    L.orc_ipv4_checksum.argtypes = [ctypes.c_void_p]
    L.orc_ipv4_checksum.restype = ctypes.c_uint16
    assert L.orc_ipv4_checksum(frame[14:].ctypes.data) == g["ipv4_checksum"]


def test_crc32_check_value(orc):
    # the published CRC-32/ISO-HDLC check value; util.c:141-195 is that CRC
    assert orc.crc32(b"123456789") == 0xCBF43926
    assert orc.crc32(b"") == 0
    import zlib
    rng = np.random.default_rng(3)
    for n in (1, 7, 8, 9, 63, 1076):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert orc.crc32(b) == zlib.crc32(b)


def test_sum_edge_lanes(orc):
    g = np.load(os.path.join(GOLDEN, "sum_edge.npz"))
    for R in range(2, 9):
        x = g[f"in_R{R}"]
        np.testing.assert_array_equal(orc.sum_q32(list(x)), g[f"sum_R{R}"])


def test_quant_known_answers(orc):
    g = json.load(open(os.path.join(GOLDEN, "quant_kat.json")))
    bits = np.array([c["bits"] for c in g["cases"]], np.uint32)
    x = bits.view(np.float32)
    for c, xv in zip(g["cases"], x):
        assert orc.lib().orc_quantise_one(float(xv), c["k"]) == c["q"], c


# ---------------- spec properties ----------------
def test_dequant_exact(orc):
    rng = np.random.default_rng(5)
    q = rng.integers(INT32_MIN, INT32_MAX, 4096, dtype=np.int64, endpoint=True).astype(np.int32)
    q[:4] = [INT32_MIN, INT32_MAX, 0, -1]
    for k in (-64, -3, 0, 25, 64):
        f = orc.dequantise(q, k)
        ref = (q.astype(np.float64).astype(np.float32).astype(np.float64) * 2.0 ** -k).astype(np.float32)
        np.testing.assert_array_equal(f.view(np.uint32), ref.view(np.uint32))


def test_reduce_matches_composition(orc):
    rng = np.random.default_rng(7)
    for R in (1, 2, 3, 8):
        xs = [rng.standard_normal(3001).astype(np.float32) for _ in range(R)]
        k = 25
        fused = orc.reduce_f32(xs, k)
        comp = orc.dequantise(orc.sum_q32([orc.quantise(x, k) for x in xs]), k)
        np.testing.assert_array_equal(fused.view(np.uint32), comp.view(np.uint32))
        np.testing.assert_array_equal(orc.quant_sum(xs, k), orc.sum_q32([orc.quantise(x, k) for x in xs]))
        # quantisation error bound vs the exact sum: R * 2^-(k+1) plus fp32 rounding of the result
        exact = np.sum(np.stack(xs).astype(np.float64), axis=0)
        err = np.abs(fused.astype(np.float64) - exact)
        assert np.all(err <= R * 2.0 ** -(k + 1) + np.abs(exact) * 2.0 ** -24 + 1e-12)


def test_choose_scale(orc):
    assert orc.choose_scale(0.0, 2) == 64
    assert orc.choose_scale(float("inf"), 2) == -64
    for amax in (1e-3, 0.5, 1.0, 3.0, 6.0, 1000.0, 1.5e9):
        for R in (1, 2, 8, 16):
            k = orc.choose_scale(amax, R)
            assert R * amax * 2.0 ** k <= 2 ** 30 or k == -64
            if k < 64:
                assert R * amax * 2.0 ** (k + 1) > 2 ** 30
    # headroom: R buckets of max |x| never wrap
    rng = np.random.default_rng(11)
    xs = [rng.standard_normal(5000).astype(np.float32) * 4 for _ in range(8)]
    k = orc.choose_scale(orc.absmax(xs), 8)
    s = np.sum(np.stack([orc.quantise(x, k).astype(np.int64) for x in xs]), axis=0)
    assert np.all(np.abs(s) < 2 ** 31)


def test_absmax_ignores_nan(orc):
    x = np.array([1.0, -5.0, np.nan, 2.0], np.float32)
    assert orc.absmax([x]) == 5.0


def test_checksum_linear(orc):
    rng = np.random.default_rng(13)
    qs = [rng.integers(INT32_MIN, INT32_MAX, 999, dtype=np.int64, endpoint=True).astype(np.int32) for _ in range(3)]
    s = orc.sum_q32(qs)
    lhs = orc.checksum_q32(s)
    rhs = sum(orc.checksum_q32(q) for q in qs) % 2 ** 32
    assert lhs == rhs
    # split checksum = sum of piece checksums with the index base
    assert orc.checksum_q32(s) == (orc.checksum_q32(s[:500]) + orc.checksum_q32(s[500:], 500)) % 2 ** 32


def test_wire_codec_roundtrip(orc):
    x = np.array([1, -1, INT32_MIN, INT32_MAX, 0x01020304], np.int32)
    w = orc.encode_be32(x)
    assert w[4] == 0x04030201
    np.testing.assert_array_equal(orc.decode_be32(w), x)


# ---------------- switch semantics (nts.c:303-501) ----------------
def _be(x):
    return x.astype(np.int32).view(np.uint32).byteswap()


def test_switch_aggregate_and_idempotence(orc):
    sw = orc.Switch(2)
    rng = np.random.default_rng(17)
    a = rng.integers(INT32_MIN, INT32_MAX, 256, dtype=np.int64, endpoint=True).astype(np.int32)
    b = rng.integers(INT32_MIN, INT32_MAX, 256, dtype=np.int64, endpoint=True).astype(np.int32)
    rc, _ = sw.ingress(0, 5, _be(a))
    assert rc == orc.SW_ABSORBED
    rc, _ = sw.ingress(0, 5, _be(a))          # retransmit before completion: dropped, not re-added
    assert rc == orc.SW_DROPPED
    rc, eg = sw.ingress(1, 5, _be(b))
    assert rc == orc.SW_BROADCAST
    want = (a.astype(np.int64) + b.astype(np.int64) + 2 ** 31) % 2 ** 32 - 2 ** 31
    np.testing.assert_array_equal(eg.byteswap().view(np.int32), want.astype(np.int32))
    rc, eg2 = sw.ingress(1, 5, _be(b))        # retransmit after completion: replay (nts.c:353-356)
    assert rc == orc.SW_REPLAY
    np.testing.assert_array_equal(eg2, eg)


def test_switch_slot_recycling(orc):
    """Completing psn clears slot psn+8 (nts.c:367): psn+16 reuses psn's slot cleanly."""
    sw = orc.Switch(2)
    one = _be(np.ones(256, np.int32))
    for psn in range(0, 40):
        sw.ingress(0, psn, one)
        rc, eg = sw.ingress(1, psn, one)
        assert rc == orc.SW_BROADCAST
        np.testing.assert_array_equal(eg.byteswap().view(np.int32), np.full(256, 2, np.int32))


@pytest.mark.parametrize("R", [2, 3, 8])
def test_loopback_random_with_retransmits(orc, R):
    rng = np.random.default_rng(100 + R)
    n = 1024 * 9 + 300            # ragged tail stays untouched (api.c:406)
    xs = [rng.integers(INT32_MIN, INT32_MAX, n, dtype=np.int64, endpoint=True).astype(np.int32) for _ in range(R)]
    init = [np.full(n, 77, np.int32) for _ in range(R)]
    rc, dsts, frames = orc.allreduce_write_loopback(xs, dup_every=3, dst_init=init)
    assert rc == 9
    want = orc.sum_q32(xs)
    for d in dsts:
        np.testing.assert_array_equal(d[: 9 * 1024], want[: 9 * 1024])
        assert np.all(d[9 * 1024:] == 77)


def test_loopback_rejects_short_len(orc):
    rc, _, _ = orc.allreduce_write_loopback([np.zeros(1024, np.int32)] * 2)
    assert rc == -1   # window posts 2 messages unconditionally (api.c:408): the reference reads past src


def test_frame_layout(orc):
    payload = np.arange(256, dtype=np.int32)
    fr = orc.build_data_frame(payload, psn=7, opcode=0x07)
    assert len(fr) == 1082                       # 54 B headers + 1024 B + 4 B ICRC
    assert fr[42] == 0x07                         # BTH opcode
    assert int.from_bytes(fr[50:54], "big") == 0x80000007   # ack-request bit | psn (util.c:386)
    body = np.frombuffer(fr[54:54 + 1024], ">i4")
    np.testing.assert_array_equal(body, payload)
    assert int.from_bytes(fr[-4:], "little") == orc.icrc(fr)
    fr2 = orc.build_data_frame(payload, psn=8, opcode=0x06, with_reth=True)
    assert len(fr2) == 1098
