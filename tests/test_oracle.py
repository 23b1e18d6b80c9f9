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


# ---------------- ACK reflection and the frame-level pipeline ----------------
def test_ack_frame_matches_captured_ack(orc):
    """orc_build_ack_frame (util.c:331-442, PACKET_TYPE_ACK) against the soft-RoCE
    ACK captured in test.c:4-22: PSN 0, MSN 1, QPN 0x11.  Every byte agrees but
    the IP identification (the reference's builder writes 0x1111, util.c:358;
    the kernel that sent the captured frame wrote 0x2695) and the IP checksum
    that covers it; with those two fields taken from the capture the ICRC is
    the captured one (test.c:21)."""
    g = json.load(open(os.path.join(GOLDEN, "icrc_test_c.json")))
    cap = bytes.fromhex(g["frame_hex"])
    fr = orc.build_ack_frame(0, msn=1, qp=0x11, dst_mac=cap[0:6], src_mac=cap[6:12],
                             src_ip=int.from_bytes(cap[26:30], "little"), dst_ip=int.from_bytes(cap[30:34], "little"),
                             src_port=int.from_bytes(cap[34:36], "big"), dst_port=int.from_bytes(cap[36:38], "big"))
    assert len(fr) == 62 and len(cap) == 58
    diff = [i for i in range(58) if fr[i] != cap[i]]
    assert diff and set(diff) <= {18, 19, 24, 25}, diff
    assert fr[42] == 0x11 and fr[50:54] == bytes(4) and fr[54:58] == bytes.fromhex("1f000001")
    patched = bytearray(fr)
    patched[18:20], patched[24:26] = cap[18:20], cap[24:26]
    assert orc.icrc(bytes(patched)) == g["icrc_u32"]
    assert int.from_bytes(fr[58:62], "little") == orc.icrc(fr)


def _conns(fan_in):
    dt = np.dtype([("src_mac", np.uint8, 6), ("dst_mac", np.uint8, 6), ("src_ip", "<u4"), ("dst_ip", "<u4"),
                   ("src_port", "<u2"), ("dst_port", "<u2"), ("qp", "<u4")])
    t = np.zeros(fan_in, dt)
    for c in range(fan_in):
        t[c]["src_mac"] = [2, 0, 0, 0, 0, c]
        t[c]["dst_mac"] = [4, 0, 0, 0, 1, c]
        t[c]["src_ip"], t[c]["dst_ip"] = 0x0100000A + c, 0x0200000A + c
        t[c]["src_port"], t[c]["dst_port"], t[c]["qp"] = 4791, 5000 + c, 0x300 + c
    return t


def _conn_kw(t, c):
    return dict(qp=int(t[c]["qp"]), src_ip=int(t[c]["src_ip"]), dst_ip=int(t[c]["dst_ip"]),
                src_port=int(t[c]["src_port"]), dst_port=int(t[c]["dst_port"]),
                src_mac=bytes(t[c]["src_mac"]), dst_mac=bytes(t[c]["dst_mac"]))


def test_pipeline_frames_opcodes_and_reth(orc):
    """orc_switch_pipeline (nts.c:303-501, root) against the payload-level
    orc_switch_ingress and the frame builder: the broadcast takes the completing
    packet's opcode and each child's kept RETH (nts.c:442, :452), a replay the
    retransmit's opcode and the retransmitting child's RETH (:437), a data
    opcode's egress has no RETH (:355, :370) even when the counted copies were
    WRITE_FIRST; ACKs reflect to their port (:403-406); other opcodes and bad
    frames change nothing."""
    fan = 3
    t = _conns(fan)
    sw, ref = orc.Switch(fan), orc.Switch(fan)
    rng = np.random.default_rng(5)
    pay = {c: rng.integers(INT32_MIN, INT32_MAX, 256, dtype=np.int64, endpoint=True).astype(np.int32) for c in range(fan)}
    reth = {c: rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for c in range(fan)}
    psn = 9
    # child 0 WRITE_FIRST, child 1 SEND_ONLY (0x04), child 2 WRITE_ONLY (0x0A): completes with RETH
    ops = {0: 0x06, 1: 0x04, 2: 0x0A}
    for c in range(fan):
        wf = ops[c] in (0x06, 0x0A)
        fr = orc.build_data_frame(pay[c], psn=psn, opcode=ops[c], with_reth=wf, reth=reth[c] if wf else None)
        rc, outs = sw.pipeline(t, c, fr)
        rc2, _ = ref.ingress(c, psn, _be(pay[c]))
        assert rc == rc2
    assert rc == orc.SW_BROADCAST
    agg = orc.sum_q32(list(pay.values()))
    for c in range(fan):
        kept = reth[c] if ops[c] in (0x06, 0x0A) else bytes(16)   # child 1's copy had no RETH: the keeper stays 0
        assert outs[c] == orc.build_data_frame(agg, psn=psn, opcode=0x0A, with_reth=True, reth=kept, **_conn_kw(t, c))
    # retransmit of child 1 as SEND_MIDDLE (0x01): replay to child 1 only, no RETH, opcode 0x01
    rc, outs = sw.pipeline(t, 1, orc.build_data_frame(pay[1], psn=psn, opcode=0x01))
    assert rc == orc.SW_REPLAY and outs[0] is None and outs[2] is None
    assert outs[1] == orc.build_data_frame(agg, psn=psn, opcode=0x01, **_conn_kw(t, 1))
    # retransmit of child 0 as WRITE_FIRST: its kept RETH
    rc, outs = sw.pipeline(t, 0, orc.build_data_frame(pay[0], psn=psn, opcode=0x06, with_reth=True, reth=bytes(16)))
    assert rc == orc.SW_REPLAY
    assert outs[0] == orc.build_data_frame(agg, psn=psn, opcode=0x06, with_reth=True, reth=reth[0], **_conn_kw(t, 0))
    # a PSN whose counted copies were WRITE_FIRST but whose completing packet is WRITE_MIDDLE: no RETH out
    for c in range(fan):
        op = 0x07 if c == fan - 1 else 0x06
        rc, outs = sw.pipeline(t, c, orc.build_data_frame(pay[c], psn=10, opcode=op, with_reth=op == 0x06,
                                                          reth=reth[c] if op == 0x06 else None))
    assert rc == orc.SW_BROADCAST
    for c in range(fan):
        assert outs[c] == orc.build_data_frame(agg, psn=10, opcode=0x07, **_conn_kw(t, c))
    # ACK reflection: to the ACK's port, PSN and MSN = PSN + 1, state untouched
    ack = orc.build_ack_frame(0x123456, qp=0x77)
    rc, outs = sw.pipeline(t, 2, ack)
    assert rc == orc.SW_ACK and outs[0] is None and outs[1] is None
    assert outs[2] == orc.build_ack_frame(0x123456, msn=0x123457, **_conn_kw(t, 2))
    # an opcode pipeline() has no case for; a bad port; a short payload
    other = bytearray(orc.build_data_frame(pay[0], psn=11, opcode=0x07))
    other[42] = 0x64
    assert sw.pipeline(t, 0, bytes(other))[0] == orc.SW_IGNORED
    assert sw.pipeline(t, fan, orc.build_data_frame(pay[0], psn=11, opcode=0x07))[0] == orc.SW_INVALID
    assert sw.pipeline(t, 0, orc.build_data_frame(pay[0][:100], psn=11, opcode=0x07))[0] == orc.SW_INVALID
    # none of those touched PSN 11's slot: its first real copies still count
    rc, _ = sw.pipeline(t, 0, orc.build_data_frame(pay[0], psn=11, opcode=0x07))
    assert rc == orc.SW_ABSORBED


def test_pipeline_ack_msn_wraps(orc):
    """PSN 0xFFFFFF: MSN = PSN + 1 = 2^24, so AETH = htonl(0x1f000000 | 2^24) (util.c:394)."""
    t = _conns(1)
    sw = orc.Switch(1)
    rc, outs = sw.pipeline(t, 0, orc.build_ack_frame(0xFFFFFF))
    assert rc == orc.SW_ACK
    assert outs[0][50:54] == bytes.fromhex("00ffffff") and outs[0][54:58] == bytes.fromhex("1f000000")


def test_pipeline_ring_sizes(orc):
    """A ring larger than the reference's: window = slots / 2, so completing PSN p
    recycles slot p + slots/2 (nts.c:367 with N generalised)."""
    for slots in (16, 64, 1024):
        sw = orc.Switch(2, slots)
        one = _be(np.ones(256, np.int32))
        sw.ingress(0, 3 + slots // 2, one)                # an arrival in the slot that PSN 3 will recycle
        sw.ingress(0, 3, one)
        assert sw.ingress(1, 3, one)[0] == orc.SW_BROADCAST
        assert sw.ingress(0, 3 + slots // 2, one)[0] == orc.SW_ABSORBED   # recycled: counts again
    with pytest.raises(ValueError):
        orc.Switch(2, 24)
