"""The oracle's non-root switch (nts.c:376-400, :408-423, :457-499) on
hand-worked sequences (CPU).  Every expected frame here is built from what the
reference's branches send -- send_roce_data / _with_reth with the aggregator
re-encoded by htonl (util.c:403-405) -- with the sums and byte orders computed
in this file, not by the restatement under test.

The reference needs libpcap to build, so its non-root branches cannot be run
here.  SURVEY §0 drove them once and recorded one output -- a child decodes
234881024 where the parent sent 14, every word's bytes reversed -- kept as
tests/golden/nonroot_down_survey.json and checked below."""
import numpy as np
import pytest

TEMPLATE = np.dtype([("src_mac", np.uint8, 6), ("dst_mac", np.uint8, 6), ("src_ip", "<u4"), ("dst_ip", "<u4"),
                     ("src_port", "<u2"), ("dst_port", "<u2"), ("qp", "<u4")])
INT32_MIN, INT32_MAX = -(2 ** 31), 2 ** 31 - 1


def _conns(rows):
    t = np.zeros(rows, TEMPLATE)
    for c in range(rows):
        t[c]["src_mac"] = [0x52, 0x54, 0, 0xAA, 0, c]
        t[c]["dst_mac"] = [0x52, 0x54, 0, 0xBB, 1, c]
        t[c]["src_ip"] = 0x0132320A + (c << 24)
        t[c]["dst_ip"] = 0x0232320A + (c << 24)
        t[c]["src_port"] = 4791
        t[c]["dst_port"] = 4791 + c
        t[c]["qp"] = 0x100 + c
    return t


def _send(orc, t, c, words, psn, op, reth=None):
    """send_roce_data[_with_reth] to row c: `words` are the aggregator's host words."""
    wf = op in (0x06, 0x0A)
    return orc.build_data_frame(np.asarray(words, np.int32), psn=psn, opcode=op, qp=int(t[c]["qp"]), with_reth=wf,
                                reth=(reth if reth is not None else bytes(16)) if wf else None,
                                src_ip=int(t[c]["src_ip"]), dst_ip=int(t[c]["dst_ip"]),
                                src_port=int(t[c]["src_port"]), dst_port=int(t[c]["dst_port"]),
                                src_mac=bytes(t[c]["src_mac"]), dst_mac=bytes(t[c]["dst_mac"]))


def _in(orc, words, psn, op, reth=None):
    """A frame arriving at the switch (any sender)."""
    wf = op in (0x06, 0x0A)
    return orc.build_data_frame(np.asarray(words, np.int32), psn=psn, opcode=op, with_reth=wf,
                                reth=(reth or bytes(16)) if wf else None)


def _wrap_sum(*xs):
    return np.sum([np.asarray(x, np.int64) for x in xs], axis=0).astype(np.uint32).view(np.int32)


def _reversed_words(y):
    """The reference's downstream words: the parent's wire bytes kept as host
    words (nts.c:413 memcpy) and htonl'd again -- each word's bytes reversed."""
    return np.frombuffer(np.asarray(y, np.int32).astype(">i4").tobytes(), "<i4")


def _pay(rng):
    return rng.integers(INT32_MIN, INT32_MAX, 256, dtype=np.int64, endpoint=True).astype(np.int32)


@pytest.mark.parametrize("flags", [0, 1])
def test_nonroot_forward_down_replay(orc, flags):
    rng = np.random.default_rng(7 + flags)
    F = 2
    t = _conns(F + 1)
    sw = orc.Switch(F, 16, nonroot=True, flags=flags)
    x0, x1, y = _pay(rng), _pay(rng), _pay(rng)
    agg = _wrap_sum(x0, x1)
    down = y if flags & orc.SW_WIRE_ORDER else _reversed_words(y)

    def step(port, frame, want_rc, want_rows):
        rc, outs = sw.pipeline(t, port, frame)
        assert rc == want_rc, (rc, want_rc)
        for c in range(F + 1):
            assert outs[c] == want_rows.get(c), c

    step(0, _in(orc, x0, 5, 0x07), orc.SW_ABSORBED, {})
    # the last child's first copy: the aggregate goes to the parent (nts.c:394-397)
    step(1, _in(orc, x1, 5, 0x08), orc.SW_FORWARD, {2: _send(orc, t, 2, agg, 5, 0x08)})
    # retransmits before the parent's result: degree 3 drops, degree 4 resends (:381-384)
    step(0, _in(orc, _pay(rng), 5, 0x07), orc.SW_DROPPED, {})
    step(1, _in(orc, _pay(rng), 5, 0x01), orc.SW_FORWARD, {2: _send(orc, t, 2, agg, 5, 0x01)})
    # an ACK from a child is reflected; one from the parent is "impossible" (:424-426)
    rc, outs = sw.pipeline(t, 0, orc.build_ack_frame(5))
    assert rc == orc.SW_ACK and outs[0] is not None and outs[1] is None and outs[2] is None
    step(2, orc.build_ack_frame(5), orc.SW_IGNORED, {})
    # the parent's result: taken once, broadcast to every child (:412-419)
    step(2, _in(orc, y, 5, 0x07), orc.SW_DOWN, {0: _send(orc, t, 0, down, 5, 0x07), 1: _send(orc, t, 1, down, 5, 0x07)})
    assert np.array_equal(sw.slot(5).view(np.int32), down if flags else np.frombuffer(y.astype(">i4").tobytes(), "<i4"))
    step(2, _in(orc, _pay(rng), 5, 0x07), orc.SW_DROPPED, {})
    # a retransmit after it: the result, to that child only (:378-380)
    step(1, _in(orc, _pay(rng), 5, 0x02), orc.SW_REPLAY, {1: _send(orc, t, 1, down, 5, 0x02)})
    # a parent packet before every child arrived is ignored (:412 second condition)
    step(0, _in(orc, x0, 6, 0x07), orc.SW_ABSORBED, {})
    step(2, _in(orc, y, 6, 0x07), orc.SW_DROPPED, {})
    step(1, _in(orc, x1, 6, 0x07), orc.SW_FORWARD, {2: _send(orc, t, 2, agg, 6, 0x07)})
    step(2, _in(orc, y, 6, 0x04), orc.SW_DOWN, {0: _send(orc, t, 0, down, 6, 0x04), 1: _send(orc, t, 1, down, 6, 0x04)})


def test_nonroot_write_first_reths(orc):
    """WRITE_FIRST / WRITE_ONLY copies: each child's RETH is kept (:470); the
    parent gets a zeroed RETH (send_roce_data_with_reth(FAN_IN, NULL), :478); the
    children get their own kept RETH back with the result (:493)."""
    rng = np.random.default_rng(11)
    F = 3
    t = _conns(F + 1)
    sw = orc.Switch(F, 16, nonroot=True)
    xs = [_pay(rng) for _ in range(F)]
    reths = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(F)]
    ops = [0x06, 0x0A, 0x06]
    for c in range(F - 1):
        rc, outs = sw.pipeline(t, c, _in(orc, xs[c], 9, ops[c], reths[c]))
        assert rc == orc.SW_ABSORBED and outs == [None] * (F + 1)
    rc, outs = sw.pipeline(t, F - 1, _in(orc, xs[F - 1], 9, ops[F - 1], reths[F - 1]))
    assert rc == orc.SW_FORWARD
    assert outs[F] == _send(orc, t, F, _wrap_sum(*xs), 9, ops[F - 1], bytes(16))
    assert outs[:F] == [None] * F
    y = _pay(rng)
    rc, outs = sw.pipeline(t, F, _in(orc, y, 9, 0x0A, rng.integers(0, 256, 16, dtype=np.uint8).tobytes()))
    assert rc == orc.SW_DOWN
    for c in range(F):
        assert outs[c] == _send(orc, t, c, _reversed_words(y), 9, 0x0A, reths[c]), c
    assert outs[F] is None


@pytest.mark.parametrize("flags", [0, 2])
def test_nonroot_slot_reuse(orc, flags):
    """The reference's non-root never recycles (clear_state_data only at the
    root, :367, :449): PSN p + 16 lands in p's slot with every bit still set, so
    its first copy is taken for a retransmit and answered with p's result.
    SW_RECYCLE clears slot p + 8 when p's result is taken, as the root does at
    completion, so p + 16 starts afresh once p + 8 completed."""
    rng = np.random.default_rng(13)
    F = 2
    t = _conns(F + 1)
    sw = orc.Switch(F, 16, nonroot=True, flags=flags)
    ys = {}
    for p in (5, 13):
        for c in range(F):
            sw.pipeline(t, c, _in(orc, _pay(rng), p, 0x07))
        ys[p] = _pay(rng)
        assert sw.pipeline(t, F, _in(orc, ys[p], p, 0x07))[0] == orc.SW_DOWN
    rc, outs = sw.pipeline(t, 0, _in(orc, _pay(rng), 21, 0x07))
    if flags & orc.SW_RECYCLE:
        assert rc == orc.SW_ABSORBED and outs == [None] * 3
    else:
        assert rc == orc.SW_REPLAY
        assert outs[0] == _send(orc, t, 0, _reversed_words(ys[5]), 21, 0x07)


def test_nonroot_bad_ports_and_lengths(orc):
    F = 2
    t = _conns(F + 1)
    sw = orc.Switch(F, 16, nonroot=True)
    good = _in(orc, np.ones(256, np.int32), 3, 0x07)
    assert sw.pipeline(t, 3, good)[0] == orc.SW_INVALID          # past the parent's port
    assert sw.pipeline(t, -1, good)[0] == orc.SW_INVALID
    short = orc.build_data_frame(np.ones(100, np.int32), psn=3, opcode=0x07)
    assert sw.pipeline(t, 2, short)[0] == orc.SW_INVALID         # the DOWN length assert (:411)
    odd = bytearray(good)
    odd[42] = 0x64
    assert sw.pipeline(t, 2, bytes(odd))[0] == orc.SW_IGNORED
    with pytest.raises(ValueError):
        orc.Switch(F, 16, nonroot=True, flags=4)


@pytest.mark.parametrize("flags", [0, 1])
def test_two_tier_tree_allreduce(orc, flags):
    """Four hosts under two non-root switches under one root (the reference's
    multi-switch topology, fan-in 2 at each tier): every host's packet goes up,
    each non-root forwards its children's aggregate to the root, the root
    broadcasts the total, each non-root takes it and sends it down.  With
    SW_WIRE_ORDER every host receives the four-way wrap-around sum; in the
    reference's byte order, every word byte-reversed."""
    rng = np.random.default_rng(17 + flags)
    P = 6
    x = [[_pay(rng) for _ in range(P)] for _ in range(4)]
    leaves = [orc.Switch(2, 16, nonroot=True, flags=flags) for _ in range(2)]
    root = orc.Switch(2, 16)
    tl, tr = _conns(3), _conns(2)
    for p in range(P):
        op = (0x07, 0x06, 0x08)[p % 3]
        up = []
        for s in range(2):
            for c in range(2):
                rc, outs = leaves[s].pipeline(tl, c, _in(orc, x[2 * s + c][p], p, op))
                if rc == orc.SW_FORWARD:
                    up.append((s, outs[2]))
        assert [s for s, _ in up] == [0, 1]
        for s, fr in up:
            rc, down = root.pipeline(tr, s, fr)
        assert rc == orc.SW_BROADCAST
        total = _wrap_sum(*[x[h][p] for h in range(4)])
        want = total if flags & orc.SW_WIRE_ORDER else _reversed_words(total)
        off = 70 if op == 0x06 else 54
        for s in range(2):
            rc, outs = leaves[s].pipeline(tl, 2, down[s])
            assert rc == orc.SW_DOWN
            for c in range(2):
                got = np.frombuffer(outs[c][off:off + 1024], ">i4").astype(np.int32)
                assert np.array_equal(got, want), (p, s, c)
                assert orc.icrc(outs[c]) == int.from_bytes(outs[c][-4:], "little")


def test_nonroot_down_matches_surveyed_reference_output(orc):
    """The one reference-produced output for the non-root role: SURVEY §0
    drove the reference's pipeline() as a non-root and recorded that a child
    decodes 234881024 where the parent sent 14 (tests/golden/
    nonroot_down_survey.json).  The restatement (flags 0) gives exactly that in
    every lane; SW_WIRE_ORDER gives the parent's 14 back."""
    import json
    import os

    from conftest import GOLDEN
    g = json.load(open(os.path.join(GOLDEN, "nonroot_down_survey.json")))
    for flags, want in ((0, g["child_value"]), (orc.SW_WIRE_ORDER, g["parent_value"])):
        t = _conns(3)
        sw = orc.Switch(2, 16, nonroot=True, flags=flags)
        for c in range(2):
            sw.pipeline(t, c, _in(orc, np.arange(256, dtype=np.int32), 3, 0x07))
        rc, outs = sw.pipeline(t, 2, _in(orc, np.full(256, g["parent_value"], np.int32), 3, 0x07))
        assert rc == orc.SW_DOWN
        for c in range(2):
            got = np.frombuffer(outs[c][54:54 + 1024], ">i4")   # what the host's ntohl decodes
            assert (got == want).all(), (flags, c)
