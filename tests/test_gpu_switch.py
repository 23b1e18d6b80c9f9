"""The reference switch's dataplane on the GPU vs the oracle (gpu): RoCE ICRC
(util.c:250-286) against the captured frame of test.c and oracle-built frames;
batched ingress (non_termination_switch.c:303-483: first-arrival add,
retransmit drop / replay) and egress frames (util.c:331-442) byte-exact.  Every
batch test runs both ways of driving the switch: `split` (inccl_switch_ingress
then inccl_switch_egress) and `batch` (inccl_switch_batch: both in one call)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
STRIDE = 1152
INT32_MIN, INT32_MAX = -(2 ** 31), 2 ** 31 - 1


def _rows(frames, dev, stride=STRIDE):
    import torch
    a = np.zeros((len(frames), stride), np.uint8)
    for i, f in enumerate(frames):
        a[i, : len(f)] = np.frombuffer(f, np.uint8)
    return torch.from_numpy(a).to(dev)


def test_icrc_golden_frame(gpu):
    from container_inc_amd import inccl
    g = json.load(open(os.path.join(GOLDEN, "icrc_test_c.json")))
    got = inccl.icrc_frames(_rows([bytes.fromhex(g["frame_hex"])], gpu)).cpu().numpy().view(np.uint32)
    assert int(got[0]) == g["icrc_u32"]


def test_icrc_random_frames(gpu, orc):
    from container_inc_amd import inccl
    rng = np.random.default_rng(21)
    frames = []
    for i in range(300):
        payload = rng.integers(INT32_MIN, INT32_MAX, 256, dtype=np.int64, endpoint=True).astype(np.int32)
        wf = bool(i % 3 == 0)
        frames.append(orc.build_data_frame(payload, psn=int(rng.integers(0, 1 << 24)), opcode=0x06 if wf else 0x07,
                                           qp=int(rng.integers(0, 1 << 24)), with_reth=wf,
                                           reth=rng.integers(0, 256, 16, dtype=np.uint8).tobytes() if wf else None,
                                           src_ip=int(rng.integers(0, 1 << 32)), dst_ip=int(rng.integers(0, 1 << 32)),
                                           src_port=int(rng.integers(0, 65536)), dst_port=4791))
    got = inccl.icrc_frames(_rows(frames, gpu)).cpu().numpy().view(np.uint32)
    for f, c in zip(frames, got):
        assert int(c) == orc.icrc(f) == int.from_bytes(f[-4:], "little")


def test_icrc_any_length(gpu, orc):
    """Random bytes at every IP length class the window covers: 28..60, random
    lengths, and the last few before the 1088-byte window is full (the leading
    zero region then ends inside lane 0, at a lane boundary, or not at all)."""
    from container_inc_amd import inccl
    rng = np.random.default_rng(22)
    lens = list(range(28, 61)) + [int(x) for x in rng.integers(28, 1089, 60)] + list(range(1060, 1089))
    frames = []
    for ipt in lens:
        f = bytearray(rng.integers(0, 256, 14 + ipt, dtype=np.uint8).tobytes())
        f[16], f[17] = ipt >> 8, ipt & 0xFF
        frames.append(bytes(f))
    got = inccl.icrc_frames(_rows(frames, gpu)).cpu().numpy().view(np.uint32)
    for ipt, f, c in zip(lens, frames, got):
        assert int(c) == orc.icrc(f), ipt


@pytest.mark.parametrize("stride,count", [(1100, 7), (1100, 1), (1104, 9), (1152, 5), (1240, 3)])
def test_icrc_row_strides_odd_counts(gpu, orc, stride, count):
    """Rows that are 4- but not 16-byte aligned, rows that end 2 bytes after a
    1098-byte frame (stride 1100), and odd frame counts (the two-frames-per-wave
    kernels' lone last frame).  Every ICRC against the oracle."""
    from container_inc_amd import inccl
    rng = np.random.default_rng(stride + count)
    lens = [1084, 1068] + [int(x) for x in rng.integers(28, 1085, max(count - 2, 0))]
    frames = []
    for ipt in lens[:count]:
        f = bytearray(rng.integers(0, 256, 14 + ipt, dtype=np.uint8).tobytes())
        f[16], f[17] = ipt >> 8, ipt & 0xFF
        frames.append(bytes(f))
    got = inccl.icrc_frames(_rows(frames, gpu, stride)).cpu().numpy().view(np.uint32)
    assert len(got) == count
    for f, c in zip(frames, got):
        assert int(c) == orc.icrc(f), len(f)


MODES = ["split", "batch"]


def _run(sw, mode, fr, pt, tmpl_dev, out_stride=STRIDE, stream=None, out=None, out_len=None):
    """One batch through the switch either way: (action, psn, out, out_len)."""
    if mode == "batch":
        return sw.batch(fr, pt, tmpl_dev, out_stride=out_stride, stream=stream, out=out, out_len=out_len)
    action, psn = sw.ingress(fr, pt, stream=stream)
    out, out_len = sw.egress(fr, pt, action, psn, tmpl_dev, out_stride=out_stride, stream=stream, out=out,
                             out_len=out_len)
    return action, psn, out, out_len


def _templates(fan_in):
    from container_inc_amd.inccl import FRAME_TEMPLATE_DTYPE
    t = np.zeros(fan_in, FRAME_TEMPLATE_DTYPE)
    for c in range(fan_in):
        t[c]["src_mac"] = [0x52, 0x54, 0, 0xAA, 0, c]
        t[c]["dst_mac"] = [0x52, 0x54, 0, 0xBB, 1, c]
        t[c]["src_ip"] = 0x0132320A + (c << 24)
        t[c]["dst_ip"] = 0x0232320A + (c << 24)
        t[c]["src_port"] = 4791
        t[c]["dst_port"] = 4791 + c
        t[c]["qp"] = 0x100 + c
    return t


def _expected_frame(orc, t, c, agg, psn, op, reth):
    wf = op in (0x06, 0x0A)
    return orc.build_data_frame(agg, psn=psn, opcode=op, qp=int(t[c]["qp"]), with_reth=wf,
                                reth=reth if wf else None, src_ip=int(t[c]["src_ip"]), dst_ip=int(t[c]["dst_ip"]),
                                src_port=int(t[c]["src_port"]), dst_port=int(t[c]["dst_port"]),
                                src_mac=bytes(t[c]["src_mac"]), dst_mac=bytes(t[c]["dst_mac"]))


DATA_OPS = (0x00, 0x01, 0x02, 0x04, 0x07, 0x08)   # SEND FIRST/MIDDLE/LAST/ONLY, WRITE MIDDLE/LAST (nts.c:314-319)
WF_OPS = (0x06, 0x0A)                               # WRITE FIRST / ONLY: a RETH before the payload (nts.c:327-328)
ACK = 0x11


def _act_map(orc, inccl):
    return {orc.SW_ABSORBED: inccl.SW_ABSORBED, orc.SW_BROADCAST: inccl.SW_COMPLETED, orc.SW_REPLAY: inccl.SW_REPLAY,
            orc.SW_DROPPED: inccl.SW_DROPPED, orc.SW_ACK: inccl.SW_ACK, orc.SW_IGNORED: inccl.SW_IGNORED,
            orc.SW_INVALID: inccl.SW_INVALID}


def _host_frame(orc, rng, psn, port, op):
    """A frame a host sends the switch: an ACK for `psn`, or a data / WRITE_FIRST
    packet with a random payload (and a random RETH); opcode 0x64 is one
    pipeline() has no case for."""
    if op == ACK:
        return orc.build_ack_frame(psn, qp=0x40 + port, src_ip=0x0A000001 + port)
    pay = rng.integers(INT32_MIN, INT32_MAX, 256, dtype=np.int64, endpoint=True).astype(np.int32)
    wf = op in WF_OPS
    f = orc.build_data_frame(pay, psn=psn, opcode=0x07 if op == 0x64 else op, qp=0x11, with_reth=wf,
                             reth=rng.integers(0, 256, 16, dtype=np.uint8).tobytes() if wf else None,
                             src_ip=0x0A000001 + port)
    if op == 0x64:
        f = f[:42] + bytes([0x64]) + f[43:]
    return f


def _random_op(rng):
    r = rng.random()
    return int(rng.choice(WF_OPS)) if r < 0.3 else int(rng.choice(DATA_OPS))


def _check_vs_pipeline(orc, inccl, ref, tmpl, frames, ports, stride, action, out, out_len, tag):
    """Every frame of the batch through the oracle's serial pipeline()
    (orc_switch_pipeline, nts.c:303-501 frames in -> frames out): the GPU's
    action, and every row it sent (or did not), byte for byte.  Returns how
    often each oracle action occurred."""
    amap = _act_map(orc, inccl)
    fan = ref.fan_in
    seen = {}
    for i, (f, port) in enumerate(zip(frames, ports)):
        rc, outs = ref.pipeline(tmpl, port, f, stride)
        seen[rc] = seen.get(rc, 0) + 1
        assert int(action[i]) == amap[rc], (tag, i, port, f[42], int(action[i]), amap[rc])
        for c in range(fan):
            row = i * fan + c
            if outs[c] is None:
                assert out_len[row] == 0, (tag, i, c)
            else:
                assert out_len[row] == len(outs[c]), (tag, i, c, int(out_len[row]), len(outs[c]))
                assert bytes(out[row, : len(outs[c])]) == outs[c], (tag, i, c)
    return seen


# 20 children: RETH words of children 16+ are loaded directly, not shuffled from the prefetch.
# Stride 1100 (4-byte but not 16-byte aligned rows): ingress's 2-byte payload
# loads and egress's dword stores instead of the 16-byte paths.
# Fan-in 2, 3, 4 and 8 take egress instances with the children loop unrolled, others the loop; frames
# arrive shuffled, so a PSN's copies span frame pairs (the sum reads them through their keys).
# Every copy of a frame carries its own opcode -- SEND, WRITE and WRITE_FIRST / ONLY
# mixed within one PSN -- and ACKs, frames with an opcode the switch ignores and
# frames on a port past fan_in are interleaved; the expected actions and frames
# come from the oracle's serial pipeline() on the same sequence.
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("fan_in,stride", [(1, STRIDE), (2, STRIDE), (3, STRIDE), (4, STRIDE), (8, STRIDE), (20, STRIDE),
                                           (31, STRIDE), (2, 1100), (4, 1100), (8, 1100), (5, 1100)])
def test_switch_batches(gpu, orc, fan_in, stride, mode):
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(100 + fan_in)
    slots, per_batch, batches = 64, 8, 5
    sw = inccl.GpuSwitch(fan_in, slots)
    ref = orc.Switch(fan_in, slots)
    tmpl = _templates(fan_in)
    tmpl_dev = torch.from_numpy(tmpl.view(np.uint8).copy()).to(gpu)
    total = {}
    for b in range(batches):
        keys = [(p, port) for p in range(b * per_batch, (b + 1) * per_batch) for port in range(fan_in)]
        # retransmits: some of this batch's frames twice, and some of the previous batch's
        dups = [keys[i] for i in rng.choice(len(keys), size=len(keys) // 4, replace=False)]
        old = [(p, port) for p in range(max(0, (b - 1) * per_batch), b * per_batch) for port in range(fan_in)]
        olds = [old[i] for i in rng.choice(len(old), size=min(3, len(old)), replace=False)] if old else []
        items = [(p, port, _random_op(rng)) for (p, port) in keys + dups + olds]
        # ACKs for any PSN, frames the switch ignores, a frame on a port past fan_in
        items += [(int(rng.integers(0, 1 << 24)), int(rng.integers(0, fan_in)), ACK) for _ in range(2 * fan_in + 2)]
        items += [(b * per_batch, 0, 0x64), (b * per_batch + 1, fan_in, 0x07)]
        items = [items[i] for i in rng.permutation(len(items))]
        frames = [_host_frame(orc, rng, p, port, op) for (p, port, op) in items]
        ports = [port for (_, port, _) in items]
        fr = _rows(frames, gpu, stride)
        pt = torch.tensor(ports, dtype=torch.int32, device=gpu)
        action, psn_out, out, out_len = _run(sw, mode, fr, pt, tmpl_dev, out_stride=stride)
        torch.cuda.synchronize()
        action, psn_out = action.cpu().numpy(), psn_out.cpu().numpy()
        out, out_len = out.cpu().numpy(), out_len.cpu().numpy()
        for i, (p, port, op) in enumerate(items):
            if port < fan_in:
                assert psn_out[i] == p, (i, p)
        for k, v in _check_vs_pipeline(orc, inccl, ref, tmpl, frames, ports, stride, action, out, out_len, b).items():
            total[k] = total.get(k, 0) + v
    want = [orc.SW_BROADCAST, orc.SW_REPLAY, orc.SW_ACK, orc.SW_IGNORED, orc.SW_INVALID]
    if fan_in > 1:   # (one child: every first copy completes its PSN)
        want += [orc.SW_ABSORBED, orc.SW_DROPPED]
    for k in want:
        assert total.get(k, 0) > 0, (k, total)
    sw.destroy()


def test_switch_rejects_bad_frames(gpu, orc):
    import torch
    from container_inc_amd import inccl
    sw = inccl.GpuSwitch(2, 16)
    good = orc.build_data_frame(np.ones(256, np.int32), psn=3, opcode=0x07)
    short = orc.build_data_frame(np.ones(100, np.int32), psn=4, opcode=0x07)   # payload != 1024 B (nts.c:350)
    ack = bytearray(good[:62])
    ack[42] = 0x11
    frames = _rows([good, short, bytes(ack), good], gpu)
    ports = torch.tensor([0, 1, 0, 5], dtype=torch.int32, device=gpu)
    action, _ = sw.ingress(frames, ports)
    assert action.cpu().tolist() == [inccl.SW_ABSORBED, inccl.SW_INVALID, inccl.SW_ACK, inccl.SW_INVALID]
    sw.destroy()


# Batches far larger than one round of the persistent egress grid (about 4096
# waves): many rounds, load batches of several rounds, a partial last round, and
# the per-round rotation of each wave's frame offset wrapping.  Every emitted
# row is checked (length, payload = htonl of the wrap-around sum, ICRC), and a
# sample of rows including the batch's last ones byte-exact against the oracle.
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("fan_in,P", [(2, 40000), (3, 21111), (4, 9999)])
def test_switch_large_batch_all_frames(gpu, orc, fan_in, P, mode):
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(300 + fan_in)
    n = fan_in * P
    base = {op: np.frombuffer(orc.build_data_frame(np.zeros(256, np.int32), psn=0, opcode=op, qp=0x11,
                                                   with_reth=(op == 0x06), reth=bytes(16) if op == 0x06 else None),
                              np.uint8) for op in (0x06, 0x07, 0x08)}
    psn = np.repeat(np.arange(P, dtype=np.uint32), fan_in)
    port = np.tile(np.arange(fan_in, dtype=np.int32), P)
    perm = rng.permutation(n)                      # arrivals interleaved across PSNs and ports
    psn, port = psn[perm], port[perm]
    op_of = np.array([0x06, 0x07, 0x07, 0x08], np.uint8)[psn % 4]
    pay = rng.integers(INT32_MIN, INT32_MAX, (n, 256), dtype=np.int64, endpoint=True).astype(np.int32)
    reth = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    frames = np.zeros((n, STRIDE), np.uint8)
    for op in (0x06, 0x07, 0x08):
        idx = np.nonzero(op_of == op)[0]
        frames[idx, : len(base[op])] = base[op]
        off = 70 if op == 0x06 else 54
        if op == 0x06:
            frames[idx, 54:70] = reth[idx]
        frames[idx, off:off + 1024] = pay[idx].astype(">i4").view(np.uint8).reshape(len(idx), 1024)
        frames[idx, 50:54] = (psn[idx] | 0x80000000).astype(">u4").view(np.uint8).reshape(len(idx), 4)
    sw = inccl.GpuSwitch(fan_in, 1 << (int(np.ceil(np.log2(P))) + 1))
    tmpl = _templates(fan_in)
    tmpl_dev = torch.from_numpy(tmpl.view(np.uint8).copy()).to(gpu)
    fr = torch.from_numpy(frames).to(gpu)
    pt = torch.from_numpy(port).to(gpu)
    action, psn_out, out, out_len = _run(sw, mode, fr, pt, tmpl_dev)
    torch.cuda.synchronize()
    act = action.cpu().numpy()
    assert np.array_equal(psn_out.cpu().numpy(), psn)
    done = act == inccl.SW_COMPLETED
    assert done.sum() == P and np.array_equal(np.sort(psn[done]), np.arange(P))
    assert (act[~done] == inccl.SW_ABSORBED).all()
    # the wrap-around sum of every PSN (nts.c:361-363)
    agg = np.zeros((P, 256), np.uint32)
    np.add.at(agg, psn, pay.view(np.uint32))
    ln = out_len.cpu().numpy().reshape(n, fan_in)
    wf = op_of == 0x06
    want_len = np.where(wf, 1098, 1082)
    assert (ln[~done] == 0).all()
    assert (ln[done] == want_len[done][:, None]).all()
    rows = (np.nonzero(done)[0][:, None] * fan_in + np.arange(fan_in)[None, :]).reshape(-1)
    o = out.view(-1, out.shape[-1])[torch.from_numpy(rows).to(gpu)]
    oc = o.cpu().numpy()
    row_frame = rows // fan_in
    off = np.where(wf[row_frame], 70, 54)
    for d in (54, 70):
        sel = off == d
        got = oc[sel, d:d + 1024].copy().view(">u4").astype(np.uint32)
        assert np.array_equal(got, agg[psn[row_frame[sel]]])
    lens = want_len[row_frame]
    crc_stored = np.array([int.from_bytes(oc[i, lens[i] - 4:lens[i]].tobytes(), "little") for i in range(len(rows))],
                          np.uint32)
    crc = inccl.icrc_frames(o).cpu().numpy().view(np.uint32)
    assert np.array_equal(crc, crc_stored)
    # byte-exact sample: the batch's last emitted rows and random ones
    src_row = {(int(p), int(c)): i for i, (p, c) in enumerate(zip(psn, port))}
    sample = list(range(len(rows) - 2 * fan_in, len(rows))) + [int(x) for x in rng.choice(len(rows), 40, replace=False)]
    for j in sample:
        f, c = int(row_frame[j]), int(rows[j] % fan_in)
        p = int(psn[f])
        want = _expected_frame(orc, tmpl, c, agg[p].view(np.int32), p, int(op_of[f]),
                               reth[src_row[(p, c)]].tobytes())
        assert bytes(oc[j, : len(want)]) == want, (j, f, c)
    sw.destroy()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("fan_in,seed", [(2, 1), (2, 2), (3, 3)])
def test_switch_serial_order_vs_oracle_reference_ring(gpu, orc, fan_in, seed, mode):
    """The reference's own ring (16 slots, window 8 with slot psn+8 cleared at
    completion, nts.c:21-25, :367) fed one frame sequence: the oracle's
    pipeline() processes it serially, the GPU in batches of at most eight
    consecutive PSNs.  Every copy of a frame carries a DIFFERENT payload and its
    own opcode, so the actions, which copy is counted (and whose RETH is kept),
    which opcode each broadcast and replay carries, and every emitted frame must
    all agree.  Retransmits land before, at and after their PSN's completion;
    ACKs are reflected in between."""
    stride = 1100 if seed == 2 else STRIDE   # seed 2: rows 4- but not 16-byte aligned
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(700 + seed)
    assert orc.SW_SLOTS == 16
    sw = inccl.GpuSwitch(fan_in, 16)
    ref = orc.Switch(fan_in)
    tmpl = _templates(fan_in)
    tmpl_dev = torch.from_numpy(tmpl.view(np.uint8).copy()).to(gpu)
    total = {}
    for b in range(12):
        new = list(range(4 * b, 4 * b + 4))
        recent = list(range(max(0, 4 * b - 4), 4 * b + 4))   # at most eight consecutive PSNs
        seq = [(p, c) for p in new for c in range(fan_in)]
        seq = [seq[i] for i in rng.permutation(len(seq))]
        # retransmits spliced in at random positions: before and after completion
        for _ in range(3 * fan_in):
            p, c = int(rng.choice(recent)), int(rng.integers(0, fan_in))
            seq.insert(int(rng.integers(0, len(seq) + 1)), (p, c))
        items = [(p, c, _random_op(rng)) for (p, c) in seq]
        for _ in range(fan_in):
            items.insert(int(rng.integers(0, len(items) + 1)), (int(rng.choice(recent)), int(rng.integers(0, fan_in)), ACK))
        frames = [_host_frame(orc, rng, p, c, op) for (p, c, op) in items]
        ports = [c for (_, c, _) in items]
        fr = _rows(frames, gpu, stride)
        pt = torch.tensor(ports, dtype=torch.int32, device=gpu)
        action, psn_out, out, out_len = _run(sw, mode, fr, pt, tmpl_dev, out_stride=stride)
        torch.cuda.synchronize()
        act, out, out_len = action.cpu().numpy(), out.cpu().numpy(), out_len.cpu().numpy()
        for k, v in _check_vs_pipeline(orc, inccl, ref, tmpl, frames, ports, stride, act, out, out_len, b).items():
            total[k] = total.get(k, 0) + v
    for k in (orc.SW_BROADCAST, orc.SW_REPLAY, orc.SW_DROPPED, orc.SW_ACK):
        assert total.get(k, 0) > 0, total   # every serial outcome occurred
    sw.destroy()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("fan_in", [3, 16, 20])
def test_switch_arrivals_in_same_parity_batches(gpu, orc, fan_in, mode):
    """A PSN whose counted arrivals fall in batches g and g + 2 with none in
    g + 1 (and again in g + 4): batch g + 2 must classify against the bitmap
    batch g left, whichever of the slot's two arrival words holds it.  The PSN's
    frames in one batch are spread over more than 256 frames (different
    classify blocks and sum waves) by ACK and ignored-opcode fillers, and its
    retransmits of ports counted in batch g come both before and after the
    batch's leader.  Fan-in 16 and 20 take the sum's key path (counted ports from
    the arrival words).  Actions and frames vs the oracle's serial pipeline()."""
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(1500 + fan_in)
    sw = inccl.GpuSwitch(fan_in, 16)
    ref = orc.Switch(fan_in)
    tmpl = _templates(fan_in)
    tmpl_dev = torch.from_numpy(tmpl.view(np.uint8).copy()).to(gpu)

    def fill(n):
        return [(int(rng.integers(0, 1 << 24)), int(rng.integers(0, fan_in)), ACK if rng.random() < 0.5 else 0x64)
                for _ in range(n)]

    half = fan_in // 2
    P, Q = 5, 6            # PSN 5 spans batches; PSN 6 completes in the batches between (recycles slot 14)
    plan = [
        # batch g: half of P's ports, far apart
        [it for c in range(half) for it in [(P, c, _random_op(rng))] + fill(150)],
        # batch g + 1: Q completes; nothing for P
        [(Q, c, _random_op(rng)) for c in range(fan_in)] + fill(300),
        # batch g + 2: retransmits of g's ports, then the rest of P's ports (the
        # leader is the lowest of them), then more retransmits after it
        fill(20) + [(P, 0, _random_op(rng))] + fill(280) +
        [it for c in range(half, fan_in - 1) for it in [(P, c, _random_op(rng))] + fill(40)] +
        [(P, c, _random_op(rng)) for c in range(half)] + fill(300) + [(P, c, _random_op(rng)) for c in range(half)],
        # batch g + 3: nothing for P
        fill(100) + [(Q, 0, _random_op(rng))],
        # batch g + 4: P's last port completes it, retransmits after it replay
        fill(10) + [(P, half, _random_op(rng))] + fill(300) + [(P, fan_in - 1, _random_op(rng))] + fill(270) +
        [(P, c, _random_op(rng)) for c in range(fan_in)],
        # batch g + 5: only retransmits of P
        [(P, c, _random_op(rng)) for c in range(fan_in)] + fill(300) + [(P, 0, _random_op(rng))],
    ]
    total = {}
    for b, items in enumerate(plan):
        frames = [_host_frame(orc, rng, p, c, op) for (p, c, op) in items]
        ports = [c for (_, c, _) in items]
        fr = _rows(frames, gpu)
        pt = torch.tensor(ports, dtype=torch.int32, device=gpu)
        action, _, out, out_len = _run(sw, mode, fr, pt, tmpl_dev)
        torch.cuda.synchronize()
        act, out, out_len = action.cpu().numpy(), out.cpu().numpy(), out_len.cpu().numpy()
        for k, v in _check_vs_pipeline(orc, inccl, ref, tmpl, frames, ports, STRIDE, act, out, out_len, b).items():
            total[k] = total.get(k, 0) + v
        assert np.array_equal(inccl_slot(sw, P, gpu), ref.slot(P)), b
    assert total.get(orc.SW_DROPPED, 0) >= 2 * half and total.get(orc.SW_REPLAY, 0) >= fan_in, total
    sw.destroy()


def test_switch_short_stride_rejected(gpu, orc):
    """A frame's header may claim more bytes than its row holds: the row stride
    bounds every read (a payload past the row is INVALID; an ICRC whose IP
    length runs past the row is not computed), and strides below the 62-B ACK
    frame are refused on the host."""
    import torch
    from container_inc_amd import inccl
    sw = inccl.GpuSwitch(2, 16)
    good = orc.build_data_frame(np.ones(256, np.int32), psn=3, opcode=0x07)   # 1082 B
    rows = np.zeros((2, 1024), np.uint8)                                      # rows shorter than the frame
    rows[0] = np.frombuffer(good[:1024], np.uint8)
    rows[1] = np.frombuffer(good[:1024], np.uint8)
    fr = torch.from_numpy(rows).to(gpu)
    action, _ = sw.ingress(fr, torch.tensor([0, 1], dtype=torch.int32, device=gpu))
    assert action.cpu().tolist() == [inccl.SW_INVALID, inccl.SW_INVALID]
    crc = inccl.icrc_frames(fr).cpu().numpy()
    assert (crc == 0).all()
    with pytest.raises(inccl.IncclError):
        inccl.icrc_frames(torch.zeros((4, 32), dtype=torch.uint8, device=gpu))
    with pytest.raises(inccl.IncclError):
        sw.ingress(torch.zeros((4, 32), dtype=torch.uint8, device=gpu), torch.zeros(4, dtype=torch.int32, device=gpu))
    sw.destroy()


@pytest.mark.parametrize("mode", MODES)
def test_switch_batch_graph_replay(gpu, orc, mode):
    """One batch's launches (claim, classify, sum, egress -- from the ingress +
    egress calls or from the batch call) captured once in a hipGraph and
    replayed over new frame contents: the batch generation is a device word
    that claim and classify advance, so every replay is a new batch (first-copy
    keys of the previous replay never count).  Batches
    alternate between the two halves of the PSN ring (each recycles the other's
    slots, nts.c:367); every replay's actions, payload sums and ICRCs are
    checked, then eager calls continue on the same state."""
    import torch
    from container_inc_amd import inccl
    fan_in, P = 2, 3000
    rng = np.random.default_rng(900)
    slots = 2 * (1 << int(np.ceil(np.log2(P))))
    half = slots // 2
    base = {op: np.frombuffer(orc.build_data_frame(np.zeros(256, np.int32), psn=0, opcode=op, qp=0x11,
                                                   with_reth=(op == 0x06), reth=bytes(16) if op == 0x06 else None),
                              np.uint8) for op in (0x06, 0x07, 0x08)}
    n = fan_in * P
    port = np.tile(np.arange(fan_in, dtype=np.int32), P)

    def batch(b):
        psn = np.repeat(np.arange(P, dtype=np.uint32), fan_in) + (half if b % 2 else 0)
        op_of = np.array([0x06, 0x07, 0x07, 0x08], np.uint8)[psn % 4]
        pay = rng.integers(INT32_MIN, INT32_MAX, (n, 256), dtype=np.int64, endpoint=True).astype(np.int32)
        frames = np.zeros((n, STRIDE), np.uint8)
        for op in (0x06, 0x07, 0x08):
            idx = np.nonzero(op_of == op)[0]
            frames[idx, : len(base[op])] = base[op]
            off = 70 if op == 0x06 else 54
            frames[idx, off:off + 1024] = pay[idx].astype(">i4").view(np.uint8).reshape(len(idx), 1024)
            frames[idx, 50:54] = (psn[idx] | 0x80000000).astype(">u4").view(np.uint8).reshape(len(idx), 4)
        return psn, op_of, pay, frames

    def check(psn, op_of, pay, action, psn_out, out, out_len):
        act = action.cpu().numpy()
        assert np.array_equal(psn_out.cpu().numpy(), psn)
        done = act == inccl.SW_COMPLETED
        assert done.sum() == P and (act[~done] == inccl.SW_ABSORBED).all()
        agg = (pay[0::2].view(np.uint32).astype(np.uint64) + pay[1::2].view(np.uint32)).astype(np.uint32)
        ln = out_len.cpu().numpy().reshape(n, fan_in)
        assert (ln[~done] == 0).all()
        rows = (np.nonzero(done)[0][:, None] * fan_in + np.arange(fan_in)[None, :]).reshape(-1)
        oc = out[torch.from_numpy(rows).to(gpu)].cpu().numpy()
        wf = op_of[rows // fan_in] == 0x06
        for d in (54, 70):
            sel = np.where(wf, 70, 54) == d
            got = oc[sel, d:d + 1024].copy().view(">u4").astype(np.uint32)
            assert np.array_equal(got, agg[(psn[rows // fan_in][sel] % half).astype(np.int64)])
        crc = inccl.icrc_frames(torch.from_numpy(oc).to(gpu)).cpu().numpy().view(np.uint32)
        lens = np.where(wf, 1098, 1082)
        stored = np.array([int.from_bytes(oc[i, lens[i] - 4:lens[i]].tobytes(), "little") for i in range(len(rows))],
                          np.uint32)
        assert np.array_equal(crc, stored)

    sw = inccl.GpuSwitch(fan_in, slots)
    tmpl_dev = torch.from_numpy(_templates(fan_in).view(np.uint8).copy()).to(gpu)
    fr = torch.zeros((n, STRIDE), dtype=torch.uint8, device=gpu)
    pt = torch.from_numpy(port).to(gpu)
    out = torch.zeros((n * fan_in, STRIDE), dtype=torch.uint8, device=gpu)
    out_len = torch.zeros(n * fan_in, dtype=torch.int32, device=gpu)
    st = torch.cuda.Stream(device=gpu)
    # one eager batch first (b = 0), then the captured one replayed for b = 1..4
    psn, op_of, pay, frames = batch(0)
    fr.copy_(torch.from_numpy(frames))
    torch.cuda.synchronize()
    a, q, _, _ = _run(sw, mode, fr, pt, tmpl_dev, stream=st, out=out, out_len=out_len)
    torch.cuda.synchronize()
    check(psn, op_of, pay, a, q, out, out_len)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        ga, gq, _, _ = _run(sw, mode, fr, pt, tmpl_dev, stream=st, out=out, out_len=out_len)
    for b in range(1, 5):
        psn, op_of, pay, frames = batch(b)
        fr.copy_(torch.from_numpy(frames))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        check(psn, op_of, pay, ga, gq, out, out_len)
    # eager again on the same state (b = 5)
    psn, op_of, pay, frames = batch(5)
    fr.copy_(torch.from_numpy(frames))
    torch.cuda.synchronize()
    a, q, _, _ = _run(sw, mode, fr, pt, tmpl_dev, stream=st, out=out, out_len=out_len)
    torch.cuda.synchronize()
    check(psn, op_of, pay, a, q, out, out_len)
    del g
    sw.destroy()


@pytest.mark.parametrize("fan_in", [2, 3])
def test_switch_split_and_batch_agree(gpu, orc, fan_in):
    """The two ways of driving the switch, fed the same frame sequence on two
    switches: identical actions, PSNs, out rows (every emitted byte) and
    lengths, batch after batch, with retransmits spread across waves (random
    arrival order) and PSNs whose ports straddle batches."""
    import torch
    rng = np.random.default_rng(1300 + fan_in)
    from container_inc_amd import inccl
    slots = 64
    sws = {m: inccl.GpuSwitch(fan_in, slots) for m in MODES}
    tmpl_dev = torch.from_numpy(_templates(fan_in).view(np.uint8).copy()).to(gpu)
    pending = []
    for b in range(8):
        keys = [(p, c) for p in range(4 * b, 4 * b + 6) for c in range(fan_in)]
        keys = [k for k in keys if k not in pending]
        carry = [keys[i] for i in rng.choice(len(keys), size=len(keys) // 3, replace=False)]   # arrive next batch
        now = [k for k in keys if k not in carry] + pending
        now += [now[i] for i in rng.choice(len(now), size=len(now) // 4, replace=False)]     # retransmits
        now = [now[i] for i in rng.permutation(len(now))]
        pending = carry
        frames = []
        for (p, c) in now:
            op = [0x06, 0x07, 0x07, 0x08][p % 4]
            pay = rng.integers(INT32_MIN, INT32_MAX, 256, dtype=np.int64, endpoint=True).astype(np.int32)
            frames.append(orc.build_data_frame(pay, psn=p, opcode=op, qp=0x11, with_reth=op == 0x06,
                                               reth=rng.integers(0, 256, 16, dtype=np.uint8).tobytes() if op == 0x06 else None))
        fr = _rows(frames, gpu)
        pt = torch.tensor([c for (_, c) in now], dtype=torch.int32, device=gpu)
        res = {}
        for m in MODES:
            a, q, o, ln = _run(sws[m], m, fr, pt, tmpl_dev,
                               out=torch.zeros((len(now) * fan_in, STRIDE), dtype=torch.uint8, device=gpu))
            torch.cuda.synchronize()
            res[m] = (a.cpu().numpy(), q.cpu().numpy(), o.cpu().numpy(), ln.cpu().numpy())
        for x, y in zip(res["split"], res["batch"]):
            assert np.array_equal(x, y), b
        for p in sorted({p for (p, _) in now}):
            assert np.array_equal(inccl_slot(sws["split"], p, gpu), inccl_slot(sws["batch"], p, gpu)), (b, p)
    for sw in sws.values():
        sw.destroy()


def inccl_slot(sw, psn, dev):
    """The aggregator words of `psn`'s slot (inccl_switch_slot), as uint32."""
    import ctypes
    import torch
    from container_inc_amd._lib import load, runtime_libs
    ptr = load().inccl_switch_slot(sw.handle, ctypes.c_uint32(psn))
    buf = torch.empty(256, dtype=torch.int32, device=dev)
    hip = ctypes.CDLL(runtime_libs()["libamdhip64"])   # the HIP runtime this process already runs on
    torch.cuda.synchronize()
    assert hip.hipMemcpy(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(ptr), ctypes.c_size_t(1024), 3) == 0
    return buf.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("mode", MODES)
def test_switch_slot_after_recycle(gpu, orc, mode):
    """inccl_switch_slot's documented behaviour around a recycle (nts.c:235-242,
    :367): while a PSN's slot holds arrivals its words are the wrap-around sum
    so far; completing PSN p recycles slot p + slots/2, whose words are then
    stale (the GPU does not zero them, unlike the reference's memset); the next
    counted arrival into that slot sums from zero, not from the stale words."""
    import torch
    from container_inc_amd import inccl
    fan_in, slots = 2, 16
    sw = inccl.GpuSwitch(fan_in, slots)
    tmpl_dev = torch.from_numpy(_templates(fan_in).view(np.uint8).copy()).to(gpu)
    rng = np.random.default_rng(1400)

    def frame(p, pay):
        return orc.build_data_frame(pay, psn=p, opcode=0x07, qp=0x11)

    def send(items):
        fr = _rows([frame(p, pay) for (p, _, pay) in items], gpu)
        pt = torch.tensor([c for (_, c, _) in items], dtype=torch.int32, device=gpu)
        a, _, _, _ = _run(sw, mode, fr, pt, tmpl_dev)
        torch.cuda.synchronize()
        return a.cpu().numpy().tolist()

    pay = {k: rng.integers(INT32_MIN, INT32_MAX, 256, dtype=np.int64, endpoint=True).astype(np.int32)
           for k in [(9, 0), (9, 1), (1, 0), (1, 1), (25, 0), (25, 1)]}
    # PSN 9 (slot 9) completes: its words are the sum
    assert send([(9, 0, pay[(9, 0)]), (9, 1, pay[(9, 1)])]) == [inccl.SW_ABSORBED, inccl.SW_COMPLETED]
    want9 = orc.sum_q32([pay[(9, 0)], pay[(9, 1)]]).view(np.uint32)
    assert np.array_equal(inccl_slot(sw, 9, gpu), want9)
    # PSN 1 completes and recycles slot 1 + 8 = 9: the words stay (stale)
    assert send([(1, 0, pay[(1, 0)]), (1, 1, pay[(1, 1)])]) == [inccl.SW_ABSORBED, inccl.SW_COMPLETED]
    assert np.array_equal(inccl_slot(sw, 9, gpu), want9)
    # PSN 25 -> slot 9 again: its first counted arrival sums from zero
    assert send([(25, 1, pay[(25, 1)])]) == [inccl.SW_ABSORBED]
    assert np.array_equal(inccl_slot(sw, 25, gpu), pay[(25, 1)].view(np.uint32))
    assert send([(25, 0, pay[(25, 0)])]) == [inccl.SW_COMPLETED]
    assert np.array_equal(inccl_slot(sw, 25, gpu), orc.sum_q32([pay[(25, 0)], pay[(25, 1)]]).view(np.uint32))
    sw.destroy()
