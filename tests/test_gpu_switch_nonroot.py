"""The non-root switch on the GPU (inccl_switch_create_nonroot;
non_termination_switch.c:376-400, :408-423, :457-499) against the oracle's
serial pipeline() (gpu): every frame's action and every row it sends, byte for
byte, in both driving modes (split ingress + egress, and one batch call), with
the reference's byte order and no-recycle (flags 0) and with each option.

Parity of the non-root role rests on the oracle restatement (the reference
needs libpcap to build): tests/test_oracle_nonroot.py checks it on hand-worked
sequences and against the one reference-produced output SURVEY §0 recorded
(tests/golden/nonroot_down_survey.json), which the GPU reproduces too."""
import numpy as np
import pytest

from test_gpu_switch import ACK, MODES, STRIDE, _host_frame, _random_op, _rows, _run, _templates

pytestmark = pytest.mark.gpu
INT32_MIN, INT32_MAX = -(2 ** 31), 2 ** 31 - 1


def _amap(orc, inccl):
    return {orc.SW_ABSORBED: inccl.SW_ABSORBED, orc.SW_BROADCAST: inccl.SW_COMPLETED, orc.SW_REPLAY: inccl.SW_REPLAY,
            orc.SW_DROPPED: inccl.SW_DROPPED, orc.SW_ACK: inccl.SW_ACK, orc.SW_IGNORED: inccl.SW_IGNORED,
            orc.SW_INVALID: inccl.SW_INVALID, orc.SW_FORWARD: inccl.SW_FORWARD, orc.SW_DOWN: inccl.SW_DOWN}


def _check(orc, inccl, ref, tmpl, frames, ports, stride, action, out, out_len, tag):
    amap = _amap(orc, inccl)
    rows = ref.rows
    seen = {}
    for i, (f, port) in enumerate(zip(frames, ports)):
        rc, outs = ref.pipeline(tmpl, port, f, stride)
        seen[rc] = seen.get(rc, 0) + 1
        assert int(action[i]) == amap[rc], (tag, i, port, f[42], int(action[i]), amap[rc])
        for c in range(rows):
            row = i * rows + c
            if outs[c] is None:
                assert out_len[row] == 0, (tag, i, c, int(out_len[row]))
            else:
                assert out_len[row] == len(outs[c]), (tag, i, c, int(out_len[row]), len(outs[c]))
                assert bytes(out[row, : len(outs[c])]) == outs[c], (tag, i, c)
    return seen


def _batch_items(rng, fan_in, psns, prev):
    """One batch: every child's first copy of each PSN, retransmits (enough
    for the resend rule's degree % fan_in == 0), copies of the parent's result
    (some before the children complete), ACKs from children and the parent,
    an opcode the switch ignores, a port past the parent; shuffled."""
    F = fan_in
    items = [(p, c, _random_op(rng)) for p in psns for c in range(F)]
    items += [(int(rng.choice(psns)), int(rng.integers(0, F)), _random_op(rng)) for _ in range(len(psns) * F // 2)]
    items += [(int(p), F, _random_op(rng)) for p in psns for _ in range(int(rng.integers(0, 3)))]
    if prev:   # late copies of the previous batch's PSNs, from children and the parent
        items += [(int(rng.choice(prev)), int(rng.integers(0, F + 1)), _random_op(rng)) for _ in range(4)]
    items += [(int(rng.integers(0, 1 << 24)), int(rng.integers(0, F + 1)), ACK) for _ in range(F + 2)]
    items += [(psns[0], 0, 0x64), (psns[0], F + 1, 0x07)]
    return [items[i] for i in rng.permutation(len(items))]


# flags: 0 = the reference (reversed downstream words, no recycle), 1 wire order, 2 recycle, 3 both.
# Fan-in 2, 3, 4 and 8 take the unrolled egress; 1, 5, 20, 31 the loop (20, 31: the parent's
# RETH past the 16 children the keeper prefetch covers).  Stride 1100: 4-byte aligned rows.
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("fan_in,stride,flags", [(2, STRIDE, 0), (2, STRIDE, 1), (2, STRIDE, 2), (3, STRIDE, 3),
                                                 (1, STRIDE, 0), (4, 1100, 0), (8, STRIDE, 2), (5, 1100, 1),
                                                 (20, STRIDE, 0), (31, STRIDE, 3)])
def test_nonroot_batches(gpu, orc, fan_in, stride, flags, mode):
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(500 + 17 * fan_in + flags)
    slots, per_batch, batches = 64, 8, 5
    sw = inccl.GpuSwitch(fan_in, slots, nonroot=True, flags=flags)
    ref = orc.Switch(fan_in, slots, nonroot=True, flags=flags)
    tmpl = _templates(fan_in + 1)
    tmpl_dev = torch.from_numpy(tmpl.view(np.uint8).copy()).to(gpu)
    total = {}
    prev = []
    for b in range(batches):
        psns = list(range(b * per_batch, (b + 1) * per_batch))
        items = _batch_items(rng, fan_in, psns, prev)
        prev = psns
        frames = [_host_frame(orc, rng, p, port, op) for (p, port, op) in items]
        ports = [port for (_, port, _) in items]
        fr = _rows(frames, gpu, stride)
        pt = torch.tensor(ports, dtype=torch.int32, device=gpu)
        action, psn_out, out, out_len = _run(sw, mode, fr, pt, tmpl_dev, out_stride=stride)
        torch.cuda.synchronize()
        action, psn_out = action.cpu().numpy(), psn_out.cpu().numpy()
        out, out_len = out.cpu().numpy(), out_len.cpu().numpy()
        for i, (p, port, op) in enumerate(items):
            if port <= fan_in:
                assert psn_out[i] == p, (i, p)
        for k, v in _check(orc, inccl, ref, tmpl, frames, ports, stride, action, out, out_len, b).items():
            total[k] = total.get(k, 0) + v
    want = [orc.SW_FORWARD, orc.SW_DOWN, orc.SW_REPLAY, orc.SW_DROPPED, orc.SW_ACK, orc.SW_IGNORED, orc.SW_INVALID]
    if fan_in > 1:
        want.append(orc.SW_ABSORBED)
    for k in want:
        assert total.get(k, 0) > 0, (k, total)
    sw.destroy()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("flags", [0, 2])
def test_nonroot_reference_ring_reuse(gpu, orc, flags, mode):
    """The reference's 16-slot ring past its first 16 PSNs: without recycling
    (the reference) PSN p + 16 meets p's bits and result, and every copy of it
    is answered from p's slot; with SW_RECYCLE it starts afresh.  Batches of 4
    PSNs (span below slots / 2 with the late copies), PSNs 0..39."""
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(600 + flags)
    F = 2
    sw = inccl.GpuSwitch(F, 16, nonroot=True, flags=flags)
    ref = orc.Switch(F, 16, nonroot=True, flags=flags)
    tmpl = _templates(F + 1)
    tmpl_dev = torch.from_numpy(tmpl.view(np.uint8).copy()).to(gpu)
    prev = []
    total = {}
    for b in range(10):
        psns = list(range(4 * b, 4 * b + 4))
        items = _batch_items(rng, F, psns, prev)
        items += [(p, F, 0x07) for p in psns]   # a result for every PSN after its children
        prev = psns
        frames = [_host_frame(orc, rng, p, port, op) for (p, port, op) in items]
        ports = [port for (_, port, _) in items]
        action, psn_out, out, out_len = _run(sw, mode, _rows(frames, gpu), torch.tensor(ports, dtype=torch.int32,
                                                                                       device=gpu), tmpl_dev)
        torch.cuda.synchronize()
        for k, v in _check(orc, inccl, ref, tmpl, frames, ports, STRIDE, action.cpu().numpy(), out.cpu().numpy(),
                           out_len.cpu().numpy(), b).items():
            total[k] = total.get(k, 0) + v
    if flags == 0:   # PSNs 16..39: stale slots, no first copy counts
        assert total[orc.SW_REPLAY] > total.get(orc.SW_ABSORBED, 0)
    sw.destroy()


def test_nonroot_result_slot_and_sums(gpu, orc):
    """A large batch (fan-in 2, 12 000 PSNs, every child's copy then the
    parent's result): every PSN forwards the wrap-around sum once, every result
    is taken, the parent rows carry htonl(sum), the child rows the result with
    each word's bytes reversed (the reference), and inccl_switch_result holds
    the parent's wire words."""
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(700)
    F, P = 2, 12000
    base = np.frombuffer(orc.build_data_frame(np.zeros(256, np.int32), psn=0, opcode=0x07, qp=0x11), np.uint8)
    n = (F + 1) * P
    psn = np.repeat(np.arange(P, dtype=np.uint32), F + 1)
    port = np.tile(np.arange(F + 1, dtype=np.int32), P)   # children first, then the parent, per PSN
    pay = rng.integers(INT32_MIN, INT32_MAX, (n, 256), dtype=np.int64, endpoint=True).astype(np.int32)
    frames = np.zeros((n, STRIDE), np.uint8)
    frames[:, : len(base)] = base
    frames[:, 54:54 + 1024] = pay.astype(">i4").view(np.uint8).reshape(n, 1024)
    frames[:, 50:54] = (psn | 0x80000000).astype(">u4").view(np.uint8).reshape(n, 4)
    sw = inccl.GpuSwitch(F, 1 << 15, nonroot=True)
    tmpl = _templates(F + 1)
    tmpl_dev = torch.from_numpy(tmpl.view(np.uint8).copy()).to(gpu)
    action, psn_out, out, out_len = sw.batch(torch.from_numpy(frames).to(gpu), torch.from_numpy(port).to(gpu), tmpl_dev)
    torch.cuda.synchronize()
    act = action.cpu().numpy().reshape(P, F + 1)
    assert (act[:, 0] == inccl.SW_ABSORBED).all() and (act[:, 1] == inccl.SW_FORWARD).all()
    assert (act[:, 2] == inccl.SW_DOWN).all()
    ln = out_len.cpu().numpy().reshape(P, F + 1, F + 1)
    assert (ln[:, 0] == 0).all()
    assert (ln[:, 1, :F] == 0).all() and (ln[:, 1, F] == 1082).all()
    assert (ln[:, 2, :F] == 1082).all() and (ln[:, 2, F] == 0).all()
    o = out.view(P, F + 1, F + 1, -1)
    agg = pay.reshape(P, F + 1, 256)[:, :F].view(np.uint32).sum(axis=1, dtype=np.uint64).astype(np.uint32)
    up = o[:, 1, F, 54:54 + 1024].cpu().numpy().copy().view(">u4").astype(np.uint32)
    assert np.array_equal(up, agg)
    y = pay.reshape(P, F + 1, 256)[:, F]
    for c in range(F):
        dn = o[:, 2, c, 54:54 + 1024].cpu().numpy().copy().view("<u4")   # bytes reversed: little-endian reads y
        assert np.array_equal(dn, y.view(np.uint32)), c
    crc = inccl.icrc_frames(o[:, 2, 0].contiguous()).cpu().numpy().view(np.uint32)
    stored = o[:, 2, 0, 1078:1082].cpu().numpy().copy().view("<u4").ravel()
    assert np.array_equal(crc, stored)
    for p in (0, 1, P - 1, int(rng.integers(0, P))):   # the result slot: the wire words, as nts.c:413 keeps them
        ptr = sw.result_ptr(p)
        import ctypes
        from container_inc_amd._lib import runtime_libs
        buf = torch.empty(256, dtype=torch.int32, device=gpu)
        hip = ctypes.CDLL(runtime_libs()["libamdhip64"])
        assert hip.hipMemcpy(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(ptr), ctypes.c_size_t(1024), 3) == 0
        torch.cuda.synchronize()
        want = np.frombuffer(y[p].astype(">i4").tobytes(), "<i4")
        assert np.array_equal(buf.cpu().numpy(), want), p
    sw.destroy()


def test_nonroot_graph_replay(gpu, orc):
    """A non-root batch captured into a hipGraph (after an uncaptured batch as
    large, which sizes the list links) and replayed with new frames each time:
    the same actions and rows as the oracle's serial pipeline()."""
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(800)
    F, per = 3, 6
    sw = inccl.GpuSwitch(F, 64, nonroot=True, flags=inccl.SW_RECYCLE)
    ref = orc.Switch(F, 64, nonroot=True, flags=orc.SW_RECYCLE)
    tmpl = _templates(F + 1)
    tmpl_dev = torch.from_numpy(tmpl.view(np.uint8).copy()).to(gpu)

    def make(b, prev):
        psns = list(range(b * per, (b + 1) * per))
        items = _batch_items(rng, F, psns, prev)[:48]
        items += [(psns[0], 0, ACK)] * (48 - len(items))
        return psns, items

    psns, items = make(0, [])
    frames = [_host_frame(orc, rng, p, port, op) for (p, port, op) in items]
    ports = [port for (_, port, _) in items]
    fr, pt = _rows(frames, gpu), torch.tensor(ports, dtype=torch.int32, device=gpu)
    action, psn_out, out, out_len = sw.batch(fr, pt, tmpl_dev)
    torch.cuda.synchronize()
    _check(orc, inccl, ref, tmpl, frames, ports, STRIDE, action.cpu().numpy(), out.cpu().numpy(),
           out_len.cpu().numpy(), 0)
    st = torch.cuda.Stream(device=gpu)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        sw.batch(fr, pt, tmpl_dev, stream=st, out=out, out_len=out_len, action=action, psn=psn_out)
    prev = psns
    for b in range(1, 5):
        psns, items = make(b, prev)
        prev = psns
        frames = [_host_frame(orc, rng, p, port, op) for (p, port, op) in items]
        ports = [port for (_, port, _) in items]
        fr.copy_(_rows(frames, gpu))
        pt.copy_(torch.tensor(ports, dtype=torch.int32, device=gpu))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        _check(orc, inccl, ref, tmpl, frames, ports, STRIDE, action.cpu().numpy(), out.cpu().numpy(),
               out_len.cpu().numpy(), b)
    sw.destroy()


@pytest.mark.parametrize("flags", [1, 3])
def test_two_tier_tree_on_gpu(gpu, orc, flags):
    """Eight hosts, four fan-in-2 non-root switches and a fan-in-4 root, all on
    the GPU, 4 096 PSNs per round: the hosts' frames -> each leaf (up batch) ->
    the leaves' FORWARD rows -> the root (one batch, port = leaf) -> the root's
    COMPLETED rows -> each leaf (port 2, down batch) -> the DOWN rows -> the
    hosts.  Every host row carries the eight-way wrap-around sum in wire order
    (SW_WIRE_ORDER; with SW_RECYCLE too for flags 3) with a valid ICRC; two
    rounds on consecutive PSN ranges, WRITE_FIRST and WRITE_MIDDLE opcodes."""
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(900 + flags)
    H, F, L, P = 8, 2, 4, 4096
    leaves = [inccl.GpuSwitch(F, 4 * P, nonroot=True, flags=flags) for _ in range(L)]
    root = inccl.GpuSwitch(L, 4 * P)
    t_leaf = torch.from_numpy(_templates(F + 1).view(np.uint8).copy()).to(gpu)
    t_root = torch.from_numpy(_templates(L).view(np.uint8).copy()).to(gpu)
    base = {op: np.frombuffer(orc.build_data_frame(np.zeros(256, np.int32), psn=0, opcode=op, with_reth=op == 0x06,
                                                   reth=bytes(16) if op == 0x06 else None), np.uint8)
            for op in (0x06, 0x07)}
    for rnd in range(2):
        psn0 = rnd * P
        pay = rng.integers(INT32_MIN, INT32_MAX, (H, P, 256), dtype=np.int64, endpoint=True).astype(np.int32)
        total = pay.view(np.uint32).sum(axis=0, dtype=np.uint64).astype(np.uint32)   # [P, 256]
        ops = np.where(np.arange(P) % 2 == 0, 0x06, 0x07).astype(np.uint8)
        fwd_rows = []
        for l in range(L):   # up: each leaf's two hosts, PSN-major
            n = F * P
            fr = np.zeros((n, STRIDE), np.uint8)
            psn = np.repeat(np.arange(P, dtype=np.uint32) + psn0, F)
            host = np.tile(np.arange(F), P) + F * l
            for op in (0x06, 0x07):
                sel = np.repeat(ops == op, F)
                fr[sel, : len(base[op])] = base[op]
                off = 70 if op == 0x06 else 54
                fr[sel, off:off + 1024] = pay[host[sel], psn[sel] - psn0].astype(">i4").view(np.uint8).reshape(-1, 1024)
            fr[:, 50:54] = (psn | 0x80000000).astype(">u4").view(np.uint8).reshape(n, 4)
            ports = torch.from_numpy(np.tile(np.arange(F, dtype=np.int32), P)).to(gpu)
            a, _, out, ln = leaves[l].batch(torch.from_numpy(fr).to(gpu), ports, t_leaf)
            torch.cuda.synchronize()
            fw = np.nonzero(a.cpu().numpy() == inccl.SW_FORWARD)[0]
            assert len(fw) == P
            fwd_rows.append(out[torch.from_numpy(fw * (F + 1) + F).to(gpu)])
        # the root: the leaves' forwards interleaved PSN by PSN, port = leaf
        rf = torch.stack(fwd_rows, dim=1).reshape(L * P, STRIDE)
        rp = torch.from_numpy(np.tile(np.arange(L, dtype=np.int32), P)).to(gpu)
        a, _, out, ln = root.batch(rf, rp, t_root)
        torch.cuda.synchronize()
        done = np.nonzero(a.cpu().numpy() == inccl.SW_COMPLETED)[0]
        assert len(done) == P
        for l in range(L):   # down: the root's frames for leaf l into its parent port
            dn = out[torch.from_numpy(done * L + l).to(gpu)]
            a2, _, out2, ln2 = leaves[l].batch(dn.contiguous(), torch.full((P,), F, dtype=torch.int32, device=gpu),
                                               t_leaf)
            torch.cuda.synchronize()
            assert (a2.cpu().numpy() == inccl.SW_DOWN).all()
            hosts = out2.view(P, F + 1, STRIDE)[:, :F].cpu().numpy()
            lens = ln2.cpu().numpy().reshape(P, F + 1)
            wf = ops == 0x06
            assert (lens[:, :F] == np.where(wf, 1098, 1082)[:, None]).all() and (lens[:, F] == 0).all()
            for d in (54, 70):
                sel = np.where(wf, 70, 54) == d
                got = hosts[sel, :, d:d + 1024].copy().view(">u4").astype(np.uint32)   # [p, child, 256]
                assert np.array_equal(got, np.repeat(total[sel][:, None, :], F, axis=1)), (rnd, l, d)
            rows = torch.from_numpy(hosts.reshape(P * F, STRIDE)).to(gpu)
            crc = inccl.icrc_frames(rows).cpu().numpy().view(np.uint32)
            ln_flat = lens[:, :F].reshape(-1)
            stored = np.array([int.from_bytes(hosts.reshape(P * F, STRIDE)[i, ln_flat[i] - 4:ln_flat[i]].tobytes(),
                                              "little") for i in range(P * F)], np.uint32)
            assert np.array_equal(crc, stored)
    for sw in leaves + [root]:
        sw.destroy()


def test_nonroot_down_matches_surveyed_reference_output(gpu, orc):
    """SURVEY §0's reference-produced output for a non-root (a child decodes
    234881024 where the parent sent 14, tests/golden/nonroot_down_survey.json)
    on the GPU switch with the reference's byte order (flags 0), and the
    parent's 14 with SW_WIRE_ORDER."""
    import json
    import os

    import torch
    from conftest import GOLDEN
    from container_inc_amd import inccl
    g = json.load(open(os.path.join(GOLDEN, "nonroot_down_survey.json")))
    for flags, want in ((0, g["child_value"]), (inccl.SW_WIRE_ORDER, g["parent_value"])):
        sw = inccl.GpuSwitch(2, 16, nonroot=True, flags=flags)
        tmpl = torch.from_numpy(_templates(3).view(np.uint8).copy()).to(gpu)
        frames = [orc.build_data_frame(np.arange(256, dtype=np.int32), psn=3, opcode=0x07) for _ in range(2)]
        frames.append(orc.build_data_frame(np.full(256, g["parent_value"], np.int32), psn=3, opcode=0x07))
        a, _, out, ln = sw.batch(_rows(frames, gpu), torch.tensor([0, 1, 2], dtype=torch.int32, device=gpu), tmpl)
        torch.cuda.synchronize()
        assert a.cpu().tolist() == [inccl.SW_ABSORBED, inccl.SW_FORWARD, inccl.SW_DOWN]
        o = out.cpu().numpy()
        for c in range(2):
            got = o[2 * 3 + c, 54:54 + 1024].copy().view(">i4")
            assert (got == want).all(), (flags, c)
        sw.destroy()
