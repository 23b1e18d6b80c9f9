"""Throughput of the GPU switch dataplane (non_termination_switch.c:303-501 +
util.c:331-442 on the GPU) vs the oracle's single-core restatement.

Workload: fan_in children x P packets of 1 KiB payload (RoCEv2 frames of 1082 B,
one WRITE_FIRST with RETH every 4th PSN), batches alternating over the two halves of the PSN ring: ingress (parse + serial-order
idempotent add) -> egress (fan_in frames per PSN: build + htonl + ICRC) -> recycle.
Reports payload GB/s = fan_in * P * 1024 / t (ingress payload bytes), frames/s,
for both ways of driving the switch (split: ingress + egress calls; batch: one
inccl_switch_batch call), and the same for the ICRC kernel alone.  CPU leg: oracle orc_switch_ingress +
orc_build_data_frame (the reference's per-packet loop, 1 core)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import container_inc_amd
    from container_inc_amd import inccl
    from oracle import oracle as O
    container_inc_amd.load()
    dev = torch.device("cuda:0")
    fan_in = int(os.environ.get("SW_FAN_IN", "2"))
    P = int(os.environ.get("SW_PSNS", str(1 << 16)))
    stride = 1152
    rng = np.random.default_rng(7)
    # build one template frame per (psn % 4 kind) and patch psn + payload on the GPU side via numpy
    frames = np.zeros((fan_in * P, stride), np.uint8)
    base = {}
    for op in (0x06, 0x07, 0x08):
        base[op] = np.frombuffer(O.build_data_frame(np.zeros(256, np.int32), psn=0, opcode=op, with_reth=(op == 0x06)),
                                 np.uint8)
    pay = rng.integers(-2 ** 31, 2 ** 31 - 1, (fan_in * P, 256), dtype=np.int64).astype(np.int32)
    psn = np.repeat(np.arange(P, dtype=np.uint32), fan_in)
    ports = np.tile(np.arange(fan_in, dtype=np.int32), P)
    for op, sel in ((0x06, psn % 4 == 0), (0x07, (psn % 4 == 1) | (psn % 4 == 2)), (0x08, psn % 4 == 3)):
        idx = np.nonzero(sel)[0]
        b = base[op]
        frames[idx, : len(b)] = b
        off = 70 if op == 0x06 else 54
        frames[idx, off:off + 1024] = pay[idx].astype(">i4").view(np.uint8).reshape(len(idx), 1024)
        p = (psn[idx] | 0x80000000).astype(">u4").view(np.uint8).reshape(len(idx), 4)
        frames[idx, 50:54] = p
    fr = torch.from_numpy(frames).to(dev)
    # a second batch with the next P PSNs: batches alternate between the two
    # halves of the 2P-slot ring, and each batch's recycle (slot psn + slots/2,
    # nts.c:367) clears the other half -- the reference's incremental clearing,
    # so no full-state reset runs between batches
    frames_b = frames.copy()
    frames_b[:, 50:54] = ((psn + P) | 0x80000000).astype(">u4").view(np.uint8).reshape(-1, 4)
    fr_b = torch.from_numpy(frames_b).to(dev)
    del frames_b
    pt = torch.from_numpy(ports).to(dev)
    sw = inccl.GpuSwitch(fan_in, 2 * (1 << int(np.ceil(np.log2(P)))))
    tmpl = np.zeros(fan_in, inccl.FRAME_TEMPLATE_DTYPE)
    tmpl["qp"] = 0x11
    tmpl["src_port"] = 4791
    tmpl["dst_port"] = 4791
    tmpl_dev = torch.from_numpy(tmpl.view(np.uint8).copy()).to(dev)
    st = torch.cuda.Stream(device=dev)
    out = torch.empty((fan_in * P * fan_in, stride), dtype=torch.uint8, device=dev)
    out_len = torch.empty(fan_in * P * fan_in, dtype=torch.int32, device=dev)
    batch = [0]

    def run(mode):
        x = fr if batch[0] % 2 == 0 else fr_b
        batch[0] += 1
        if mode == "batch":
            a, q, o, ln = sw.batch(x, pt, tmpl_dev, stream=st, out=out, out_len=out_len)
            return a, o, ln
        a, q = sw.ingress(x, pt, stream=st)
        o, ln = sw.egress(x, pt, a, q, tmpl_dev, stream=st, out=out, out_len=out_len)
        return a, o, ln

    def check(mode):
        if os.environ.get("SWITCH_BENCH_NOCHECK"):   # timing-only ablations (their frames are wrong on purpose)
            return
        a, o, ln = run(mode)
        torch.cuda.synchronize()
        acts = a.cpu().numpy()
        assert (acts == inccl.SW_COMPLETED).sum() == P, f"{mode}: every psn completes once"
        # spot-check egress frames against the oracle (this batch's PSNs are p or p + P)
        base_psn = 0 if (batch[0] - 1) % 2 == 0 else P
        for f in rng.choice(len(acts), 8, replace=False):
            if acts[f] != inccl.SW_COMPLETED:
                continue
            p = int(psn[f])
            agg = O.sum_q32([pay[p * fan_in + c] for c in range(fan_in)])
            op = 0x06 if p % 4 == 0 else (0x08 if p % 4 == 3 else 0x07)
            want = O.build_data_frame(agg, psn=p + base_psn, opcode=op, qp=0x11, with_reth=(op == 0x06), reth=bytes(16))
            got = o[f * fan_in].cpu().numpy()[: len(want)].tobytes()
            assert got == want, f"{mode}: egress frame {f} differs from the oracle"

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    iters = 10
    payload_bytes = fan_in * P * 1024
    for mode in ("split", "batch"):
        check(mode)
        run(mode)   # the other half of the ring
        with torch.cuda.stream(st):
            e0.record(st)
            for _ in range(iters):
                run(mode)
            e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        check(mode)   # every PSN of every later batch still completes exactly once
        print(json.dumps({"what": "GPU switch dataplane batch, eager: " +
                                  ("inccl_switch_ingress (claim / classify / sum) + inccl_switch_egress" if mode == "split" else
                                   "inccl_switch_batch (claim / classify / sum / egress in one call)"),
                          "mode": mode, "fan_in": fan_in, "psns": P, "ingress_frames": fan_in * P,
                          "egress_frames": fan_in * P, "ms": round(ms, 4),
                          "payload_GBs": round(payload_bytes / (ms * 1e-3) / 1e9, 2),
                          "frames_per_s": round(2 * fan_in * P / (ms * 1e-3), 1)}), flush=True)
        # the same batches captured in a hipGraph (SW_GRAPH_BATCHES batches,
        # even: alternating halves of the ring) and replayed: no launch gaps
        # between the captured kernels, one graph launch per replay
        nb = int(os.environ.get("SW_GRAPH_BATCHES", "2"))
        assert nb >= 2 and nb % 2 == 0, "SW_GRAPH_BATCHES: an even count (the batches alternate ring halves)"
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(nb):
                run(mode)
        g.replay()
        torch.cuda.synchronize()
        reps = 5
        with torch.cuda.stream(st):
            e0.record(st)
            for _ in range(reps):
                g.replay()
            e1.record(st)
        torch.cuda.synchronize()
        ms_g = e0.elapsed_time(e1) / (nb * reps)
        check(mode)   # eager again after the replays: still one completion per PSN
        del g
        print(json.dumps({"what": "GPU switch dataplane batch, hipGraph-replayed", "mode": mode, "batches_per_graph": nb,
                          "fan_in": fan_in, "psns": P, "ms": round(ms_g, 4),
                          "payload_GBs": round(payload_bytes / (ms_g * 1e-3) / 1e9, 2)}), flush=True)
    icrc_out = torch.empty(fan_in * P, dtype=torch.int32, device=dev)
    with torch.cuda.stream(st):
        inccl.icrc_frames(fr, stream=st)
        e0.record(st)
        for _ in range(iters):
            inccl.icrc_frames(fr, stream=st)
        e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    print(json.dumps({"what": "GPU ICRC of 1082/1098-B frames", "frames": fan_in * P, "ms": round(ms, 4),
                      "frame_GBs": round(fan_in * P * 1082 / (ms * 1e-3) / 1e9, 2)}), flush=True)
    del icrc_out
    # CPU: the oracle's per-packet switch + egress framing (1 core), bounded sample
    Pc = min(P, 4096)
    swc = O.Switch(fan_in)
    t0 = time.perf_counter()
    n_eg = 0
    for p in range(Pc):
        for c in range(fan_in):
            f = p * fan_in + c
            body = pay[f].astype(">i4").view(np.uint32)
            rc, eg = swc.ingress(c, p, body)
            if rc == O.SW_BROADCAST:
                agg_host = eg.byteswap().view(np.int32)
                for cc in range(fan_in):
                    O.build_data_frame(agg_host, psn=p, opcode=0x07)
                    n_eg += 1
    dt = time.perf_counter() - t0
    print(json.dumps({"what": "CPU oracle switch (orc_switch_ingress + orc_build_data_frame per egress, 1 core, "
                              "python-driven per packet)", "psns": Pc, "egress_frames": n_eg, "s": round(dt, 3),
                      "payload_GBs": round(fan_in * Pc * 1024 / dt / 1e9, 4)}), flush=True)
    sw.destroy()


if __name__ == "__main__":
    main()
