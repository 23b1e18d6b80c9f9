"""Where the N = 1 step loses time beyond the kernel: back-to-back eager launches
of the fused kernel vs the same launches replayed from one hipGraph, per-launch
event time.  The rocprofv3 kernel duration is the floor both approach.

    python tools/gap_probe.py [--mib 256] [--iters 50]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mib", type=int, default=256)
    p.add_argument("--iters", type=int, default=50)
    p.add_argument("--R", type=int, default=2)
    a = p.parse_args()
    import torch
    import container_inc_amd
    from container_inc_amd import inccl
    container_inc_amd.load()
    dev = torch.device("cuda:0")
    n = a.mib * (1 << 20) // 4
    g = torch.Generator(device=dev).manual_seed(1000)
    xs = [torch.randn(n, generator=g, device=dev) for _ in range(a.R)]
    out = torch.empty(n, device=dev)
    st = torch.cuda.Stream(device=dev)
    alg = (a.R + 1) * 4 * n

    def timed(fn, reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    def launch():
        inccl.reduce_f32(xs, 25, out=out, stream=st.cuda_stream)

    for _ in range(5):
        launch()
    torch.cuda.synchronize()
    ref = out.clone()
    rows = []
    for rep in range(3):
        ms = timed(launch, a.iters) / a.iters
        rows.append({"mode": "eager", "rep": rep, "us_per_launch": round(ms * 1e3, 2),
                     "GBs": round(alg / (ms * 1e-3) / 1e9, 1)})
    # one launch bracketed by its own events
    singles = []
    for _ in range(10):
        singles.append(timed(launch, 1))
    rows.append({"mode": "single", "us_min": round(min(singles) * 1e3, 2),
                 "us_med": round(sorted(singles)[5] * 1e3, 2)})
    # hipGraph of iters launches
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        torch.cuda.synchronize()
        graph.capture_begin()
        for _ in range(a.iters):
            inccl.reduce_f32(xs, 25, out=out, stream=torch.cuda.current_stream().cuda_stream)
        graph.capture_end()
    torch.cuda.synchronize()
    out.zero_()
    with torch.cuda.stream(st):
        graph.replay()
    torch.cuda.synchronize()
    same = bool(torch.equal(out, ref))
    for rep in range(3):
        with torch.cuda.stream(st):
            ms = timed(graph.replay, 1) / a.iters
        rows.append({"mode": "graph", "rep": rep, "us_per_launch": round(ms * 1e3, 2),
                     "GBs": round(alg / (ms * 1e-3) / 1e9, 1), "bit_identical": same})
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
