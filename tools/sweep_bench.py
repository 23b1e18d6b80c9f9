"""Bucket-size sweep on one GPU (BASELINE config 5, single-GPU leg): fused
quantise+sum+dequantise of R=2 buckets from 4 KiB (one reference message,
api.h:39) to 256 MiB; eager launches vs hipGraph replay (torch.cuda.CUDAGraph
capturing the C-ABI call on its stream).  One JSON line per size."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import container_inc_amd
    from container_inc_amd import inccl
    container_inc_amd.load()
    dev = torch.device("cuda:0")
    R = 2
    sizes = [4 << 10]
    while sizes[-1] < (256 << 20):
        sizes.append(sizes[-1] * 4)
    for b in sizes:
        n = b // 4
        xs = [torch.randn(n, device=dev) for _ in range(R)]
        out = torch.empty(n, device=dev)
        st = torch.cuda.Stream(device=dev)
        iters = 200 if b <= (16 << 20) else 30
        with torch.cuda.stream(st):
            for _ in range(5):
                inccl.reduce_f32(xs, 25, out=out, stream=st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(iters):
                inccl.reduce_f32(xs, 25, out=out, stream=st.cuda_stream)
            e1.record(st)
        torch.cuda.synchronize()
        eager_us = e0.elapsed_time(e1) * 1e3 / iters
        # graph: capture `per` calls, replay
        per = 20
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(per):
                inccl.reduce_f32(xs, 25, out=out, stream=st.cuda_stream)
        torch.cuda.synchronize()
        reps = max(2, iters // per)
        with torch.cuda.stream(st):
            g.replay()
            e0.record(st)
            for _ in range(reps):
                g.replay()
            e1.record(st)
        torch.cuda.synchronize()
        graph_us = e0.elapsed_time(e1) * 1e3 / (reps * per)
        alg = (R + 1) * b
        print(json.dumps({"bucket_bytes": b, "R": R, "eager_us": round(eager_us, 2), "graph_us": round(graph_us, 2),
                          "eager_GBs_alg": round(alg / eager_us / 1e3, 1),
                          "graph_GBs_alg": round(alg / graph_us / 1e3, 1)}), flush=True)
        del g


if __name__ == "__main__":
    main()
