"""Where a small eager fused reduce's time goes, from Python (N = 1, R = 2,
k = 25): host wall time per call over back-to-back calls on one stream (one
synchronisation at the end), for 4 KiB .. 4 MiB buckets, through each layer:

  eager      inccl.reduce_f32 (argument checks + ctypes marshalling + C + launch)
  marshal    the Python side of that call alone (checks, pointer array, stream
             handle; no ctypes call)
  ctypes     inccl_stream_op through ctypes with every argument built beforehand
  prepared   inccl.prepare_reduce_f32(...)() = one inccl_op_run ctypes call
  graph1     a hipGraph holding one call, replayed once per call (torch.cuda.CUDAGraph)
  graph20    a hipGraph holding 20 calls, per call (device rate of back-to-back kernels)

One JSON line per size.  tools/call_overhead.c measures the same from C."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_call(fn, iters, sync):
    for _ in range(max(10, iters // 10)):
        fn()
    sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    sync()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    import torch
    from container_inc_amd import inccl
    from container_inc_amd._lib import load
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    st = torch.cuda.Stream(device=dev)
    h = st.cuda_stream
    lib = load()
    iters = int(os.environ.get("ITERS", "3000"))
    for b in (4 << 10, 64 << 10, 1 << 20, 4 << 20):
        n = b // 4
        xs = [torch.randn(n, device=dev) for _ in range(2)]
        out = torch.empty(n, device=dev)
        torch.cuda.synchronize()
        sync = torch.cuda.synchronize
        row = {"bucket_bytes": b, "R": 2}
        row["eager_us"] = per_call(lambda: inccl.reduce_f32(xs, 25, out=out, stream=h), iters, sync)

        def marshal():   # stream_op's Python work without the library call
            srcs = list(xs)
            ptrs = [inccl._dev_ptr(s, torch.float32, f"srcs[{i}]", n) for i, s in enumerate(srcs)]
            inccl._dev_ptr(out, torch.float32, "out", n)
            inccl._check_scale(25)
            inccl._ptr_array(ptrs)
            inccl._stream_handle(h)
        row["marshal_us"] = per_call(marshal, iters, lambda: None)
        arr = inccl._ptr_array([x.data_ptr() for x in xs])
        args = (0, 0, arr, 2, ctypes.c_void_p(out.data_ptr()), ctypes.c_size_t(n), 25, None, 2, ctypes.c_void_p(h))
        f = lib.inccl_stream_op
        row["ctypes_us"] = per_call(lambda: f(*args), iters, sync)
        op = inccl.prepare_reduce_f32(xs, 25, out=out, stream=h)
        row["prepared_us"] = per_call(op, iters, sync)
        for per in (1, 20):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                for _ in range(per):
                    inccl.reduce_f32(xs, 25, out=out, stream=h)
            row[f"graph{per}_us"] = per_call(g.replay, max(100, iters // per), sync) / per
            del g
        op.destroy()
        print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in row.items()}), flush=True)


if __name__ == "__main__":
    main()
