"""Run one hot-path kernel K times on resident buffers -- the command profiled
by rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE) and used for tuning sweeps.

    python tools/kernel_probe.py --kernel fused --R 2 --mib 256 --iters 20
    python tools/kernel_probe.py --kernel fused --R 2 --mib 256 --sets 4   # cold: four sets rotated
    python tools/kernel_probe.py --sweep
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--kernel", default="fused", choices=["fused", "quant_sum", "dequant", "sum_q32", "absmax", "quantise", "bf16", "f16"])
    p.add_argument("--R", type=int, default=2)
    p.add_argument("--mib", type=int, default=256)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--grid-cap", type=int, default=0)
    p.add_argument("--no-nt", action="store_true")
    p.add_argument("--sweep", action="store_true")
    p.add_argument("--sets", type=int, default=1,
                   help="fused: rotate this many independent input/output sets (cold when they exceed the caches)")
    a = p.parse_args()
    import torch
    import container_inc_amd
    from container_inc_amd import inccl
    container_inc_amd.load()
    dev = torch.device("cuda:0")
    n = a.mib * (1 << 20) // 4
    R = a.R
    g = torch.Generator(device=dev).manual_seed(1000)
    sets = [[torch.randn(n, generator=g, device=dev) for _ in range(R)] for _ in range(max(1, a.sets))]
    xs = sets[0]
    outs = [torch.empty(n, device=dev) for _ in range(max(1, a.sets))]
    turn = [0]
    qs = [torch.randint(-2 ** 26, 2 ** 26, (n,), device=dev, dtype=torch.int32) for _ in range(R)]
    outf = torch.empty(n, device=dev)
    outq = torch.empty(n, device=dev, dtype=torch.int32)
    n16 = a.mib * (1 << 20) // 2   # bf16 / fp16 buckets of the same size in bytes
    dt16 = torch.float16 if a.kernel == "f16" else torch.bfloat16
    is16 = a.kernel in ("bf16", "f16")
    hs = [torch.randn(n16, generator=g, device=dev).to(dt16) for _ in range(R)] if is16 else []
    outh = torch.empty(n16, device=dev, dtype=dt16) if is16 else None
    st = torch.cuda.Stream(device=dev)

    def run(kind):
        s = st.cuda_stream
        if kind == "fused":
            i = turn[0] % len(sets)
            turn[0] += 1
            inccl.reduce_f32(sets[i], 25, out=outs[i], stream=s)
        elif kind == "quant_sum":
            inccl.quant_sum(xs, 25, out=outq, stream=s)
        elif kind == "quantise":
            inccl.quantise(xs[0], 25, out=outq, stream=s)
        elif kind == "dequant":
            inccl.dequantise(qs[0], 25, out=outf, stream=s)
        elif kind == "sum_q32":
            inccl.sum_q32(qs, out=outq, stream=s)
        elif kind == "absmax":
            inccl.absmax_word(xs, stream=s)
        elif kind == "bf16":
            inccl.reduce_bf16(hs, 25, out=outh, stream=s)
        elif kind == "f16":
            inccl.reduce_f16(hs, 25, out=outh, stream=s)

    def alg_bytes(kind):
        return {"fused": (R + 1) * 4 * n, "quant_sum": (R + 1) * 4 * n, "quantise": 8 * n, "dequant": 8 * n,
                "sum_q32": (R + 1) * 4 * n, "absmax": R * 4 * n, "bf16": (R + 1) * 2 * n16, "f16": (R + 1) * 2 * n16}[kind]

    def timeit(kind, iters):
        for _ in range(3):
            run(kind)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(iters):
            run(kind)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        return ms, alg_bytes(kind) / (ms * 1e-3) / 1e9

    if a.sweep:
        res = []
        for nt in (True, False):
            for cap in (512, 1024, 2048, 4096, 8192, 1 << 30):
                inccl.set_tuning(cap, nt)
                for kind in ("fused",):
                    ms, gbs = timeit(kind, a.iters)
                    res.append({"kernel": kind, "nt": nt, "grid_cap": cap, "ms": round(ms, 5), "GBs": round(gbs, 1)})
                    print(json.dumps(res[-1]), flush=True)
        inccl.set_tuning(0, True)
        for kind in ("fused", "quant_sum", "quantise", "dequant", "sum_q32", "absmax"):
            ms, gbs = timeit(kind, a.iters)
            print(json.dumps({"kernel": kind, "default": True, "ms": round(ms, 5), "GBs": round(gbs, 1)}), flush=True)
        return
    inccl.set_tuning(a.grid_cap, not a.no_nt)
    ms, gbs = timeit(a.kernel, a.iters)
    print(json.dumps({"kernel": a.kernel, "R": R, "n": n, "sets": a.sets, "ms": round(ms, 5), "GBs": round(gbs, 1),
                      "frac": round(gbs / 8000.0, 4), "alg_bytes": alg_bytes(a.kernel)}))


if __name__ == "__main__":
    main()
