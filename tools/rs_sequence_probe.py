"""The N > 1 bench's engine sequence (tuning -> 16-bit legs -> reduce-scatter
leg: bench.py main, bf16_engines, reduce_scatter_engines) with exact
fixed-point data, so that every call of every engine is checked exactly on
every rank without the oracle.  One rank per process, started from a shell
(tools/gpu_rs_sequence.sh), every rank on device 0.

    python tools/rs_sequence_probe.py RANK PORT WORLD [MIB] [--rccl] [--random]

--skew: rank 0 starts every step 0.2 s after the others (in the bench, rank 0
runs the oracle check of the previous engine while the others go on).
--bench-like: each step on a new torch side stream with a preallocated out
(bench.py reduce_scatter_engines / bf16_engines), not comm.stream.
--rccl: before each step's engine list, a call on the rccl engine as the bench
makes one (it fails on one GPU: RCCL refuses two ranks on one device; the
error is expected and recorded).  --random: N(0,1) buckets at k = 25, as the
bench, checked against the float64 sum wrapped like the int32 partials
(exact: the partials are integers).

Rank r's buckets are (r + 1) * b and (r + 1) * b / 2 with b[i] = ((i % 4093) -
2046) * 2^-12: every quantised partial and sum is exact at k = 20, so the
reduced bucket is the exact sum (16-bit buckets: the sum of the rounded
inputs, rounded once).  Prints one JSON line per step: engine, op, format,
bytes, and per call the number of wrong elements."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    rank, port, world = int(args[0]), int(args[1]), int(args[2])
    mib = float(args[3]) if len(args) > 3 else 256.0
    with_rccl = "--rccl" in sys.argv
    rand = "--random" in sys.argv
    benchlike = "--bench-like" in sys.argv   # the bench's form: a torch side stream per leg, a preallocated out
    skew = "--skew" in sys.argv   # rank 0 enters each step 0.2 s late (the bench's rank-0 oracle check)
    os.environ.setdefault("INCCL_ENGINE", "p2p")
    os.environ["INCCL_DEVICE"] = "0"
    os.environ.setdefault("INCCL_BOOT_TIMEOUT", "120")
    import torch
    from container_inc_amd import inccl
    dev = torch.device("cuda", 0)
    grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port, device=0)
    comm = inccl.inccl_communicator_create(grp, 0)
    k = 25 if rand else 20
    bad_total = 0
    legs = {}

    def inputs(n, dt):
        if rand:   # every rank regenerates every rank's buckets from its seed
            qs = torch.zeros(n, device=dev, dtype=torch.int64)
            mine = None
            for r in range(world):
                g = torch.Generator(device=dev)
                g.manual_seed(9100 + r)
                xr = [torch.randn(n, generator=g, device=dev).to(dt) for _ in range(2)]
                for x in xr:   # the quantiser: round half to even at 2^-k, saturate to int32
                    q = torch.round(x.double() * 2.0 ** k).clamp(-2 ** 31, 2 ** 31 - 1).to(torch.int64)
                    qs += q
                if r == rank:
                    mine = xr
            qs = ((qs + 2 ** 31) % 2 ** 32 - 2 ** 31)   # int32 wrap-around sum
            want = (qs.double() * 2.0 ** -k).float().to(dt) if dt == torch.float32 else None
            if want is None:   # 16-bit: dequantise in fp32, then round once
                want = (qs.to(torch.float32) * 2.0 ** -k).to(dt)
            torch.cuda.synchronize()
            return mine, want
        i = torch.arange(n, device=dev, dtype=torch.int64)
        b = ((i % 4093) - 2046).to(torch.float32) * 2.0 ** -12
        mine = [(b * float(rank + 1)).to(dt), (b * float(rank + 1) * 0.5).to(dt)]
        acc = torch.zeros(n, device=dev, dtype=torch.float32)
        for r in range(world):
            acc += (b * float(r + 1)).to(dt).float() + (b * float(r + 1) * 0.5).to(dt).float()
        torch.cuda.synchronize()   # made on torch's stream; the calls run on comm.stream
        return mine, acc.to(dt)

    def step(eng, op, dt, nbytes):
        nonlocal bad_total
        es = 4 if dt == torch.float32 else 2
        n = int(nbytes) // es
        n -= n % (world * 64)
        xs, full = inputs(n, dt)
        shard = n // world
        want = full if op == "ar" else full[rank * shard:(rank + 1) * shard]
        row = {"rank": rank, "engine": eng, "op": op, "dtype": str(dt).split(".")[-1], "n": n, "bad": []}
        sh = comm.stream
        pre = None
        if benchlike:   # one stream and one out per leg (op, format, size), shared by its engines
            key = (op, str(dt), n)
            if key not in legs:
                legs.clear()   # the previous leg's stream and out are dropped, as the bench's are
                legs[key] = (torch.cuda.Stream(device=dev), torch.empty(shard if op == "rs" else n, device=dev, dtype=dt))
                torch.cuda.synchronize()
            sh = legs[key][0].cuda_stream
            pre = legs[key][1]
        if skew and rank == 0:
            import time
            time.sleep(0.2)
        try:
            comm.set_engine(eng)
            for _ in range(3):
                if op == "rs":
                    out = comm.reduce_scatter(xs, out=pre, scale_exp=k, stream=sh)
                elif dt == torch.float32:
                    out = comm.allreduce_f32(xs, out=pre, scale_exp=k, stream=sh)
                else:
                    fn = comm.allreduce_bf16 if dt == torch.bfloat16 else comm.allreduce_f16
                    out = fn(xs, out=pre if pre is not None else torch.empty_like(xs[0]), scale_exp=k, stream=sh)
                torch.cuda.synchronize()
                row["bad"].append(int((out != want).sum().item()))
        except Exception as e:  # noqa: BLE001
            row["error"] = repr(e)[:300]
        bad_total += sum(row["bad"])
        print(json.dumps(row), flush=True)

    big = mib * (1 << 20)
    f32, b16, h16 = torch.float32, torch.bfloat16, torch.float16
    rc = ("rccl",) if with_rccl else ()
    for eng in rc + ("p2p", "mesh", "meshw"):            # tuning
        step(eng, "ar", f32, big)
    for dt in (b16, h16):                                # the bf16 / f16 keys
        for eng in rc + ("p2p", "mesh", "meshw"):
            step(eng, "ar", dt, big)
    for eng in rc + ("p2p", "mesh"):                     # the reduce_scatter key
        step(eng, "rs", f32, big)
    for small in (64 << 10, 1 << 20):
        for eng in rc + ("p2p", "ll"):
            step(eng, "rs", f32, small)
    comm.barrier()
    comm.destroy()
    grp.destroy()
    print(json.dumps({"rank": rank, "bad_total": bad_total}), flush=True)


if __name__ == "__main__":
    main()
