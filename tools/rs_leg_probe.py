"""bench.py's reduce_scatter key alone (reduce_scatter_engines: 256 MiB on
rccl / p2p / mesh, then 64 KiB and 1 MiB on rccl / p2p / ll), repeated, with
the bench's own setup: a gloo process group, the communicator created on the
automatic engine (on one GPU RCCL refuses and every rank falls back to p2p).
Every rank on device 0.  Rank 0 prints one JSON line per row.

    python -m torch.distributed.run --nproc-per-node W --master-addr 127.0.0.1 \\
        tools/rs_leg_probe.py [REPEATS] [--no-rccl] [--digits]

--digits: the same call pattern on data whose base-8 digits name each rank's
contribution (digits_leg), so a wrong element says whose partial was wrong.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def digits_leg(comm, dev, rank: int, world: int, mib: float, engines) -> list:
    """reduce_scatter_engines' call pattern (per engine: inputs A, B, A with a
    synchronisation and a copy after each, then 15 more calls; gloo between
    engines) on data that names its sender: rank r's buckets quantise (k = 20)
    to d * 8^r with d in 1..3 (set A) or 4..6 (set B), so each base-8 digit of a
    reduced element is one rank's contribution.  A wrong element decodes to the
    digit of every rank: 0 = that rank's partial was missing (zero), a set-B
    digit in a set-A call = a stale partial of the other set."""
    import torch
    import torch.distributed as dist
    n = int(mib * (1 << 20)) // 4
    n -= n % (world * 64)
    shard = n // world
    i = torch.arange(n, device=dev, dtype=torch.int64)
    sets = []
    for base in (1, 4):
        d = ((i % 3) + base).to(torch.float32)
        x = d * float(8 ** rank) * 2.0 ** -20
        want = torch.zeros(n, device=dev, dtype=torch.float64)
        for r in range(world):
            want += d.double() * float(8 ** r)
        sets.append(([x, torch.zeros_like(x)], (want * 2.0 ** -20).float()[rank * shard:(rank + 1) * shard]))
    out = torch.empty(shard, device=dev)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    rows = []
    for eng in engines:
        row = {"engine": eng, "mib": mib, "calls": []}
        try:
            comm.set_engine(eng)
            for call, si in enumerate((0, 1, 0) + (0,) * 15):
                xs, want = sets[si]
                comm.reduce_scatter(xs, out=out, scale_exp=20, stream=st.cuda_stream)
                torch.cuda.synchronize()
                bad = (out != want).nonzero().flatten()
                if bad.numel():
                    e = int(bad[0])
                    g = int(round(float(out[e]) * 2 ** 20))
                    w = int(round(float(want[e]) * 2 ** 20))
                    row["calls"].append({"call": call, "set": "AB"[si], "bad": int(bad.numel()), "first": e,
                                         "got_digits": [(g >> (3 * r)) & 7 for r in range(world)],
                                         "want_digits": [(w >> (3 * r)) & 7 for r in range(world)]})
        except Exception as ex:  # noqa: BLE001
            row["error"] = repr(ex)[:200]
        everyone = [None] * world
        dist.all_gather_object(everyone, row)
        rows.append({"engine": eng, "mib": mib, "bad_ranks": {r: x["calls"] for r, x in enumerate(everyone) if x["calls"]},
                     "errors": {r: x["error"] for r, x in enumerate(everyone) if "error" in x}})
    return rows


def main():
    repeats = int(next((a for a in sys.argv[1:] if not a.startswith("--")), "2"))
    no_rccl = "--no-rccl" in sys.argv
    digits = "--digits" in sys.argv
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    os.environ.setdefault("INCCL_BOOT_TIMEOUT", "120")
    import torch
    import torch.distributed as dist
    import bench
    from container_inc_amd import inccl
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    port = int(os.environ.get("MASTER_PORT", "29500")) + 17
    grp = inccl.inccl_group_create(world, rank, os.environ.get("MASTER_ADDR", "127.0.0.1"), port=port, device=0)
    comm = inccl.inccl_communicator_create(grp, 0)
    big = ("p2p", "mesh") if no_rccl else ("rccl", "p2p", "mesh")
    small = ("p2p", "ll") if no_rccl else ("rccl", "p2p", "ll")
    if digits:
        for rep in range(repeats):
            rows = digits_leg(comm, dev, rank, world, 256, big)
            for mib in (1 / 16, 1.0):
                rows += digits_leg(comm, dev, rank, world, mib, small)
            if rank == 0:
                for r in rows:
                    print(json.dumps({"rep": rep, **r}), flush=True)
        comm.destroy()
        grp.destroy()
        dist.destroy_process_group()
        return
    if "--bench-digits" in sys.argv:   # bench.reduce_scatter_engines itself on digit-coded data (k = 25)
        def sets(mib):
            n = int(mib * (1 << 20)) // 4
            i = torch.arange(n, device=dev, dtype=torch.int64)
            out = []
            for base in (1, 4):
                d = ((i % 3) + base).to(torch.float32)
                out.append([d * float(8 ** rank) * 2.0 ** -25, torch.zeros(n, device=dev)])
            torch.cuda.synchronize()
            return out

        def decode(t, mib, eng):
            n = int(mib * (1 << 20)) // 4
            shard = n // world
            i = torch.arange(rank * shard, (rank + 1) * shard, device=dev, dtype=torch.int64)
            want = torch.zeros(shard, device=dev, dtype=torch.float64)
            for r in range(world):
                want += ((i % 3) + 1).double() * float(8 ** r)
            got = torch.round(t.double() * 2.0 ** 25)
            bad = (got != want).nonzero().flatten()
            rec = {"engine": eng, "mib": mib, "rank": rank, "bad": int(bad.numel())}
            if bad.numel():
                e = int(bad[0])
                g, w = int(got[e]), int(want[e])
                rec.update(first=e, got_digits=[(g >> (3 * r)) & 7 for r in range(world)],
                           want_digits=[(w >> (3 * r)) & 7 for r in range(world)])
                # how many bad elements, per rank-digit position that is wrong
                gi = got[bad].to(torch.int64)
                wi = want[bad].to(torch.int64)
                rec["wrong_digit_counts"] = [int(((gi >> (3 * r)) & 7).ne((wi >> (3 * r)) & 7).sum()) for r in range(world)]
            return rec

        for rep in range(repeats):
            for mib, engs in ((256, big), (1 / 16, small), (1.0, small)):
                firsts = {}
                rows = bench.reduce_scatter_engines(comm, dev, 2, rank, world, mib, engs, inputs=sets(mib),
                                                    first_out=firsts)
                recs = [decode(t, mib, eng) for eng, t in firsts.items()]
                everyone = [None] * world
                dist.all_gather_object(everyone, recs)
                if rank == 0:
                    for rr in everyone:
                        for r in rr:
                            if r["bad"]:
                                print(json.dumps({"rep": rep, **r}), flush=True)
                    print(json.dumps({"rep": rep, "mib": mib, "rows": [(x["engine"], x["ok"], x["bit_identical"]) for x in rows]}), flush=True)
        comm.destroy()
        grp.destroy()
        dist.destroy_process_group()
        return
    for rep in range(repeats):
        rows = bench.reduce_scatter_engines(comm, dev, 2, rank, world, engines=big)
        for mib in (1 / 16, 1.0):
            rows += bench.reduce_scatter_engines(comm, dev, 2, rank, world, mib, small)
        if rank == 0:
            for r in rows:
                p = r.get("parity_vs_oracle") or {}
                p3 = r.get("parity_vs_oracle_call3") or {}
                print(json.dumps({"rep": rep, "engine": r["engine"], "mib": r["bucket_mib"], "ok": r["ok"],
                                  "identical": r["bit_identical"], "bad": p.get("mismatches"),
                                  "bad_by_rank": p.get("mismatches_by_rank"), "bad_call3": p3.get("mismatches")}),
                      flush=True)
    comm.destroy()
    grp.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
