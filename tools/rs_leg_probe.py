"""bench.py's reduce_scatter key alone (reduce_scatter_engines: 256 MiB on
rccl / p2p / mesh, then 64 KiB and 1 MiB on rccl / p2p / ll), repeated, with
the bench's own setup: a gloo process group, the communicator created on the
automatic engine (on one GPU RCCL refuses and every rank falls back to p2p).
Every rank on device 0.  Rank 0 prints one JSON line per row.

    python -m torch.distributed.run --nproc-per-node W --master-addr 127.0.0.1 \\
        tools/rs_leg_probe.py [REPEATS] [--no-rccl]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    repeats = int(next((a for a in sys.argv[1:] if not a.startswith("--")), "2"))
    no_rccl = "--no-rccl" in sys.argv
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
