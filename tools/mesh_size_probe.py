"""Two ranks on one GPU: mesh / meshw engine call times as the bucket grows
(regrowth included), one line per call.  argv: engine sizes_mib...
Environment INCCL_IPC_MEM selects the IPC buffer kind."""
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rank_main(rank, port, engine, sizes):
    os.environ["INCCL_ENGINE"] = engine
    os.environ["INCCL_DEVICE"] = "0"
    os.environ.setdefault("INCCL_LL_TIMEOUT_MS", "2000")
    sys.path.insert(0, ROOT)
    import torch
    from container_inc_amd import inccl
    dev = torch.device("cuda:0")
    grp = inccl.inccl_group_create(2, rank, "127.0.0.1", port=port)
    comm = inccl.inccl_communicator_create(grp, 0)
    for mib in sizes:
        n = (mib << 20) // 4
        xs = [torch.randn(n, device=dev) for _ in range(2)]
        out = torch.empty(n, device=dev)
        torch.cuda.synchronize()
        for i in range(4):
            t0 = time.perf_counter()
            comm.allreduce_f32(xs, out=out, scale_exp=24, stream=comm.stream)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if rank == 0:
                print(f"{engine} {os.environ.get('INCCL_IPC_MEM', 'default')} {mib} MiB call {i}: {dt * 1e3:.2f} ms",
                      flush=True)
        del xs, out
    if rank == 0:
        print("kind", comm.ipc_mem_kind(engine), flush=True)
    comm.destroy()
    grp.destroy()


if __name__ == "__main__":
    engine = sys.argv[1]
    sizes = [int(s) for s in sys.argv[2:]]
    ctx = mp.get_context("spawn")
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ps = [ctx.Process(target=rank_main, args=(r, port, engine, sizes)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join()
    sys.exit(max(p.exitcode or 0 for p in ps))
