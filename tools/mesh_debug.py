"""mesh engine at world 1 on one GPU: which chunks of dst come out wrong, for a
few grid sizes ($INCCL_MESH_GRID) -- a debugging aid."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from container_inc_amd import inccl
    from oracle import oracle as O
    dev = torch.device("cuda:0")
    os.environ["INCCL_MASTER_PORT"] = "0"
    os.environ["INCCL_FORCE_SHARDED"] = "1"
    os.environ["INCCL_LL_MAX_BYTES"] = "0"
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    comm.set_engine("mesh")
    rng = np.random.default_rng(5)
    for n in [int(a) for a in sys.argv[1:]] or [4096, 65536, 1 << 20]:
        xs = [rng.standard_normal(n).astype(np.float32) for _ in range(2)]
        want = O.reduce_f32(xs, 25).view(np.uint32)
        for it in range(3):
            out = torch.full((n,), float("nan"), device=dev)
            try:
                comm.allreduce_f32([torch.from_numpy(x).to(dev) for x in xs], out=out, scale_exp=25)
                torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001
                print(f"n={n} it={it}: raised {e}", flush=True)
                continue
            got = out.cpu().numpy().view(np.uint32)
            bad = np.nonzero(got != want)[0]
            nan = int(np.count_nonzero(np.isnan(out.cpu().numpy())))
            print(f"n={n} it={it}: bad={len(bad)} nan={nan} first={bad[:3].tolist()} last={bad[-3:].tolist()}",
                  flush=True)
            if it == 0 and len(bad):
                g32 = got.view(np.float32)
                w32 = want.view(np.float32)
                a0 = O.reduce_f32([xs[0]], 25)
                a1 = O.reduce_f32([xs[1]], 25)
                for i in bad[:12]:
                    print(f"   i={i} got={g32[i]!r} want={w32[i]!r} x0={xs[0][i]!r} x1={xs[1][i]!r} "
                          f"only0={a0[i]!r} only1={a1[i]!r} nb={g32[max(0, i - 1):i + 2].tolist()} "
                          f"wnb={w32[max(0, i - 1):i + 2].tolist()}", flush=True)
    if os.environ.get("MESH_TIME"):
        # one rank: every chunk's push / reduce / gather runs on this GPU's HBM --
        # the kernel's scheduling and local efficiency without xGMI
        import time
        n = 64 << 20   # 256 MiB
        xs = [torch.randn(n, device=dev) for _ in range(2)]
        out = torch.empty(n, device=dev)
        st = torch.cuda.Stream(device=dev)   # not the null stream: NULL means "the communicator's stream"
        torch.cuda.set_stream(st)
        for _ in range(3):
            comm.allreduce_f32(xs, out=out, scale_exp=25, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            comm.allreduce_f32(xs, out=out, scale_exp=25, stream=torch.cuda.current_stream().cuda_stream)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        want = O.reduce_f32([x.cpu().numpy() for x in xs], 25).view(np.uint32)
        bad = int(np.count_nonzero(out.cpu().numpy().view(np.uint32) != want))
        print(f"time-check bad={bad}", flush=True)
        print(f"time grid={os.environ.get('INCCL_MESH_GRID', 'default')} chunk={os.environ.get('INCCL_MESH_CHUNK', 'default')}"
              f" 256MiB R=2 W=1: {ms * 1e3:.1f} us, {28 * n / ms / 1e6:.0f} GB/s of HBM traffic (28 B/elem)", flush=True)
    comm.destroy()
    grp.destroy()


if __name__ == "__main__":
    main()
