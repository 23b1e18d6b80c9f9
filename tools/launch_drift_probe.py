"""Debugging aid: per-launch time of the fused kernel (R = 2 x 256 MiB) over
long back-to-back runs, issued through the communicator (allreduce_f32) or the
stateless call (reduce_f32), in blocks of 50 launches; HIP events around each
block.  Shows whether launch time drifts with sustained load."""
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
    n = (256 << 20) // 4
    g = torch.Generator(device=dev).manual_seed(1000)
    xs = [torch.randn(n, generator=g, device=dev) for _ in range(2)]
    out = torch.empty(n, device=dev)
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1", device=0)
    comm = inccl.inccl_communicator_create(grp, 0)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    seq = []
    for block in range(int(os.environ.get("BLOCKS", "16"))):
        via = "comm" if (block // 2) % 2 == 0 else "stateless"
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(50):
            if via == "comm":
                comm.allreduce_f32(xs, out=out, scale_exp=25, stream=st.cuda_stream)
            else:
                inccl.reduce_f32(xs, 25, out=out, stream=st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        seq.append({"block": block, "via": via, "us_per_launch": round(e0.elapsed_time(e1) * 1e3 / 50, 2)})
    print(json.dumps(seq), flush=True)
    comm.destroy()
    grp.destroy()


if __name__ == "__main__":
    main()
