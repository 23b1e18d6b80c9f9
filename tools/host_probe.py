"""BASELINE config 3 at one bucket size, a few repetitions: the command under a
rocprofv3 kernel + memory-copy trace of the host pipeline
(inccl_allreduce_f32_host).  A profiling aid.

    python tools/host_probe.py [bucket_mib] [reps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import container_inc_amd
    from container_inc_amd import inccl
    container_inc_amd.load()
    bucket_mib = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    n = (1 << 30) // 4
    x = torch.randn(n, dtype=torch.float32).pin_memory()
    y = torch.empty(n, dtype=torch.float32).pin_memory()
    comm.allreduce_f32_host(x, y, scale_exp=24, bucket_bytes=bucket_mib << 20)
    t0 = time.perf_counter()
    for _ in range(reps):
        comm.allreduce_f32_host(x, y, scale_exp=24, bucket_bytes=bucket_mib << 20)
    dt = (time.perf_counter() - t0) / reps
    print(f"bucket {bucket_mib} MiB: {dt * 1e3:.2f} ms per 1 GiB ({(1 << 30) / dt / 1e9:.1f} GB/s)", flush=True)
    comm.destroy()
    grp.destroy()


if __name__ == "__main__":
    main()
