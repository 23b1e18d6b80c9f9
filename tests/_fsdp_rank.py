"""One rank of the FSDP comm-hook tests (tests/test_fsdp_hook.py,
tests/test_gpu_fsdp.py): a small MLP under FullyShardedDataParallel (gloo
process group for FSDP's own parameter all-gathers) with
``container_inc_amd.fsdp.reduce_scatter_hook`` (FULL_SHARD) or
``allreduce_hook`` (NO_SHARD) on every unit's gradient.  Every hooked call's
result must equal the oracle's reduce of all ranks' gradients at
``choose_scale(absmax, W)``, sliced to this rank's shard (FULL_SHARD), divided
by W, bit for bit.

``mode`` "cpu": the communicator is tests/_ddp_rank.py's GlooStandIn (the
engine's contract restated with the oracle over gloo); "gpu": the real library
on cuda:0 (engine p2p; every rank shares the card)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(rank, world, port, q, mode, sharded=True, engine="p2p", boot_port=None, dtype="f32"):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        if mode == "gpu":
            os.environ["INCCL_ENGINE"] = engine
        import torch
        import torch.distributed as dist
        from torch.distributed.fsdp import FullyShardedDataParallel as FSDP
        from torch.distributed.fsdp import ShardingStrategy

        from _ddp_rank import GlooStandIn, _bits
        from container_inc_amd import fsdp, inccl
        from oracle import oracle as O

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        if mode == "gpu":
            torch.cuda.set_device(0)
            dev = torch.device("cuda", 0)
            grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=boot_port, device=0)
            comm = inccl.inccl_communicator_create(grp, 0)
        else:
            dev = torch.device("cpu")
            comm = GlooStandIn(world)
        wdt = {"bf16": torch.bfloat16, "f16": torch.float16}.get(dtype, torch.float32)
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(96, 512), torch.nn.Tanh(), torch.nn.Linear(512, 300),
                                    torch.nn.Tanh(), torch.nn.Linear(300, 10)).to(dev, wdt)
        net = FSDP(model, device_id=dev, use_orig_params=False,
                   sharding_strategy=ShardingStrategy.FULL_SHARD if sharded else ShardingStrategy.NO_SHARD)
        state = fsdp.HookState(comm=comm)
        seen = []

        def hook(st, grad, output=None):
            before = grad.detach().clone()
            if sharded:
                fsdp.reduce_scatter_hook(st, grad, output)
                seen.append((before, output.detach().clone()))
            else:
                fsdp.allreduce_hook(st, grad)
                seen.append((before, grad.detach().clone()))

        net.register_comm_hook(state, hook)
        gen = torch.Generator().manual_seed(100 + rank)
        report = {"calls": 0, "bit_exact": True, "checked": 0}
        for it in range(2):
            x = torch.randn(64, 96, generator=gen).to(dev, wdt)
            y = (torch.randn(64, 10, generator=gen) * (10.0 ** it)).to(dev, wdt)
            seen.clear()
            torch.nn.functional.mse_loss(net(x), y).backward()
            if dev.type == "cuda":
                torch.cuda.synchronize()
            for before, after in seen:
                allb = [None] * world
                dist.all_gather_object(allb, _bits(before.reshape(-1)).tobytes())
                if dtype == "f32":
                    every = [np.frombuffer(b, np.float32) for b in allb]
                    k = O.choose_scale(O.absmax(every), world)
                    full = O.reduce_f32(every, k)
                    t = torch.from_numpy(full)
                else:
                    every = [np.frombuffer(b, np.uint16) for b in allb]
                    absmax, reduce = (O.absmax_bf16, O.reduce_bf16) if dtype == "bf16" else (O.absmax_f16, O.reduce_f16)
                    k = O.choose_scale(absmax(every), world)
                    t = torch.from_numpy(reduce(every, k).view(np.int16)).view(wdt)
                if sharded:
                    shard = t.numel() // world
                    t = t[rank * shard:(rank + 1) * shard]
                want = _bits(t / world)   # the mean (exact for W = 2, 4)
                report["checked"] += 1
                if not np.array_equal(_bits(after.reshape(-1)), want):
                    report["bit_exact"] = False
            # FSDP's sharded .grad holds the averaged shard it was handed
            for p in net.parameters():
                assert p.grad is not None
            net.zero_grad()
        report["calls"] = state.calls
        q.put((rank, report))
        if mode == "gpu":
            comm.destroy()
            grp.destroy()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, {"error": repr(e), "tb": traceback.format_exc()}))
