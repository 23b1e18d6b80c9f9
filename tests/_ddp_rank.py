"""One rank of the DDP comm-hook tests (tests/test_ddp_hook.py, tests/test_gpu_ddp.py).

A small MLP under DistributedDataParallel (gloo process group), a tiny bucket
cap so the gradients travel in several buckets, and
``container_inc_amd.ddp.allreduce_hook`` on every bucket.  Each rank reports:

* ``buckets``: how many buckets the hook reduced per iteration;
* ``bit_exact``: every hooked bucket equals the oracle's ``reduce_f32`` of all
  ranks' buckets at ``choose_scale(absmax, W)``, divided by W (W = 2, 4: exact);
* ``grad_err``: max |DDP grad - mean of the ranks' local grads| over the
  quantisation bound of the bucket it travelled in (<= 1 expected).

``mode`` "cpu": the communicator is :class:`GlooStandIn` (the engine's contract
restated with the oracle over gloo), so the hook's plumbing is tested without a
GPU.  ``mode`` "gpu": the real library on cuda:0 (every rank shares the card;
engine p2p, because RCCL refuses two ranks on one GPU).
"""
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class GlooStandIn:
    """CPU stand-in for ``inccl.Communicator.allreduce_f32`` (test infrastructure)."""

    def __init__(self, world):
        self.group = types.SimpleNamespace(world_size=world)
        self.nonfinite = False

    def set_nonfinite(self, propagate=True):
        """inccl_comm_set_nonfinite: under auto scale, a NaN / +-Inf anywhere makes the result NaN"""
        self.nonfinite = bool(propagate)

    def allreduce_f32(self, srcs, out=None, scale_exp=25, chunks=1, stream=None):
        import torch
        import torch.distributed as dist
        from container_inc_amd import inccl
        from oracle import oracle as O
        W = self.group.world_size
        got = [torch.empty_like(srcs[0]) for _ in range(W)]
        dist.all_gather(got, srcs[0].contiguous())
        every = [g.numpy() for g in got]
        if self.nonfinite and scale_exp == inccl.SCALE_AUTO and O.any_nonfinite(every, "f32"):
            return out.fill_(float("nan"))
        k = O.choose_scale(O.absmax(every), W) if scale_exp == inccl.SCALE_AUTO else scale_exp
        out.copy_(torch.from_numpy(O.reduce_f32(every, k)))
        return out

    def _allreduce_16(self, srcs, out, scale_exp, absmax, reduce, dtype):
        import torch
        import torch.distributed as dist
        from container_inc_amd import inccl
        W = self.group.world_size
        # gloo has no 16-bit types: the bit patterns travel widened to int32
        mine = srcs[0].contiguous().view(torch.int16).to(torch.int32)
        got = [torch.empty_like(mine) for _ in range(W)]
        dist.all_gather(got, mine)
        every = [g.numpy().astype(np.uint16) for g in got]
        kind = "f16" if dtype == torch.float16 else "bf16"
        from oracle import oracle as O
        if self.nonfinite and scale_exp == inccl.SCALE_AUTO and O.any_nonfinite(every, kind):
            return out.fill_(float("nan"))
        k = O_choose(absmax(every), W) if scale_exp == inccl.SCALE_AUTO else scale_exp
        out.copy_(torch.from_numpy(reduce(every, k).view(np.int16)).view(dtype))
        return out

    def allreduce_bf16(self, srcs, out=None, scale_exp=25, stream=None):
        import torch
        from oracle import oracle as O
        return self._allreduce_16(srcs, out, scale_exp, O.absmax_bf16, O.reduce_bf16, torch.bfloat16)

    def allreduce_f16(self, srcs, out=None, scale_exp=25, stream=None):
        import torch
        from oracle import oracle as O
        return self._allreduce_16(srcs, out, scale_exp, O.absmax_f16, O.reduce_f16, torch.float16)


    def reduce_scatter(self, srcs, out=None, scale_exp=25, stream=None):
        """inccl_reduce_scatter_f32 restated: this rank's shard of the oracle's reduce"""
        import torch
        import torch.distributed as dist
        from container_inc_amd import inccl
        from oracle import oracle as O
        W, me = self.group.world_size, dist.get_rank()
        got = [torch.empty_like(srcs[0]) for _ in range(W)]
        dist.all_gather(got, srcs[0].contiguous())
        every = [g.numpy() for g in got]
        shard = every[0].size // W
        if self.nonfinite and scale_exp == inccl.SCALE_AUTO and O.any_nonfinite(every, "f32"):
            return out.fill_(float("nan"))
        k = O.choose_scale(O.absmax(every), W) if scale_exp == inccl.SCALE_AUTO else scale_exp
        out.copy_(torch.from_numpy(O.reduce_f32(every, k)[me * shard:(me + 1) * shard]))
        return out


def O_choose(amax, W):
    from oracle import oracle as O
    return O.choose_scale(amax, W)


def _bits(t):
    """bit patterns of an fp32 (uint32) or bf16 / fp16 (uint16) tensor as numpy"""
    import torch
    if t.dtype in (torch.bfloat16, torch.float16):
        return t.detach().view(torch.int16).cpu().numpy().view(np.uint16)
    return t.detach().cpu().numpy().view(np.uint32)


def run(rank, world, port, q, mode, iters=2, dtype="f32", as_view=False, engine="p2p", boot_port=None,
        poison=None):
    """dtype "bf16" / "f16": a bf16 / fp16 model, so DDP's buckets are bf16 / fp16
    (inccl_allreduce_bf16 / _f16);
    poison "propagate" / "saturate": one iteration whose last rank has an infinite
    target (every local gradient of that rank non-finite), with the hook's
    communicator propagating non-finite inputs or not; the report then holds
    ``found_inf`` (a loss scaler's check on this rank's averaged .grad) and
    ``all_nan``;
    as_view: gradient_as_bucket_view=True (the grads are views of the buckets);
    boot_port: the library bootstrap's port, chosen free by the parent (gloo uses `port`)."""
    try:
        sys.path.insert(0, ROOT)
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        if mode == "gpu":
            os.environ["INCCL_ENGINE"] = engine
        import torch
        import torch.distributed as dist
        from torch.nn.parallel import DistributedDataParallel as DDP

        from container_inc_amd import ddp, inccl
        from oracle import oracle as O

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        if mode == "gpu":
            torch.cuda.set_device(0)
            dev = torch.device("cuda", 0)
            grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=boot_port, device=0)
            assert grp is not None, "group create failed"
            comm = inccl.inccl_communicator_create(grp, 0)
            assert comm is not None and comm.engine == engine, comm and comm.engine
        else:
            dev = torch.device("cpu")
            comm = GlooStandIn(world)

        torch.manual_seed(0)   # the same initial weights on every rank
        model = torch.nn.Sequential(torch.nn.Linear(96, 512), torch.nn.Tanh(), torch.nn.Linear(512, 500),
                                    torch.nn.Tanh(), torch.nn.Linear(500, 300), torch.nn.Tanh(),
                                    torch.nn.Linear(300, 10)).to(dev)
        wdt = {"bf16": torch.bfloat16, "f16": torch.float16}.get(dtype, torch.float32)
        model = model.to(wdt)
        import copy
        local = copy.deepcopy(model)   # non-DDP twin: this rank's own gradients
        net = DDP(model, device_ids=[0] if mode == "gpu" else None, bucket_cap_mb=0.25,
                  gradient_as_bucket_view=as_view)
        state = ddp.HookState(comm=comm, propagate_nonfinite=poison != "saturate")
        seen = []

        def hook(st, bucket):
            before = bucket.buffer().detach().clone()
            fut = ddp.allreduce_hook(st, bucket)
            seen.append((before, bucket.buffer()))
            return fut

        net.register_comm_hook(state, hook)
        opt = torch.optim.SGD(net.parameters(), lr=0.05)
        opt_local = torch.optim.SGD(local.parameters(), lr=0.05)
        report = {"buckets": [], "bit_exact": True, "grad_err": 0.0}
        gen = torch.Generator().manual_seed(100 + rank)
        if poison:
            x = torch.randn(64, 96, generator=gen).to(dev, wdt)
            y = torch.randn(64, 10, generator=gen).to(dev, wdt)
            if rank == world - 1:
                y[0, 0] = float("inf")
            opt.zero_grad()
            torch.nn.functional.mse_loss(net(x), y).backward()
            if dev.type == "cuda":
                torch.cuda.synchronize()
            grads = [p.grad.detach().float() for p in net.module.parameters()]
            report["found_inf"] = bool(any(not torch.isfinite(g).all() for g in grads))
            report["all_nan"] = bool(all(torch.isnan(g).all() for g in grads))
            report["calls"] = state.calls
            q.put((rank, report))
            if mode == "gpu":
                comm.destroy()
                grp.destroy()
            dist.destroy_process_group()
            return
        for it in range(iters):
            x = torch.randn(64, 96, generator=gen).to(dev, wdt)
            y = (torch.randn(64, 10, generator=gen) * (10.0 ** it)).to(dev, wdt)   # later iterations: larger grads
            seen.clear()
            opt.zero_grad()
            torch.nn.functional.mse_loss(net(x), y).backward()
            if dev.type == "cuda":
                torch.cuda.synchronize()
            report["buckets"].append(len(seen))
            # every hooked bucket vs the oracle on all ranks' bucket inputs
            for before, after in seen:
                allb = [None] * world
                dist.all_gather_object(allb, _bits(before).tobytes())
                if dtype in ("bf16", "f16"):
                    every = [np.frombuffer(b, np.uint16) for b in allb]
                    absmax, reduce = (O.absmax_bf16, O.reduce_bf16) if dtype == "bf16" else (O.absmax_f16, O.reduce_f16)
                    k = O.choose_scale(absmax(every), world)
                    s16 = torch.from_numpy(reduce(every, k).view(np.int16)).view(wdt)
                    want = _bits(s16 / world)   # the hook's div_ (exact for W = 2, 4)
                else:
                    every = [np.frombuffer(b, np.float32) for b in allb]
                    k = O.choose_scale(O.absmax(every), world)
                    want = (O.reduce_f32(every, k) / np.float32(world)).view(np.uint32)
                if not np.array_equal(_bits(after), want):
                    report["bit_exact"] = False
            # DDP's averaged grads vs the mean of the ranks' local grads.  Bound per
            # lane: W quantisation errors of 2^-(k+1) each, divided by W, at the
            # smallest scale any bucket can have (k from the largest |grad| of all),
            # plus the rounding of the sum to the bucket's format (2^-23 relative for
            # fp32, 2^-8 for bf16, 2^-11 for fp16, doubled for slack); fp16 adds its
            # subnormal spacing 2^-24 as an absolute floor (the sum's rounding and the
            # hook's div_ each lose up to half of it, doubled for slack)
            opt_local.zero_grad()
            torch.nn.functional.mse_loss(local(x), y).backward()
            means, ddp_grads = [], []
            for p, pl in zip(net.module.parameters(), local.parameters()):
                g = pl.grad.detach().float().cpu().numpy()
                allg = [None] * world
                dist.all_gather_object(allg, g.tobytes())
                stack = np.stack([np.frombuffer(b, np.float32).astype(np.float64) for b in allg])
                means.append((stack.mean(axis=0), float(np.max(np.abs(stack)))))
                ddp_grads.append(p.grad.detach().float().cpu().numpy().astype(np.float64).ravel())
            k = O.choose_scale(np.float32(max(a for _, a in means)), world)
            for (mean, _), got in zip(means, ddp_grads):
                rel = {"bf16": 2.0 ** -7, "f16": 2.0 ** -10}.get(dtype, 2.0 ** -23)
                floor = 2.0 ** -23 if dtype == "f16" else 0.0
                bound = 2.0 ** -(k + 1) + np.abs(mean) * rel + floor
                report["grad_err"] = max(report["grad_err"], float(np.max(np.abs(got - mean) / bound)))
            opt.step()
            # the local twin follows the DDP model so the next iteration starts equal
            with torch.no_grad():
                for p, pl in zip(net.module.parameters(), local.parameters()):
                    pl.copy_(p)
        report["calls"] = state.calls
        q.put((rank, report))
        if mode == "gpu":
            comm.destroy()
            grp.destroy()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, {"error": repr(e), "tb": traceback.format_exc()}))
