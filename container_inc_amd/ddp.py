"""PyTorch DDP communication hook over the INCCL engine -- the caller of this path.

The reference's only caller is ``host.c:39-47``: it creates a group and a
communicator, then calls ``inccl_allreduce_write`` on one int32 buffer.  In a
training job the caller of a gradient-aggregation engine is the data-parallel
wrapper, which hands over one flat fp32 gradient bucket at a time.  This module
plugs the engine in there: ``DistributedDataParallel.register_comm_hook`` with
:func:`allreduce_hook` sends every bucket through ``inccl_allreduce_f32``
(quantise -> int32 sum across ranks -> dequantise; the int32 sum is the
reference switch's aggregate, ``non_termination_switch.c:361-363``) and returns
the bucket averaged over the ranks, as DDP's built-in allreduce hook does.

Numerics: the scale defaults to ``SCALE_AUTO`` -- the bucket's absmax over every
rank picks the largest exponent whose int32 sum cannot overflow
(``orc_choose_scale``), so a bucket of any magnitude keeps ~30 significant bits
of its largest element.  Non-finite gradients: the hook switches its
communicator to ``set_nonfinite(True)``, so a NaN or +-Inf in any rank's bucket
makes the whole averaged bucket NaN on every rank -- a mixed-precision loss
scaler (``torch.amp.GradScaler``) then sees the overflow and skips the step, as
it would after a float allreduce.  (The quantiser alone would map NaN to 0 and
saturate +-Inf: a finite, wrong gradient.)  The averaged result is bit-identical to the oracle's
``reduce_f32`` of the same buckets divided by the world size.

fp32, bf16 and fp16 CUDA buckets are accepted (bf16 / fp16 through
``inccl_allreduce_bf16`` / ``_f16``: the same int32 sums, the result rounded to
the bucket's format).  For a power-of-two world the mean comes out of the
dequantise stage itself (``inccl_comm_set_average``: scale 2^-(k + log2 W)),
for every format alike; otherwise the hook divides by W in torch.  Anything
else raises (no silent fallback to another collective).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

from . import inccl
from ._lib import IncclError


@dataclass
class HookState:
    """What :func:`allreduce_hook` needs: the communicator, the scale and
    whether to average.  ``calls`` counts the buckets reduced (for tests and
    logging)."""

    comm: object
    scale_exp: int = inccl.SCALE_AUTO
    average: bool = True
    calls: int = 0
    folded: bool | None = None   # the mean comes out of the dequantise stage (inccl_comm_set_average)
    propagate_nonfinite: bool = True   # NaN / +-Inf anywhere -> the bucket is NaN (inccl_comm_set_nonfinite)
    _nonfinite_set: bool = False

    def fold_average(self) -> bool:
        """Once: let the engine return the mean (power-of-two worlds: 2^-log2 W is
        folded into the dequantise scale, bit-identical to dividing, one pass
        fewer); otherwise the hook divides.  This switches the communicator
        itself to averaging: give the hook a communicator of its own."""
        if self.folded is None:
            self.folded = False
            if self.average and self.world_size > 1 and hasattr(self.comm, "set_average"):
                try:
                    self.comm.set_average(True)
                    self.folded = True
                except IncclError:
                    pass
        return self.folded

    def apply_nonfinite(self) -> None:
        """Once: the communicator's non-finite mode (auto scale only)."""
        if not self._nonfinite_set:
            self._nonfinite_set = True
            if hasattr(self.comm, "set_nonfinite"):
                self.comm.set_nonfinite(self.propagate_nonfinite)

    @property
    def world_size(self) -> int:
        return self.comm.group.world_size


def allreduce_hook(state: HookState, bucket):
    """DDP comm hook: ``bucket.buffer()`` <- mean over ranks, through INCCL.

    The collective runs on the communicator's own stream, after the work queued
    so far on the current stream (the gradients of this bucket), so the backward
    pass keeps computing the next buckets' gradients on its stream while this
    one is exchanged -- the overlap DDP gets from its own collectives.  The
    returned future is CUDA-aware: DDP's wait on it orders its copy-back into
    ``.grad`` after the reduction."""
    import torch

    buf = bucket.buffer()
    name = {torch.float32: "allreduce_f32", torch.bfloat16: "allreduce_bf16", torch.float16: "allreduce_f16"}.get(buf.dtype)
    if name is None:
        raise IncclError(f"inccl DDP hook: fp32, bf16 or fp16 gradient buckets only, got {buf.dtype}")
    reduce = getattr(state.comm, name)
    state.apply_nonfinite()
    w = state.world_size
    divide = state.average and w > 1 and not state.fold_average()
    if not buf.is_cuda:   # reaches the communicator, which refuses it ("must live on the GPU")
        reduce([buf], out=buf, scale_exp=state.scale_exp, stream=None)
        if divide:
            buf.div_(w)
        fut = torch.futures.Future()
    else:
        side = torch.cuda.ExternalStream(state.comm.stream, device=buf.device)
        side.wait_stream(torch.cuda.current_stream(buf.device))
        with torch.cuda.stream(side):
            reduce([buf], out=buf, scale_exp=state.scale_exp, stream=side.cuda_stream)
            if divide:
                buf.div_(w)
            # the bucket is used on `side` now: the caching allocator must not
            # hand its memory out before this stream's work is done
            buf.record_stream(side)
            fut = torch.futures.Future(devices=[buf.device])
            fut.set_result(buf)   # records an event on `side`; wait() makes the waiter's stream wait on it
    if not buf.is_cuda:
        fut.set_result(buf)
    state.calls += 1
    return fut


def communicator_from_env(port_offset: int = 17, device: int | None = None, engine: str | None = None):
    """Create the INCCL group + communicator for this rank from the torchrun
    environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT).  The
    group's bootstrap listens on MASTER_PORT + ``port_offset`` so it does not
    collide with torch.distributed's own store.  ``engine`` as in
    ``Communicator.set_engine`` (default: the library's choice)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0"))
    master = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500")) + port_offset
    grp = inccl.inccl_group_create(world, rank, master, port=port, device=device)
    if grp is None:
        from ._lib import load
        raise IncclError("inccl_group_create failed: " + load().inccl_last_error().decode(errors="replace"))
    comm = inccl.inccl_communicator_create(grp, 0)
    if comm is None:
        grp.destroy()
        from ._lib import load
        raise IncclError("inccl_communicator_create failed: " + load().inccl_last_error().decode(errors="replace"))
    if engine:
        comm.set_engine(engine)
    return comm


def register(ddp_model, comm, scale_exp: int = inccl.SCALE_AUTO, average: bool = True) -> HookState:
    """Route every gradient bucket of ``ddp_model`` through ``comm``; returns the hook state."""
    state = HookState(comm=comm, scale_exp=scale_exp, average=average)
    ddp_model.register_comm_hook(state, allreduce_hook)
    return state
