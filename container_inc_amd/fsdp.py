"""PyTorch FSDP communication hooks over the INCCL engine -- the sharded-
gradient caller of this path.

``FullyShardedDataParallel`` with a sharded strategy hands its communication
hook the flat, unsharded gradient of one FSDP unit (padded to a multiple of the
world size) and the shard it must fill (``reduce_scatter_hook(state, grad,
output)``, the signature of torch's own ``default_hooks.reduce_scatter_hook``).
:func:`reduce_scatter_hook` fills it through ``inccl_reduce_scatter_*``:
quantise -> int32 sum across ranks (the reference switch's aggregate,
``non_termination_switch.c:361-363``) kept per shard -> dequantise -- and
returns the shard averaged over the ranks, as torch's hook does.  With
``NO_SHARD`` FSDP calls ``hook(state, grad)`` instead; :func:`allreduce_hook`
reduces the whole gradient in place.

Numerics and modes are the DDP hook's (``container_inc_amd/ddp.py``): auto
scale, the mean folded into the dequantise stage for a power-of-two world
(``inccl_comm_set_average``; otherwise the hook divides), and non-finite
gradients propagated as NaN (``inccl_comm_set_nonfinite``) so a loss scaler
skips the step on every rank.  Both change the communicator: give the hook one
of its own.  The collective runs on the current stream -- FSDP calls its hook
on its own post-backward stream already -- so the shard is ready for FSDP's next
use without further synchronisation.  fp32, bf16 and fp16 gradients.
"""
from __future__ import annotations

from ._lib import IncclError
from .ddp import HookState


def _check(state: HookState, grad):
    import torch
    if grad.dtype not in (torch.float32, torch.bfloat16, torch.float16):
        raise IncclError(f"inccl FSDP hook: fp32, bf16 or fp16 gradients only, got {grad.dtype}")
    state.apply_nonfinite()
    w = state.world_size
    return w, state.average and w > 1 and not state.fold_average()


def _stream(t):
    import torch
    return torch.cuda.current_stream(t.device).cuda_stream if t.is_cuda else None


def reduce_scatter_hook(state: HookState, grad, output):
    """FSDP sharded-strategy hook: ``output`` <- this rank's shard of the mean of
    every rank's ``grad`` (grad.numel() == W * output.numel())."""
    w, divide = _check(state, grad)
    if grad.numel() != w * output.numel() or output.dtype != grad.dtype:
        raise IncclError(f"inccl FSDP hook: a {grad.numel()}-element gradient does not shard into "
                         f"{w} x {output.numel()} ({output.dtype})")
    if not output.is_contiguous():   # the shard is written in place: a reshaped copy would lose it
        raise IncclError("inccl FSDP hook: the output shard must be contiguous")
    state.comm.reduce_scatter([grad.reshape(-1)], out=output.reshape(-1), scale_exp=state.scale_exp,
                              stream=_stream(grad))
    if divide:
        output.div_(w)
    state.calls += 1


def allreduce_hook(state: HookState, grad):
    """FSDP ``NO_SHARD`` hook: ``grad`` <- the mean of every rank's ``grad``, in place."""
    import torch
    w, divide = _check(state, grad)
    fn = {torch.float32: "allreduce_f32", torch.bfloat16: "allreduce_bf16", torch.float16: "allreduce_f16"}[grad.dtype]
    if not grad.is_contiguous():   # reduced in place: a reshaped copy would lose the result
        raise IncclError("inccl FSDP hook: the gradient must be contiguous")
    flat = grad.reshape(-1)
    getattr(state.comm, fn)([flat], out=flat, scale_exp=state.scale_exp, stream=_stream(grad))
    if divide:
        grad.div_(w)
    state.calls += 1


def register(fsdp_model, comm, sharded: bool = True, **kw) -> HookState:
    """Route every FSDP unit's gradient reduction of ``fsdp_model`` through ``comm``
    (``sharded``: reduce-scatter, for the sharded strategies; else allreduce, for
    NO_SHARD); returns the hook state.  ``kw``: HookState fields."""
    state = HookState(comm=comm, **kw)
    fsdp_model.register_comm_hook(state, reduce_scatter_hook if sharded else allreduce_hook)
    return state
