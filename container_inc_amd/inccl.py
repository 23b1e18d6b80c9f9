"""Python host mirror of the INCCL interface over ``libinccl_amd.so``.

Reference interface: ``repository/include/api.h:93-101`` (group / communicator /
``inccl_allreduce_write`` / ``inccl_allreduce_sendrecv``), kept with the same
names, argument meaning (``len`` in int32 elements, communicator ``size`` in
bytes, whole-message rule of ``api.c:406``) and error behaviour (``None`` from a
failed group create, ``api.c:82-98``).  The additive fp32 / device API of
``include/inccl_amd.h`` is exposed on torch tensors (PyTorch is plumbing here:
device memory and streams).

Every compute call goes through the HIP library; nothing here computes on the
CPU.  Shapes and dtypes are validated on the host before any launch.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from ._lib import IncclError, check, load

KIND_F32, KIND_Q32, KIND_Q32BE, KIND_BF16, KIND_F16 = 0, 1, 2, 3, 4
SCALE_MIN, SCALE_MAX, SCALE_AUTO = -64, 64, 0x7FFFFFFF
MAX_LOCAL_INPUTS = 8
ABSMAX_FLAG_NONFINITE = 2        # inccl_amd.h INCCL_ABSMAX_FLAG_NONFINITE
NONFINITE_SATURATE, NONFINITE_NAN = 0, 1
PAYLOAD_LEN = 1024           # util.h:85
MESSAGE_SIZE = 4 * PAYLOAD_LEN   # api.h:39
PAYLOAD_COUNT = MESSAGE_SIZE // 4  # api.h:40
WINDOW_SIZE = 8192           # api.h:38
MASTER_PORT = 52223          # parameter.h:1


def _torch():
    import torch
    return torch


def _dev_ptr(t, dtype, name: str, numel: int | None = None) -> int:
    torch = _torch()
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor, got {type(t)!r}")
    if t.device.type != "cuda":
        raise ValueError(f"{name}: tensor must live on the GPU (got {t.device})")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: tensor must be contiguous")
    if numel is not None and t.numel() < numel:
        raise ValueError(f"{name}: needs {numel} elements, has {t.numel()}")
    return t.data_ptr()


def _stream_handle(stream) -> int | None:
    torch = _torch()
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def _ptr_array(ptrs: Sequence[int]):
    return (ctypes.c_void_p * len(ptrs))(*ptrs)


def _check_scale(k: int) -> int:
    k = int(k)
    if k != SCALE_AUTO and not (SCALE_MIN <= k <= SCALE_MAX):
        raise ValueError(f"scale exponent {k} outside [{SCALE_MIN}, {SCALE_MAX}]")
    return k


_TORCH_KIND = {KIND_F32: "float32", KIND_Q32: "int32", KIND_Q32BE: "int32", KIND_BF16: "bfloat16",
               KIND_F16: "float16"}


def stream_op(in_kind: int, out_kind: int, srcs, out=None, scale_exp: int = 0, n: int | None = None,
              amax_word=None, scale_R: int = 0, stream=None):
    """Generic ``out = OUT(sum_r IN(srcs[r]))`` (see inccl_kernels.hip)."""
    torch = _torch()
    if len(srcs) < 1 or len(srcs) > MAX_LOCAL_INPUTS:
        raise ValueError(f"1..{MAX_LOCAL_INPUTS} inputs per launch, got {len(srcs)}")
    in_dt = getattr(torch, _TORCH_KIND[in_kind])
    out_dt = getattr(torch, _TORCH_KIND[out_kind])
    if n is None:
        n = srcs[0].numel()
    ptrs = [_dev_ptr(s, in_dt, f"srcs[{i}]", n) for i, s in enumerate(srcs)]
    if out is None:
        out = torch.empty(n, dtype=out_dt, device=srcs[0].device)
    optr = _dev_ptr(out, out_dt, "out", n)
    aptr = None
    if amax_word is not None:
        aptr = _dev_ptr(amax_word, torch.int32, "amax_word", 1)
    else:
        scale_exp = _check_scale(scale_exp)
    rc = load().inccl_stream_op(in_kind, out_kind, _ptr_array(ptrs), len(ptrs), optr, n, int(scale_exp), aptr,
                                int(scale_R), _stream_handle(stream))
    check(rc, "inccl_stream_op")
    return out


class PreparedOp:
    """``stream_op`` (or, with ``comm``, ``Communicator.allreduce_f32`` / ``_bf16``
    / ``_f16``) with its arguments checked and bound once (inccl_op_create /
    inccl_op_create_allreduce_f32 / _allreduce16): each call is then one ctypes call with one
    argument, for small buckets whose per-call cost is launch and marshalling,
    not HBM.  Holds references to the bound tensors; call destroy() (or drop
    it) when done -- before the communicator, for a prepared allreduce."""

    def __init__(self, in_kind: int, out_kind: int, srcs, out, scale_exp: int, scale_R: int = 0, stream=None,
                 comm=None, chunks: int = 1):
        torch = _torch()
        srcs = list(srcs)
        if len(srcs) < 1 or len(srcs) > MAX_LOCAL_INPUTS:
            raise ValueError(f"1..{MAX_LOCAL_INPUTS} inputs per launch, got {len(srcs)}")
        in_dt, out_dt = getattr(torch, _TORCH_KIND[in_kind]), getattr(torch, _TORCH_KIND[out_kind])
        n = srcs[0].numel()
        ptrs = [_dev_ptr(s, in_dt, f"srcs[{i}]", n) for i, s in enumerate(srcs)]
        if out is None:
            out = torch.empty(n, dtype=out_dt, device=srcs[0].device)
        optr = _dev_ptr(out, out_dt, "out", n)
        if int(scale_exp) == SCALE_AUTO:
            raise ValueError("a prepared op takes a fixed scale exponent")
        self.srcs, self.out, self.stream, self.comm = srcs, out, stream, comm   # kept alive while bound
        lib = load()
        if comm is None:
            h = lib.inccl_op_create(in_kind, out_kind, _ptr_array(ptrs), len(ptrs), optr, n, _check_scale(scale_exp),
                                    int(scale_R), _stream_handle(stream))
        elif in_kind == KIND_F32:
            h = lib.inccl_op_create_allreduce_f32(comm.handle, _ptr_array(ptrs), len(ptrs), optr, n,
                                                  _check_scale(scale_exp), int(chunks), _stream_handle(stream))
        else:
            h = lib.inccl_op_create_allreduce16(comm.handle, in_kind, _ptr_array(ptrs), len(ptrs), optr, n,
                                                _check_scale(scale_exp), _stream_handle(stream))
        if not h:
            raise IncclError(lib.inccl_last_error().decode(errors="replace"))
        self._h = ctypes.c_void_p(h)
        self._run = lib.inccl_op_run

    def __call__(self):
        rc = self._run(self._h)
        if rc:
            check(rc, "inccl_op_run")
        return self.out

    def destroy(self):
        if self._h is not None:
            load().inccl_op_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:  # noqa: BLE001 -- interpreter teardown
            pass


def prepare_reduce_f32(srcs, scale_exp: int, out=None, stream=None) -> PreparedOp:
    """A prepared ``reduce_f32`` (the fused single-GPU bucket reduce)."""
    srcs = list(srcs)
    return PreparedOp(KIND_F32, KIND_F32, srcs, out, scale_exp, scale_R=len(srcs), stream=stream)


def quantise(x, scale_exp: int, wire_be: bool = False, out=None, stream=None):
    """fp32 -> int32 fixed point (+ optional htonl, api.c:300-302)."""
    return stream_op(KIND_F32, KIND_Q32BE if wire_be else KIND_Q32, [x], out, scale_exp, stream=stream)


def dequantise(q, scale_exp: int, wire_be: bool = False, out=None, stream=None):
    """int32 (optionally big-endian, api.c:428-430) -> fp32."""
    return stream_op(KIND_Q32BE if wire_be else KIND_Q32, KIND_F32, [q], out, scale_exp, stream=stream)


def reduce_f32(srcs, scale_exp: int, out=None, stream=None):
    """Fused single-GPU bucket reduce dequant(sum_r quant(srcs[r]))."""
    return stream_op(KIND_F32, KIND_F32, list(srcs), out, scale_exp, scale_R=len(srcs), stream=stream)


def quant_sum(srcs, scale_exp: int, wire_be: bool = False, out=None, stream=None):
    return stream_op(KIND_F32, KIND_Q32BE if wire_be else KIND_Q32, list(srcs), out, scale_exp, stream=stream)


def sum_q32(srcs, in_be: bool = False, out_be: bool = False, out=None, stream=None):
    """The switch aggregate (non_termination_switch.c:361-363) on the GPU."""
    return stream_op(KIND_Q32BE if in_be else KIND_Q32, KIND_Q32BE if out_be else KIND_Q32, list(srcs), out, 0,
                     stream=stream)


def sum_dequant(srcs, scale_exp: int, in_be: bool = False, out=None, stream=None):
    return stream_op(KIND_Q32BE if in_be else KIND_Q32, KIND_F32, list(srcs), out, scale_exp, stream=stream)


def reduce_bf16(srcs, scale_exp: int, out=None, stream=None):
    """Fused single-GPU bfloat16 bucket reduce: bf16_rne(dequant(sum_r quant(srcs[r])))."""
    return stream_op(KIND_BF16, KIND_BF16, list(srcs), out, scale_exp, scale_R=len(srcs), stream=stream)


def reduce_f16(srcs, scale_exp: int, out=None, stream=None):
    """Fused single-GPU fp16 bucket reduce: f16_rne(dequant(sum_r quant(srcs[r])))."""
    return stream_op(KIND_F16, KIND_F16, list(srcs), out, scale_exp, scale_R=len(srcs), stream=stream)


def absmax_f16(srcs, stream=None) -> float:
    torch = _torch()
    n = srcs[0].numel()
    ptrs = [_dev_ptr(s, torch.float16, f"srcs[{i}]", n) for i, s in enumerate(srcs)]
    word = torch.zeros(4, dtype=torch.int32, device=srcs[0].device)
    rc = load().inccl_absmax_f16(_ptr_array(ptrs), len(ptrs), n, _dev_ptr(word, torch.int32, "word", 1), 1,
                                 _stream_handle(stream))
    check(rc, "inccl_absmax_f16")
    bits = int(word[0].item()) & 0xFFFFFFFF
    return float(np.array([bits], np.uint32).view(np.float32)[0])


def absmax_bf16(srcs, stream=None) -> float:
    torch = _torch()
    n = srcs[0].numel()
    ptrs = [_dev_ptr(s, torch.bfloat16, f"srcs[{i}]", n) for i, s in enumerate(srcs)]
    word = torch.zeros(4, dtype=torch.int32, device=srcs[0].device)
    rc = load().inccl_absmax_bf16(_ptr_array(ptrs), len(ptrs), n, _dev_ptr(word, torch.int32, "word", 1), 1,
                                  _stream_handle(stream))
    check(rc, "inccl_absmax_bf16")
    bits = int(word[0].item()) & 0xFFFFFFFF
    return float(np.array([bits], np.uint32).view(np.float32)[0])


def absmax_word(srcs, word=None, stream=None):
    """Device absmax over R buckets; returns the int32 word tensor holding float bits."""
    torch = _torch()
    n = srcs[0].numel()
    ptrs = [_dev_ptr(s, torch.float32, f"srcs[{i}]", n) for i, s in enumerate(srcs)]
    if word is None:
        word = torch.zeros(4, dtype=torch.int32, device=srcs[0].device)
    rc = load().inccl_absmax_f32(_ptr_array(ptrs), len(ptrs), n, _dev_ptr(word, torch.int32, "word", 1), 1,
                                 _stream_handle(stream))
    check(rc, "inccl_absmax_f32")
    return word


def absmax_bits(srcs, nonfinite_flag: bool = False, stream=None) -> int:
    """The raw absmax word (fp32 bits of max |x|) of fp32 / bf16 / fp16 buckets;
    nonfinite_flag: INCCL_ABSMAX_FLAG_NONFINITE (a NaN or +-Inf sets bit 31)."""
    torch = _torch()
    n = srcs[0].numel()
    fn, dt = {torch.float32: ("inccl_absmax_f32", torch.float32), torch.bfloat16: ("inccl_absmax_bf16", torch.bfloat16),
              torch.float16: ("inccl_absmax_f16", torch.float16)}[srcs[0].dtype]
    ptrs = [_dev_ptr(s, dt, f"srcs[{i}]", n) for i, s in enumerate(srcs)]
    word = torch.zeros(4, dtype=torch.int32, device=srcs[0].device)
    rc = getattr(load(), fn)(_ptr_array(ptrs), len(ptrs), n, _dev_ptr(word, torch.int32, "word", 1),
                             1 | (ABSMAX_FLAG_NONFINITE if nonfinite_flag else 0), _stream_handle(stream))
    check(rc, fn)
    return int(word[0].item()) & 0xFFFFFFFF


def absmax(srcs, stream=None) -> float:
    w = absmax_word(srcs, stream=stream)
    bits = int(w[0].item()) & 0xFFFFFFFF
    return float(np.array([bits], np.uint32).view(np.float32)[0])


def reduce_f32_auto(srcs, out=None, word=None, stream=None):
    torch = _torch()
    n = srcs[0].numel()
    ptrs = [_dev_ptr(s, torch.float32, f"srcs[{i}]", n) for i, s in enumerate(srcs)]
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=srcs[0].device)
    if word is None:
        word = torch.zeros(4, dtype=torch.int32, device=srcs[0].device)
    rc = load().inccl_reduce_f32_auto(_ptr_array(ptrs), len(ptrs), _dev_ptr(out, torch.float32, "out", n), n,
                                      _dev_ptr(word, torch.int32, "word", 1), _stream_handle(stream))
    check(rc, "inccl_reduce_f32_auto")
    return out


def checksum_q32(q, index_base: int = 0, stream=None) -> int:
    torch = _torch()
    word = torch.zeros(4, dtype=torch.int32, device=q.device)
    rc = load().inccl_checksum_q32(_dev_ptr(q, torch.int32, "q"), q.numel(), int(index_base),
                                   _dev_ptr(word, torch.int32, "word", 1), 1, _stream_handle(stream))
    check(rc, "inccl_checksum_q32")
    return int(word[0].item()) & 0xFFFFFFFF


def choose_scale(amax: float, R_total: int) -> int:
    return int(load().inccl_choose_scale(ctypes.c_float(amax), int(R_total)))


def set_tuning(grid_cap: int = 0, nt_loads: bool = True) -> None:
    load().inccl_set_tuning(int(grid_cap), 1 if nt_loads else 0)


def version() -> str:
    return load().inccl_version().decode()


# ---------------------------------------------------------------------------
# groups / communicators (reference api.h:42-101)
# ---------------------------------------------------------------------------
class Group:
    def __init__(self, handle: int):
        if not handle:
            raise IncclError(load().inccl_last_error().decode(errors="replace") or "group create failed")
        self.handle = handle

    @property
    def rank(self) -> int:
        return load().inccl_group_rank(self.handle)

    @property
    def world_size(self) -> int:
        return load().inccl_group_size(self.handle)

    @property
    def device(self) -> int:
        return load().inccl_group_device(self.handle)

    @property
    def transport(self) -> str:
        return load().inccl_group_transport(self.handle).decode()

    def destroy(self) -> int:
        rc = 1
        if self.handle:
            rc = load().inccl_group_destroy(self.handle)
            self.handle = None
        return rc


class Communicator:
    def __init__(self, group: Group, handle: int):
        if not handle:
            raise IncclError(load().inccl_last_error().decode(errors="replace") or "communicator create failed")
        self.group = group
        self.handle = handle

    @property
    def stream(self) -> int:
        return load().inccl_comm_stream(self.handle)

    @property
    def engine(self) -> str:
        return load().inccl_comm_engine(self.handle).decode()

    def set_engine(self, name: str) -> None:
        check(load().inccl_comm_set_engine(self.handle, name.encode()), "inccl_comm_set_engine")

    def barrier(self) -> None:
        check(load().inccl_comm_barrier(self.handle), "inccl_comm_barrier")

    def ipc_mem_kind(self, engine: str) -> int:
        """hipDeviceMalloc* flags of the engine's IPC buffer (0 coarse, 1 fine-grained, 3 uncached)."""
        rc = load().inccl_comm_ipc_mem_kind(self.handle, engine.encode())
        if rc < 0:
            check(rc, "inccl_comm_ipc_mem_kind")
        return rc

    def clear_error(self) -> bool:
        """Collective: True if an ll / mesh wait had timed out; rebuilds their buffers."""
        rc = load().inccl_comm_clear_error(self.handle)
        if rc < 0:
            check(rc, "inccl_comm_clear_error")
        return rc == 1

    STAGE_NAMES = ("quant", "reduce_scatter", "dequant", "all_gather", "copy", "allreduce", "ipc")

    def set_stage_timing(self, on: bool = True) -> None:
        """Per-stage HIP-event timing of this rank's later non-captured calls
        (include/inccl_amd.h inccl_comm_set_stage_timing; diagnostics, never in
        a timed loop)."""
        check(load().inccl_comm_set_stage_timing(self.handle, 1 if on else 0), "inccl_comm_set_stage_timing")

    def stage_times(self) -> dict:
        """The last call's stages: {stage: us summed over its chunks, ...,
        "wall_us": first start to last end, "overlap_us": sum - wall,
        "stages": how many were recorded}; synchronises their events."""
        import ctypes
        kinds = len(self.STAGE_NAMES)
        us = (ctypes.c_double * kinds)()
        wall = ctypes.c_double(0.0)
        n = load().inccl_comm_stage_times(self.handle, ctypes.cast(us, ctypes.c_void_p), kinds,
                                          ctypes.cast(ctypes.pointer(wall), ctypes.c_void_p))
        if n < 0:
            check(n, "inccl_comm_stage_times")
        out = {name: round(us[i], 2) for i, name in enumerate(self.STAGE_NAMES) if us[i] > 0.0}
        out["wall_us"] = round(wall.value, 2)
        out["overlap_us"] = round(sum(us[i] for i in range(kinds)) - wall.value, 2)
        out["stages"] = n
        return out

    def set_average(self, on: bool = True) -> None:
        """Results of allreduce_f32 / _bf16 become the mean over ranks (power-of-two
        worlds; raises IncclError otherwise).  Bit-identical to sum / W."""
        check(load().inccl_comm_set_average(self.handle, 1 if on else 0), "inccl_comm_set_average")

    def set_nonfinite(self, propagate: bool = True) -> None:
        """propagate=True (INCCL_NONFINITE_NAN): a NaN or +-Inf in any rank's
        buckets makes every element of an auto-scaled allreduce's result NaN, as a
        loss scaler needs to see; False restores the quantiser's spec (NaN -> 0,
        +-Inf saturates).  Set it alike on every rank."""
        check(load().inccl_comm_set_nonfinite(self.handle, 1 if propagate else 0), "inccl_comm_set_nonfinite")

    # -- reference collectives on host int32 arrays (api.c:330-452) --
    def allreduce_write(self, src: np.ndarray, length: int, dst: np.ndarray) -> None:
        _host_int32_call(load().inccl_allreduce_write, self.handle, src, length, dst)

    def allreduce_sendrecv(self, src: np.ndarray, length: int, dst: np.ndarray) -> None:
        _host_int32_call(load().inccl_allreduce_sendrecv, self.handle, src, length, dst)

    def host_register(self, a) -> None:
        """Pin a host array for direct DMA by allreduce_write / _sendrecv (the
        reference registers its payload buffers with ibv_reg_mr, api.c:170-176).
        Keep `a` alive until host_deregister or destroy."""
        p, nbytes = _host_buf(a)
        check(load().inccl_host_register(self.handle, p, nbytes), "inccl_host_register")

    def host_deregister(self, a) -> None:
        p, _ = _host_buf(a)
        check(load().inccl_host_deregister(self.handle, p), "inccl_host_deregister")

    # -- additive device API --
    def allreduce_f32(self, srcs, out=None, scale_exp: int = 25, chunks: int = 1, stream=None):
        torch = _torch()
        srcs = list(srcs)
        if not 1 <= len(srcs) <= MAX_LOCAL_INPUTS:
            raise ValueError(f"1..{MAX_LOCAL_INPUTS} local buckets, got {len(srcs)}")
        n = srcs[0].numel()
        ptrs = [_dev_ptr(s, torch.float32, f"srcs[{i}]", n) for i, s in enumerate(srcs)]
        if out is None:
            out = torch.empty(n, dtype=torch.float32, device=srcs[0].device)
        optr = _dev_ptr(out, torch.float32, "out", n)
        rc = load().inccl_allreduce_f32_pipelined(self.handle, _ptr_array(ptrs), len(ptrs), optr, n,
                                                  _check_scale(scale_exp), int(chunks), _stream_handle(stream))
        check(rc, "inccl_allreduce_f32")
        return out

    def prepare_allreduce_f32(self, srcs, out=None, scale_exp: int = 25, chunks: int = 1, stream=None) -> PreparedOp:
        """``allreduce_f32`` with its arguments bound once: ``op()`` runs it."""
        return PreparedOp(KIND_F32, KIND_F32, srcs, out, scale_exp, stream=stream, comm=self, chunks=chunks)

    def prepare_allreduce_bf16(self, srcs, out=None, scale_exp: int = 25, stream=None) -> PreparedOp:
        """``allreduce_bf16`` with its arguments bound once: ``op()`` runs it."""
        return PreparedOp(KIND_BF16, KIND_BF16, srcs, out, scale_exp, stream=stream, comm=self)

    def prepare_allreduce_f16(self, srcs, out=None, scale_exp: int = 25, stream=None) -> PreparedOp:
        """``allreduce_f16`` with its arguments bound once: ``op()`` runs it."""
        return PreparedOp(KIND_F16, KIND_F16, srcs, out, scale_exp, stream=stream, comm=self)

    def allreduce_f16(self, srcs, out=None, scale_exp: int = SCALE_AUTO, stream=None):
        """IEEE fp16 buckets (include/inccl_amd.h inccl_allreduce_f16)."""
        torch = _torch()
        srcs = list(srcs)
        if not 1 <= len(srcs) <= MAX_LOCAL_INPUTS:
            raise ValueError(f"1..{MAX_LOCAL_INPUTS} local buckets, got {len(srcs)}")
        n = srcs[0].numel()
        ptrs = [_dev_ptr(s, torch.float16, f"srcs[{i}]", n) for i, s in enumerate(srcs)]
        if out is None:
            out = torch.empty(n, dtype=torch.float16, device=srcs[0].device)
        optr = _dev_ptr(out, torch.float16, "out", n)
        rc = load().inccl_allreduce_f16(self.handle, _ptr_array(ptrs), len(ptrs), optr, n, _check_scale(scale_exp),
                                        _stream_handle(stream))
        check(rc, "inccl_allreduce_f16")
        return out

    def reduce_scatter(self, srcs, out=None, scale_exp: int = SCALE_AUTO, stream=None):
        """Reduce-scatter of fp32 / bf16 / fp16 buckets (include/inccl_amd.h
        inccl_reduce_scatter_*): every rank passes R buckets of n = W * shard
        elements and gets back its shard of the reduced result."""
        torch = _torch()
        srcs = list(srcs)
        if not 1 <= len(srcs) <= MAX_LOCAL_INPUTS:
            raise ValueError(f"1..{MAX_LOCAL_INPUTS} local buckets, got {len(srcs)}")
        dt = srcs[0].dtype
        fn = {torch.float32: "inccl_reduce_scatter_f32", torch.bfloat16: "inccl_reduce_scatter_bf16",
              torch.float16: "inccl_reduce_scatter_f16"}.get(dt)
        if fn is None:
            raise TypeError(f"reduce_scatter: fp32, bf16 or fp16 buckets, got {dt}")
        n, W = srcs[0].numel(), self.group.world_size
        if n % W:
            raise ValueError(f"reduce_scatter: {n} elements do not split into {W} shards")
        ptrs = [_dev_ptr(s, dt, f"srcs[{i}]", n) for i, s in enumerate(srcs)]
        if out is None:
            out = torch.empty(n // W, dtype=dt, device=srcs[0].device)
        optr = _dev_ptr(out, dt, "out", n // W)
        rc = getattr(load(), fn)(self.handle, _ptr_array(ptrs), len(ptrs), optr, n, _check_scale(scale_exp),
                                 _stream_handle(stream))
        check(rc, fn)
        return out

    def allreduce_bf16(self, srcs, out=None, scale_exp: int = SCALE_AUTO, stream=None):
        """bfloat16 buckets (include/inccl_amd.h inccl_allreduce_bf16)."""
        torch = _torch()
        srcs = list(srcs)
        if not 1 <= len(srcs) <= MAX_LOCAL_INPUTS:
            raise ValueError(f"1..{MAX_LOCAL_INPUTS} local buckets, got {len(srcs)}")
        n = srcs[0].numel()
        ptrs = [_dev_ptr(s, torch.bfloat16, f"srcs[{i}]", n) for i, s in enumerate(srcs)]
        if out is None:
            out = torch.empty(n, dtype=torch.bfloat16, device=srcs[0].device)
        optr = _dev_ptr(out, torch.bfloat16, "out", n)
        rc = load().inccl_allreduce_bf16(self.handle, _ptr_array(ptrs), len(ptrs), optr, n, _check_scale(scale_exp),
                                         _stream_handle(stream))
        check(rc, "inccl_allreduce_bf16")
        return out

    def allreduce_q32(self, src, out=None, stream=None):
        torch = _torch()
        n = src.numel()
        if out is None:
            out = torch.empty_like(src)
        rc = load().inccl_allreduce_q32(self.handle, _dev_ptr(src, torch.int32, "src"),
                                        _dev_ptr(out, torch.int32, "out", n), n, _stream_handle(stream))
        check(rc, "inccl_allreduce_q32")
        return out

    def allreduce_f32_host(self, src, dst, scale_exp: int = 25, bucket_bytes: int = 64 << 20) -> None:
        """Host-memory buckets (numpy arrays or pinned CPU tensors)."""
        sp, sn = _host_ptr(src, np.float32, "src")
        dp, dn = _host_ptr(dst, np.float32, "dst")
        if dn < sn:
            raise ValueError("dst smaller than src")
        rc = load().inccl_allreduce_f32_host(self.handle, sp, dp, sn, _check_scale(scale_exp), int(bucket_bytes))
        check(rc, "inccl_allreduce_f32_host")

    def destroy(self) -> int:
        rc = 0
        if self.handle:
            rc = load().inccl_communicator_destroy(self.handle)
            self.handle = None
        return rc


def _host_buf(a):
    if isinstance(a, np.ndarray):
        if not a.flags["C_CONTIGUOUS"]:
            raise ValueError("expected a contiguous numpy array")
        return a.ctypes.data, a.nbytes
    torch = _torch()
    if isinstance(a, torch.Tensor) and a.device.type == "cpu" and a.is_contiguous():
        return a.data_ptr(), a.numel() * a.element_size()
    raise ValueError("expected a contiguous numpy array or CPU tensor")


def _host_ptr(a, np_dtype, name):
    torch = None
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover
        pass
    if torch is not None and isinstance(a, torch.Tensor):
        if a.device.type != "cpu" or not a.is_contiguous() or a.dtype != getattr(torch, np.dtype(np_dtype).name):
            raise ValueError(f"{name}: expected a contiguous CPU {np.dtype(np_dtype).name} tensor")
        return a.data_ptr(), a.numel()
    if not isinstance(a, np.ndarray) or a.dtype != np_dtype or not a.flags["C_CONTIGUOUS"]:
        raise ValueError(f"{name}: expected a contiguous numpy {np.dtype(np_dtype).name} array")
    return a.ctypes.data, a.size


def _host_int32_call(fn, handle, src, length, dst):
    sp, sn = _host_ptr(src, np.int32, "src")
    dp, dn = _host_ptr(dst, np.int32, "dst")
    length = int(length)
    n = (length // PAYLOAD_COUNT) * PAYLOAD_COUNT   # api.c:406 whole messages
    if length < 0 or sn < n or dn < n:
        raise ValueError(f"len={length} exceeds src ({sn}) or dst ({dn})")
    fn(handle, sp, ctypes.c_uint32(length), dp)


# -- reference-named entry points (api.h:93-101) --
def inccl_group_create(world_size: int, rank: int, master_ip: str = "127.0.0.1", port: int = 0,
                       device: int = -1) -> Group | None:
    """NULL (None) on failure, like api.c:82-98."""
    h = load().inccl_group_create_ex(int(world_size), int(rank), master_ip.encode(), int(port), int(device))
    return Group(h) if h else None


def inccl_group_create_local(world_size: int, rank: int, hub: str = "default", device: int = -1) -> Group | None:
    h = load().inccl_group_create_local(int(world_size), int(rank), hub.encode(), int(device))
    return Group(h) if h else None


def inccl_group_destroy(group: Group) -> int:
    return group.destroy()


def inccl_communicator_create(group: Group, size: int) -> Communicator | None:
    h = load().inccl_communicator_create(group.handle, ctypes.c_uint32(int(size)))
    return Communicator(group, h) if h else None


def inccl_communicator_destroy(comm: Communicator) -> int:
    return comm.destroy()


def inccl_allreduce_write(comm: Communicator, src_data: np.ndarray, length: int, dst_data: np.ndarray) -> None:
    comm.allreduce_write(src_data, length, dst_data)


def inccl_allreduce_sendrecv(comm: Communicator, src_data: np.ndarray, length: int, dst_data: np.ndarray) -> None:
    comm.allreduce_sendrecv(src_data, length, dst_data)


# ---------------------------------------------------------------------------
# the reference switch's dataplane on the GPU (non_termination_switch.c:303-501,
# util.c:331-442); frames are rows of a uint8 CUDA tensor [count, stride]
# ---------------------------------------------------------------------------
SW_IGNORED, SW_ABSORBED, SW_COMPLETED, SW_DROPPED, SW_REPLAY, SW_ACK, SW_INVALID, SW_FORWARD, SW_DOWN = range(9)
SW_WIRE_ORDER, SW_RECYCLE = 1, 2   # non-root switch flags (inccl_switch_create_nonroot)
FRAME_TEMPLATE_DTYPE = np.dtype([("src_mac", np.uint8, 6), ("dst_mac", np.uint8, 6), ("src_ip", "<u4"),
                                 ("dst_ip", "<u4"), ("src_port", "<u2"), ("dst_port", "<u2"), ("qp", "<u4")])
assert FRAME_TEMPLATE_DTYPE.itemsize == 28


def _frames_arg(frames, name="frames"):
    torch = _torch()
    if frames.dim() != 2:
        raise ValueError(f"{name}: expected [count, stride] uint8")
    if frames.shape[1] % 4:
        raise ValueError(f"{name}: stride must be a multiple of 4")
    # strides below the 62-B ACK frame reach the library, which refuses them
    return _dev_ptr(frames, torch.uint8, name), frames.shape[0], frames.shape[1]


def icrc_frames(frames, stream=None):
    """ICRC (util.c:250-286) of every frame row; returns an int32 tensor of the uint32 values."""
    torch = _torch()
    ptr, count, stride = _frames_arg(frames)
    out = torch.empty(count, dtype=torch.int32, device=frames.device)
    check(load().inccl_icrc_frames(ptr, stride, count, _dev_ptr(out, torch.int32, "out"), _stream_handle(stream)),
          "inccl_icrc_frames")
    return out


class GpuSwitch:
    """A switch whose state and dataplane live on the GPU: the root (fan_in
    children), or with nonroot=True a non-root whose parent is port fan_in
    (non_termination_switch.c:376-400, :408-423, :457-499; `flags`
    SW_WIRE_ORDER | SW_RECYCLE, 0 = the reference).  A non-root has fan_in + 1
    output rows and templates per input frame, the parent's last."""

    def __init__(self, fan_in: int, slots: int = 1024, device: int = -1, nonroot: bool = False, flags: int = 0):
        self.fan_in = int(fan_in)
        self.nonroot = bool(nonroot)
        self.rows = self.fan_in + (1 if self.nonroot else 0)
        if self.nonroot:
            self.handle = load().inccl_switch_create_nonroot(self.fan_in, int(slots), int(device), int(flags))
        else:
            self.handle = load().inccl_switch_create(self.fan_in, int(slots), int(device))
        if not self.handle:
            raise IncclError(load().inccl_last_error().decode(errors="replace"))

    def reset(self, stream=None):
        check(load().inccl_switch_reset(self.handle, _stream_handle(stream)), "inccl_switch_reset")

    def ingress(self, frames, ports, stream=None):
        torch = _torch()
        ptr, count, stride = _frames_arg(frames)
        pp = _dev_ptr(ports, torch.int32, "ports", count)
        action = torch.empty(count, dtype=torch.int32, device=frames.device)
        psn = torch.empty(count, dtype=torch.int32, device=frames.device)
        check(load().inccl_switch_ingress(self.handle, ptr, stride, count, pp, action.data_ptr(), psn.data_ptr(),
                                          _stream_handle(stream)), "inccl_switch_ingress")
        return action, psn

    def _out_args(self, frames, count, templates, out_stride, out, out_len):
        torch = _torch()
        rows = self.rows
        if templates.dtype != torch.uint8 or templates.numel() != 28 * rows:
            raise ValueError(f"templates: {rows} x 28-byte inccl_frame_template records (uint8)")
        if out is None:
            out = torch.empty((count * rows, out_stride), dtype=torch.uint8, device=frames.device)
        elif out.dtype != torch.uint8 or out.dim() != 2 or out.shape[0] < count * rows:
            raise ValueError(f"out: uint8 [count * {rows}, out_stride]")
        if out_len is None:
            out_len = torch.empty(count * rows, dtype=torch.int32, device=frames.device)
        _dev_ptr(out, torch.uint8, "out")
        _dev_ptr(out_len, torch.int32, "out_len", count * rows)
        return out, out_len

    def batch(self, frames, ports, templates, out_stride: int = 1152, stream=None, out=None, out_len=None,
              action=None, psn=None):
        """ingress + egress of one batch in one call (inccl_switch_batch): the
        same actions, PSNs, rows and lengths as ingress() then egress()."""
        torch = _torch()
        ptr, count, stride = _frames_arg(frames)
        pp = _dev_ptr(ports, torch.int32, "ports", count)
        out, out_len = self._out_args(frames, count, templates, out_stride, out, out_len)
        if action is None:
            action = torch.empty(count, dtype=torch.int32, device=frames.device)
        if psn is None:
            psn = torch.empty(count, dtype=torch.int32, device=frames.device)
        check(load().inccl_switch_batch(self.handle, ptr, stride, count, pp, _dev_ptr(action, torch.int32, "action", count),
                                        _dev_ptr(psn, torch.int32, "psn", count),
                                        _dev_ptr(templates, torch.uint8, "templates"), out.data_ptr(), out.shape[1],
                                        out_len.data_ptr(), _stream_handle(stream)), "inccl_switch_batch")
        return action, psn, out, out_len

    def egress(self, frames, ports, action, psn, templates, out_stride: int = 1152, stream=None, out=None,
               out_len=None):
        """Row i * rows + c is row c's frame for input frame i; out_len says
        which rows were written (bytes, or 0).  Unwritten rows keep whatever the
        buffer held: `out` / `out_len` may be passed in and reused."""
        torch = _torch()
        ptr, count, stride = _frames_arg(frames)
        out, out_len = self._out_args(frames, count, templates, out_stride, out, out_len)
        out_stride = out.shape[1]
        check(load().inccl_switch_egress(self.handle, ptr, stride, count, _dev_ptr(ports, torch.int32, "ports", count),
                                         _dev_ptr(action, torch.int32, "action", count),
                                         _dev_ptr(psn, torch.int32, "psn", count),
                                         _dev_ptr(templates, torch.uint8, "templates"), out.data_ptr(), out_stride,
                                         out_len.data_ptr(), _stream_handle(stream)), "inccl_switch_egress")
        return out, out_len

    def result_ptr(self, psn: int) -> int:
        """Device address of a non-root's result slot for `psn` (inccl_switch_result)."""
        p = load().inccl_switch_result(self.handle, int(psn))
        if not p:
            raise IncclError("inccl_switch_result: not a non-root switch")
        return p

    def destroy(self):
        if self.handle:
            load().inccl_switch_destroy(self.handle)
            self.handle = None
