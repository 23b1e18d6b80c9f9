"""Loader for the in-tree ``libinccl_amd.so`` (C ABI of include/api.h + include/inccl_amd.h).

The product has no CPU fallback: if the library is missing this module raises
immediately, and every compute call fails loudly without a GPU.
"""
from __future__ import annotations

import ctypes
import os
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libinccl_amd.so")

# Public symbols, one per declaration in include/api.h and include/inccl_amd.h.
# (name, restype, argtypes)
_P = ctypes.c_void_p
_I = ctypes.c_int
_SZ = ctypes.c_size_t
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_F = ctypes.c_float
_S = ctypes.c_char_p

SIGNATURES = {
    # include/api.h (reference repository/include/api.h:93-101)
    "inccl_group_create": (_P, [_I, _I, _S]),
    "inccl_group_destroy": (_I, [_P]),
    "inccl_communicator_create": (_P, [_P, _U32]),
    "inccl_communicator_destroy": (_I, [_P]),
    "inccl_allreduce_sendrecv": (None, [_P, _P, _U32, _P]),
    "inccl_allreduce_write": (None, [_P, _P, _U32, _P]),
    # include/inccl_amd.h
    "inccl_last_error": (_S, []),
    "inccl_version": (_S, []),
    "inccl_quantise_f32": (_I, [_P, _P, _SZ, _I, _I, _P]),
    "inccl_dequantise_q32": (_I, [_P, _P, _SZ, _I, _I, _P]),
    "inccl_reduce_f32": (_I, [_P, _I, _P, _SZ, _I, _P]),
    "inccl_reduce_f32_auto": (_I, [_P, _I, _P, _SZ, _P, _P]),
    "inccl_quant_sum_f32": (_I, [_P, _I, _P, _SZ, _I, _I, _P]),
    "inccl_sum_q32": (_I, [_P, _I, _P, _SZ, _I, _I, _P]),
    "inccl_sum_dequant_q32": (_I, [_P, _I, _P, _SZ, _I, _I, _P]),
    "inccl_stream_op": (_I, [_I, _I, _P, _I, _P, _SZ, _I, _P, _I, _P]),
    "inccl_absmax_f32": (_I, [_P, _I, _SZ, _P, _I, _P]),
    "inccl_checksum_q32": (_I, [_P, _SZ, _U64, _P, _I, _P]),
    "inccl_choose_scale": (_I, [_F, _I]),
    "inccl_set_tuning": (None, [_I, _I]),
    "inccl_op_create": (_P, [_I, _I, _P, _I, _P, _SZ, _I, _I, _P]),
    "inccl_op_run": (_I, [_P]),
    "inccl_op_destroy": (_I, [_P]),
    "inccl_op_create_allreduce_f32": (_P, [_P, _P, _I, _P, _SZ, _I, _I, _P]),
    "inccl_op_create_allreduce16": (_P, [_P, _I, _P, _I, _P, _SZ, _I, _P]),
    "inccl_group_create_ex": (_P, [_I, _I, _S, _I, _I]),
    "inccl_group_create_local": (_P, [_I, _I, _S, _I]),
    "inccl_group_rank": (_I, [_P]),
    "inccl_group_size": (_I, [_P]),
    "inccl_group_device": (_I, [_P]),
    "inccl_ipc_max_bytes": (_SZ, []),
    "inccl_group_ipc_max_bytes": (_SZ, [_P]),
    "inccl_hsa_runtime_release": (_U32, []),
    "inccl_hsa_runtime_build": (_S, []),
    "inccl_rccl_version": (_I, [_P, _P]),
    "inccl_group_transport": (_S, [_P]),
    "inccl_comm_stream": (_P, [_P]),
    "inccl_comm_barrier": (_I, [_P]),
    "inccl_comm_set_engine": (_I, [_P, _S]),
    "inccl_comm_engine": (_S, [_P]),
    "inccl_comm_ipc_mem_kind": (_I, [_P, _S]),
    "inccl_comm_clear_error": (_I, [_P]),
    "inccl_comm_set_average": (_I, [_P, _I]),
    "inccl_comm_set_nonfinite": (_I, [_P, _I]),
    "inccl_comm_set_stage_timing": (_I, [_P, _I]),
    "inccl_comm_stage_times": (_I, [_P, _P, _I, _P]),
    "inccl_reduce_scatter_f32": (_I, [_P, _P, _I, _P, _SZ, _I, _P]),
    "inccl_reduce_scatter_bf16": (_I, [_P, _P, _I, _P, _SZ, _I, _P]),
    "inccl_reduce_scatter_f16": (_I, [_P, _P, _I, _P, _SZ, _I, _P]),
    "inccl_allreduce_f32": (_I, [_P, _P, _I, _P, _SZ, _I, _P]),
    "inccl_allreduce_f32_pipelined": (_I, [_P, _P, _I, _P, _SZ, _I, _I, _P]),
    "inccl_allreduce_bf16": (_I, [_P, _P, _I, _P, _SZ, _I, _P]),
    "inccl_absmax_bf16": (_I, [_P, _I, _SZ, _P, _I, _P]),
    "inccl_allreduce_f16": (_I, [_P, _P, _I, _P, _SZ, _I, _P]),
    "inccl_absmax_f16": (_I, [_P, _I, _SZ, _P, _I, _P]),
    "inccl_allreduce_q32": (_I, [_P, _P, _P, _SZ, _P]),
    "inccl_allreduce_f32_host": (_I, [_P, _P, _P, _SZ, _I, _SZ]),
    "inccl_host_register": (_I, [_P, _P, _SZ]),
    "inccl_host_deregister": (_I, [_P, _P]),
    "inccl_switch_create": (_P, [_I, _U32, _I]),
    "inccl_switch_create_nonroot": (_P, [_I, _U32, _I, _I]),
    "inccl_switch_result": (_P, [_P, _U32]),
    "inccl_switch_destroy": (_I, [_P]),
    "inccl_switch_reset": (_I, [_P, _P]),
    "inccl_switch_slot": (_P, [_P, _U32]),
    "inccl_switch_ingress": (_I, [_P, _P, _SZ, _SZ, _P, _P, _P, _P]),
    "inccl_switch_egress": (_I, [_P, _P, _SZ, _SZ, _P, _P, _P, _P, _P, _SZ, _P, _P]),
    "inccl_switch_batch": (_I, [_P, _P, _SZ, _SZ, _P, _P, _P, _P, _P, _SZ, _P, _P]),
    "inccl_icrc_frames": (_I, [_P, _SZ, _SZ, _P, _P]),
}

_lib = None


class IncclError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load the library (RTLD_GLOBAL so the HIP runtime is shared with torch)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise IncclError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(make -C container_inc_amd/csrc).  There is no CPU fallback.")
    # torch bundles its own HIP/HSA/RCCL runtimes under the same sonames.  Load
    # it first so this library binds to those copies: loading /opt/rocm's
    # libamdhip64 first and torch's later puts two HSA runtimes in one process.
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - pure C consumers need no torch
        pass
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


RUNTIME_LIBS = ("libamdhip64", "libhsa-runtime64", "librccl", "libinccl_amd")


def runtime_libs() -> dict:
    """Which HIP, HSA and RCCL runtimes this process has mapped, from
    /proc/self/maps, and the HIP runtime's version (hipRuntimeGetVersion of the
    copy the process bound to).  libinccl_amd.so is built against /opt/rocm's
    headers but, loaded after torch, binds to torch's bundled runtimes (same
    sonames); a C program binds to /opt/rocm's.  This records which."""
    found = {}
    try:
        with open("/proc/self/maps") as f:
            for ln in f:
                parts = ln.split()
                if len(parts) < 6:
                    continue
                path = parts[5]
                base = os.path.basename(path)
                for key in RUNTIME_LIBS:
                    if base.startswith(key + ".so") and key not in found:
                        found[key] = os.path.realpath(path)
    except OSError:
        pass
    if "libamdhip64" in found:
        try:
            hip = ctypes.CDLL(found["libamdhip64"])
            v = ctypes.c_int(0)
            if hip.hipRuntimeGetVersion(ctypes.byref(v)) == 0:
                found["hip_runtime_version"] = v.value
        except OSError:
            pass
    if "libinccl_amd" in found:
        # RCCL: the NCCL_VERSION_CODE the library was compiled against and the
        # ncclGetVersion of the librccl it bound to; the HSA runtime's own ROCm
        # release (its build string), which sets the IPC bound (csrc/runtime.c)
        lib = load()
        c, ld = ctypes.c_int(0), ctypes.c_int(0)
        if lib.inccl_rccl_version(ctypes.byref(c), ctypes.byref(ld)) == 0:
            found["rccl_compiled"], found["rccl_loaded"] = c.value, ld.value
        # the HSA queries initialise HIP (hipInit + hsa_init, csrc/runtime.c):
        # only asked in a process that has initialised the GPU already, so that
        # reporting versions never initialises it behind the caller's back (a
        # launcher that forks or relaunches afterwards must not have a GPU
        # context)
        torch = sys.modules.get("torch")
        if torch is not None and torch.cuda.is_initialized():
            found["hsa_release"] = int(lib.inccl_hsa_runtime_release())
            found["hsa_build"] = lib.inccl_hsa_runtime_build().decode(errors="replace")
            found["ipc_max_bytes"] = int(lib.inccl_ipc_max_bytes())
        else:
            found["hsa_release"] = found["hsa_build"] = found["ipc_max_bytes"] = None
            found["hsa_note"] = "not queried: the GPU is not initialised in this process (the query would do it)"
    return found


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().inccl_last_error().decode(errors="replace")
        raise IncclError(f"{what} failed (rc={rc}): {msg}")
