"""container_inc_amd -- MI355X-native engine for the INCCL gradient-aggregation hot path.

C ABI: ``include/api.h`` (drop-in for In-NetLab/container_inc's
``repository/include/api.h``) and ``include/inccl_amd.h`` (additive fp32 /
device API), implemented by ``libinccl_amd.so`` (C11 host code + HIP kernels
for gfx950 + RCCL).  ``container_inc_amd.inccl`` is the Python host mirror.
"""
import os
import subprocess

from . import inccl  # noqa: F401
from ._lib import LIB_PATH, IncclError, load  # noqa: F401

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")


def build(jobs: int = 4) -> str:
    """Compile libinccl_amd.so in-tree (hipcc --offload-arch=gfx950 + gcc)."""
    subprocess.check_call(["make", "-s", f"-j{jobs}", "-C", CSRC])
    return LIB_PATH
