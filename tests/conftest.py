"""Shared test setup.

Markers: ``gpu`` -- needs a real MI355X (run with ``-m gpu``).  Everything else
runs on CPU: the oracle against the golden fixtures, the C-ABI surface of
libinccl_amd.so (loads + exports, no compute), the TCP bootstrap, and the
multi-rank shard plan over ``gloo``.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_sessionstart(session):
    """Which HIP / HSA / RCCL copies this test process is bound to (DESIGN.md
    "Runtimes"), at the top of every test log (-q included)."""
    tr = session.config.pluginmanager.get_plugin("terminalreporter")
    if tr is not None:
        tr.write_line(_runtime_line())


def _runtime_line():
    try:
        import torch  # noqa: F401 -- loaded first, as the package does
        import container_inc_amd as cia
        if os.path.exists(cia.LIB_PATH):
            cia.load()
        from container_inc_amd._lib import runtime_libs
        return f"runtime: {runtime_libs()}"
    except Exception as e:  # noqa: BLE001
        return f"runtime: unknown ({e!r})"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP kernels / RCCL)")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def lib():
    import container_inc_amd as cia
    if not os.path.exists(cia.LIB_PATH):
        cia.build()
    return cia.load()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    import container_inc_amd as cia
    if not os.path.exists(cia.LIB_PATH):
        cia.build()
    cia.load()
    # The multi-process tests put every rank on this one GPU.  Processes started
    # from here on (this process's HIP runtime is already up, so it keeps its
    # own count) open two hardware queues each instead of four: eight ranks x
    # four queues oversubscribe the GPU's queue slots and the scheduler time-
    # slices the ranks (DESIGN.md "Mesh reduce-scatter route", liveness).
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("INCCL_TEST_RANK_HW_QUEUES", "2")
    return torch.device("cuda:0")
