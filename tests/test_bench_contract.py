"""bench.py's pure helpers on CPU: the N > 1 xGMI roofline arithmetic and the
sweep's size list (BASELINE config 5 plus north_star's 1024 MiB point)."""
import importlib
import sys

from conftest import ROOT


def _bench():
    sys.path.insert(0, ROOT)
    return importlib.import_module("bench")


def test_xgmi_roofline_arithmetic():
    b = _bench()
    B = 256 << 20
    for W in (2, 4, 8):
        t = 1e-3
        r = b.xgmi_roofline(W, B, t)
        link_bytes = 4 * (W - 1) * B // W     # RS + AG, int32 then fp32, both directions counted
        assert r["link_bytes_per_rank_per_step"] == link_bytes
        assert r["bound"] == "xgmi" and r["unit"] == "GB/s"
        assert abs(r["peak"] - (W - 1) * b.XGMI_LINK_GBS_BIDIR) < 0.1
        assert abs(r["achieved"] - link_bytes / t / 1e9) < 0.1
        assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3


def test_sweep_sizes():
    b = _bench()
    sizes = b.SWEEP_BYTES
    assert sizes[0] == 4 << 10                      # one reference message (api.h:39)
    assert (256 << 20) in sizes and (1 << 30) in sizes
    assert all(y == 4 * x for x, y in zip(sizes[:-2], sizes[1:-1]))   # x4 steps up to 256 MiB
