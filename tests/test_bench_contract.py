"""bench.py's pure helpers on CPU: the N > 1 xGMI roofline arithmetic and the
sweep's size list (BASELINE config 5 plus north_star's 1024 MiB point)."""
import importlib
import sys

import pytest

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


def test_oracle_lanes_cover_boundaries():
    b = _bench()
    from container_inc_amd.plan import chunk_plan
    for n, W, ch in ((1 << 20, 8, 1), ((1 << 20) + 37, 3, 4), (1000, 2, 1), (64, 8, 1)):
        lanes = b.oracle_lanes(n, W, ch, 4096)
        assert lanes == sorted(set(lanes)) and lanes[0] == 0 and lanes[-1] == n - 1
        s = set(lanes)
        for off, cnt, shard in chunk_plan(n, W, ch):
            for g in range(W):
                c = off + g * shard
                if 0 < c < n:
                    assert c in s and c - 1 in s
        for g in range(1, W):
            assert n * g // W in s


def test_oracle_check_world1_detects_mismatch(orc):
    """The bench's sampled oracle check at world 1, on CPU tensors: the
    oracle's own result passes, one flipped lane at a sampled index fails."""
    import numpy as np
    import torch
    b = _bench()
    rng = np.random.default_rng(5)
    xs = [rng.standard_normal(5000).astype(np.float32) for _ in range(3)]
    want = orc.reduce_f32(xs, 25)
    srcs = [torch.from_numpy(x) for x in xs]
    out = torch.from_numpy(want.copy())
    lanes = b.oracle_lanes(5000, 1, 1, 100)
    r = b.oracle_check(srcs, out, lanes, 25, 0, 1)
    assert r["mismatches"] == 0 and r["lanes"] == len(lanes)
    out[lanes[7]] += 1.0
    assert b.oracle_check(srcs, out, lanes, 25, 0, 1)["mismatches"] == 1


def test_world_size_mismatch_is_an_error():
    import os
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], capture_output=True,
                       text=True, env=env, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=2 but --gpus=1" in p.stderr


def test_watchdog_emits_line_and_exits_nonzero():
    """A run past its budget prints one JSON line naming the stuck stage and
    exits 3 (a hang never reads as success)."""
    import json
    import os
    import subprocess
    code = ("import sys, time; sys.path.insert(0, %r); import bench; bench.STAGE['stage'] = 'sweep 4096 B engine x'; "
            "w = bench.Watchdog(1.0, 0); time.sleep(30)" % ROOT)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 3, p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["value"] is None and "sweep 4096 B engine x" in line["error"]


@pytest.mark.parametrize("fmt", ["bf16", "f16"])
def test_oracle_check_16bit_world1(orc, fmt):
    import numpy as np
    import torch
    b = _bench()
    rng = np.random.default_rng(6)
    conv, red, dt = ((orc.f32_to_bf16, orc.reduce_bf16, torch.bfloat16) if fmt == "bf16"
                     else (orc.f32_to_f16, orc.reduce_f16, torch.float16))
    xs = [conv(rng.standard_normal(700).astype(np.float32)) for _ in range(2)]
    want = red(xs, 25)
    srcs = [torch.from_numpy(x.view(np.int16)).view(dt) for x in xs]
    out = torch.from_numpy(want.view(np.int16).copy()).view(dt)
    lanes = b.oracle_lanes(700, 1, 1, 50)
    assert b.oracle_check(srcs, out, lanes, 25, 0, 1, fmt=fmt)["mismatches"] == 0
    out.view(torch.int16)[lanes[2]] ^= 1
    assert b.oracle_check(srcs, out, lanes, 25, 0, 1, fmt=fmt)["mismatches"] == 1


def _keeper_run(body: str):
    import os
    import subprocess
    code = ("import sys, os, signal; sys.path.insert(0, %r); import bench; bench.KEEPER[0] = bench.LineKeeper(); "
            % ROOT) + body
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                          env=dict(os.environ))


def test_line_keeper_prints_when_rank0_dies():
    """Rank 0 killed (SIGKILL: no handler runs) after the headline: the keeper
    prints the measured line with the stage it died in."""
    import json
    p = _keeper_run("bench.RESULT[0] = {'metric': bench.METRIC, 'value': 12.5, 'sweep': [{'bucket_bytes': 4096}]}; "
                    "bench.set_stage('sweep 16384 B engine mesh'); os.kill(os.getpid(), signal.SIGKILL)")
    assert p.returncode == -9
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["value"] == 12.5 and line["sweep"] == [{"bucket_bytes": 4096}]
    assert "sweep 16384 B engine mesh" in line["error"] and "headline measured" in line["error"]


def test_line_keeper_before_headline_and_silent_after_print():
    import json
    p = _keeper_run("bench.set_stage('engine tuning: mesh'); os._exit(7)")
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 7 and line["value"] is None and "engine tuning: mesh" in line["error"]
    p = _keeper_run("bench.RESULT[0] = {'metric': bench.METRIC, 'value': 1.0}; print('{\"the\": \"line\"}', flush=True); "
                    "bench.KEEPER[0].update(printed=True)")
    assert p.returncode == 0 and p.stdout.strip().splitlines() == ['{"the": "line"}']
