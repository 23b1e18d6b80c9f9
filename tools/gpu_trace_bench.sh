#!/bin/bash
# the driver's N=1 bench command, then the same under rocprofv3 --kernel-trace with per-launch analysis
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --json-out gpurun_out/bench_driverflags.json > gpurun_out/bench_driverflags.log 2>&1 || { tail gpurun_out/bench_driverflags.log; exit 4; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_driverflags.json')); print('driver flags:', d['value'], d['ms_per_step'], d['settle_steps'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline_cold']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o run -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extras --json-out gpurun_out/bench_traced.json > gpurun_out/trace.log 2>&1 || { tail gpurun_out/trace.log; exit 5; }
python3 - <<'P'
import csv, json
rows = [r for r in csv.DictReader(open("gpurun_out/trace/run_kernel_trace.csv")) if "k_stream_vec" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print("launches", len(rows))
print(" ".join(f"{x:.0f}" for x in d))
b = json.load(open("gpurun_out/bench_traced.json"))
s = b["settle_steps"]
timed = d[s + 10: s + 60]
print("timed steps: mean", round(sum(timed) / len(timed), 2), "bench ms_per_step", b["ms_per_step"], "kernel_ms", b["roofline"]["kernel_ms"])
P
