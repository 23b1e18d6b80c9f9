#!/bin/bash
# stream-kernel store policy change: correctness, then hot/cold and per-R sweeps, then the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_edges.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 gpurun_out/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 5 120 ./tools/tune/tune_cold > gpurun_out/tune_cold_wt.jsonl 2>&1 || exit 4
timeout -k 5 200 ./tools/tune/tune_stream > gpurun_out/tune_stream_wt.jsonl 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --json-out gpurun_out/bench_wt.json > gpurun_out/bench_wt.log 2>&1 || exit 6
python3 -c "
import json; d=json.load(open('gpurun_out/bench_wt.json')); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline_cold'], d['sizes'], d['host_e2e']['GBps'])"
