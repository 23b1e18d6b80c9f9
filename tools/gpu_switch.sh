#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "switch or icrc or p2p" > gpurun_out/pytest_sw.log 2>&1 || { echo tests failed; tail -30 gpurun_out/pytest_sw.log; exit 4; }
tail -2 gpurun_out/pytest_sw.log
timeout -k 10 600 python tools/switch_bench.py > gpurun_out/switch_bench.log 2>&1 || { echo failed; tail -20 gpurun_out/switch_bench.log; exit 5; }
cat gpurun_out/switch_bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profsw -o run --output-format csv -- python tools/switch_bench.py > gpurun_out/profsw.log 2>&1 || { echo prof failed; tail gpurun_out/profsw.log; exit 7; }
