#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
timeout -k 10 600 python tools/switch_bench.py > gpurun_out/switch_bench.log 2>&1 || { echo failed; tail -20 gpurun_out/switch_bench.log; exit 5; }
cat gpurun_out/switch_bench.log
SW_FAN_IN=8 SW_PSNS=16384 timeout -k 10 600 python tools/switch_bench.py > gpurun_out/switch_bench8.log 2>&1 || { echo failed; tail -20 gpurun_out/switch_bench8.log; exit 6; }
cat gpurun_out/switch_bench8.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profsw -o run --output-format csv -- python tools/switch_bench.py > gpurun_out/profsw.log 2>&1 || { echo prof failed; tail gpurun_out/profsw.log; exit 7; }
cut -c1-160 gpurun_out/profsw/run_kernel_stats.csv | head -12
