#!/bin/bash
# bench (new default grid) + rocprof stats -> host-memory rates -> size sweep
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench3.json > gpurun_out/bench3.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench3.log; exit 5; }
cat gpurun_out/bench3.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof3.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof3.log; exit 6; }
grep -h k_stream gpurun_out/prof3/run_kernel_stats.csv | cut -c1-200
timeout -k 10 600 python tools/host_bench.py > gpurun_out/host_bench.log 2>&1 || { echo host_bench failed; tail -20 gpurun_out/host_bench.log; exit 7; }
cat gpurun_out/host_bench.log
timeout -k 10 600 python tools/sweep_bench.py > gpurun_out/sweep_sizes.log 2>&1 || { echo sweep failed; tail -20 gpurun_out/sweep_sizes.log; exit 8; }
cat gpurun_out/sweep_sizes.log
