#!/bin/bash
# Full evidence pass: GPU tests -> bench (N=1) -> rocprofv3 kernel-trace stats of
# the same bench command (its own JSON line kept beside the stats, so the live
# HIP-event kernel time and the profiled average come from one process) -> PMC FETCH_SIZE / WRITE_SIZE passes for the dominant kernels.
# Every GPU step has its own time limit; the script stops at the first abnormal exit.
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 5; }
cat gpurun_out/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline --json-out gpurun_out/bench_profiled.json > gpurun_out/prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof.log; exit 6; }
grep -h k_stream gpurun_out/prof/run_kernel_stats.csv | cut -c1-220
cat gpurun_out/bench_profiled.json
for k in fused quant_sum; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${k}_$c -o pmc -- python tools/kernel_probe.py --kernel $k --R 2 --mib 256 --iters 5 > gpurun_out/pmc_${k}_$c.log 2>&1 || { echo "pmc $k $c failed"; tail gpurun_out/pmc_${k}_$c.log; exit 7; }
  done
done
echo done
