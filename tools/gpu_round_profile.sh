#!/bin/bash
# Full evidence pass: GPU tests -> bench (N=1, all keys) -> rocprofv3 kernel-trace
# stats of the bench's timed workload (--no-extras: the size list and cold run
# would mix other sizes of the same kernel into its average) -> separate PMC
# FETCH_SIZE / WRITE_SIZE passes for the dominant kernels -> 2-rank rehearsal.
# Every GPU step has its own time limit; the script stops at the first abnormal exit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=40 --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
fi
timeout -k 10 600 python -u bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 5; }
echo "bench ok"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extras --json-out gpurun_out/bench_profiled.json > gpurun_out/prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof.log; exit 6; }
grep -h k_stream gpurun_out/prof/run_kernel_stats.csv | cut -c1-200
# the bench's frac_cold (cold_run: four rotated input/output sets, 3 GiB, beyond
# the Infinity Cache) reproduced from a kernel trace: the same rotation, so
# 805,306,368 B / k_stream_vec's average duration / 8 TB/s is frac_cold
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cold -o run --output-format csv -- python3 tools/kernel_probe.py --kernel fused --R 2 --mib 256 --sets 4 --iters 40 > gpurun_out/prof_cold.log 2>&1 || { echo prof cold failed; tail -20 gpurun_out/prof_cold.log; exit 6; }
grep -h k_stream gpurun_out/prof_cold/run_kernel_stats.csv | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bf16 -o run --output-format csv -- python3 tools/kernel_probe.py --kernel bf16 --R 2 --mib 256 --iters 50 > gpurun_out/prof_bf16.log 2>&1 || { echo prof bf16 failed; tail -20 gpurun_out/prof_bf16.log; exit 6; }
for k in fused quant_sum bf16 f16; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${k}_$c -o pmc -- python3 tools/kernel_probe.py --kernel $k --R 2 --mib 256 --iters 5 > gpurun_out/pmc_${k}_$c.log 2>&1 || { echo "pmc $k $c failed"; tail gpurun_out/pmc_${k}_$c.log; exit 7; }
  done
done
echo "pmc ok"
if [ -z "$SKIP_REHEARSAL" ]; then
  bash tools/gpu_rehearse.sh 2 20 5 || exit 8
fi
echo done
