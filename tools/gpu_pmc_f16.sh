#!/bin/bash
# fp16 bucket kernel evidence: separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
# passes over k_stream16<F16,F16,2> (2 x 256 MiB), then a kernel-trace stats run.
# Every GPU step has its own limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_f16_$c -o pmc -- python3 tools/kernel_probe.py --kernel f16 --R 2 --mib 256 --iters 5 > gpurun_out/pmc_f16_$c.log 2>&1 || { echo "pmc $c failed"; tail gpurun_out/pmc_f16_$c.log; exit 7; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f16 -o run --output-format csv -- python3 tools/kernel_probe.py --kernel f16 --R 2 --mib 256 --iters 50 > gpurun_out/prof_f16.log 2>&1 || { echo "prof failed"; tail gpurun_out/prof_f16.log; exit 6; }
grep -h k_stream16 gpurun_out/prof_f16/run_kernel_stats.csv | cut -c1-220
tail -3 gpurun_out/prof_f16.log
