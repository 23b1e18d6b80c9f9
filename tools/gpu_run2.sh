#!/bin/bash
# tests -> PMC traffic passes (FETCH_SIZE, WRITE_SIZE separately) -> tuning sweep
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$c -o pmc -- python tools/kernel_probe.py --kernel fused --R 2 --mib 256 --iters 5 > gpurun_out/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail gpurun_out/pmc_$c.log; exit 6; }
done
timeout -k 10 300 python tools/kernel_probe.py --sweep --iters 30 > gpurun_out/sweep.log 2>&1 || { echo sweep failed; tail gpurun_out/sweep.log; exit 7; }
cat gpurun_out/sweep.log
