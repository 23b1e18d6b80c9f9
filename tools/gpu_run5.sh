#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 ./tools/tune/tune_stream > gpurun_out/tune_stream.log 2>&1 || { echo tune failed; tail gpurun_out/tune_stream.log; exit 5; }
cat gpurun_out/tune_stream.log
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmcq_$c -o pmc -- python tools/kernel_probe.py --kernel quant_sum --R 2 --mib 256 --iters 5 > gpurun_out/pmcq_$c.log 2>&1 || { echo "pmc $c failed"; tail gpurun_out/pmcq_$c.log; exit 6; }
done
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
exit $rc
