#!/bin/bash
# GPU session: tests -> smoke -> bench -> rocprof kernel-trace stats.  Stops at the
# first step that ends abnormally (fault, abort, timeout); a plain test failure
# (pytest exit 1) still lets the measurement steps run.
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 4; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench1.json > gpurun_out/bench1.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench1.log; exit 5; }
cat gpurun_out/bench1.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof.log; exit 6; }
find gpurun_out/prof -name '*stats*' | head
