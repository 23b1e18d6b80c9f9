#!/bin/bash
# GPU switch dataplane: tests, then the batch benchmark.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_switch.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/pytest_switch.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/switch_bench.py > gpurun_out/switch_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/switch_bench.log | tail -8
exit $rc
