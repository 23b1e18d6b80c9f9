#!/bin/bash
# a -k selection of the GPU suite ($1), with the regrowth trace on
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
INCCL_TRACE=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "$1" > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/pytest_quick.log | tail -12
exit $rc
