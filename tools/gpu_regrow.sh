#!/bin/bash
# IPC regrowth test (3 ranks on one GPU, p2p and mesh) with the per-growth
# handle / mapping trace on.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
INCCL_TRACE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_regrow.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_regrow.log 2>&1
rc=$?; echo "regrow rc=$rc"; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/pytest_regrow.log | tail -6
exit $rc
