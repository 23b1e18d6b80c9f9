#!/bin/bash
# Round 3: the switch tests (fan-in 1 and 31 added)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_switch.log 2>&1
rc=$?; tail -1 $O/pytest_switch.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_switch.log | head -20; exit $rc; }
