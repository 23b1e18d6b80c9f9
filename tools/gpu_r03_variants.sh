#!/bin/bash
# Round 3: the switch kernels' A/B hooks against the oracle (tests/test_gpu_switch_variants.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03variants
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_switch_variants.py --durations=10 > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 5; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest.log | tail -10
