#!/bin/bash
# Switch tests + the switch batch with and without ACKs, under rocprofv3.
cd "$GRAFT_REPO_ROOT" || exit 3
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/switch_confirm.log 2>&1 || { tail -20 gpurun_out/switch_confirm.log; exit 4; }
tail -1 gpurun_out/switch_confirm.log
bash tools/gpu_switch_acks.sh ${1:-_confirm}
