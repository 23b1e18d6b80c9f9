#!/bin/bash
# p2p engine: multi-process tests, the back-to-back stress script, N=2 rehearsal
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_p2p.py -q -x > gpurun_out/pytest_p2p.log 2>&1; rc=$?
echo "p2p tests rc=$rc"; tail -5 gpurun_out/pytest_p2p.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/p2p_debug.py > gpurun_out/p2p_debug.log 2>&1; rc=$?
echo "p2p_debug rc=$rc"; grep -v amdgpu.ids gpurun_out/p2p_debug.log | tail -8
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_rehearse_n2.sh
