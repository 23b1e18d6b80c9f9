#!/bin/bash
# ll engine: multi-process tests (p2p + ll + peer timeout), then the small-bucket sweep
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_p2p.py -q -x > gpurun_out/pytest_p2p.log 2>&1; rc=$?
echo "p2p/ll tests rc=$rc"; tail -30 gpurun_out/pytest_p2p.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ll_sweep.py --out gpurun_out/ll_sweep.jsonl > gpurun_out/ll_sweep.log 2>&1; rc=$?
echo "ll sweep rc=$rc"; grep -v amdgpu.ids gpurun_out/ll_sweep.log | tail -12
exit $rc
