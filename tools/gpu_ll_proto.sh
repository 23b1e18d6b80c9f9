#!/bin/bash
# ll kernel protocols (write-through vs fences): tests on the default, then both sweeps
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_p2p.py -q -x > gpurun_out/pytest_p2p.log 2>&1; rc=$?
echo "p2p/ll tests rc=$rc"; tail -5 gpurun_out/pytest_p2p.log
[ $rc -ne 0 ] && exit $rc
for proto in wt fence; do
  INCCL_LL_PROTOCOL=$proto timeout -k 10 300 python tools/ll_sweep.py --out gpurun_out/ll_sweep_$proto.jsonl > gpurun_out/ll_sweep_$proto.log 2>&1 || exit $?
  echo "protocol $proto"; python3 -c "import sys,json;[print(d['bucket_bytes'],d['us_per_call_p2p'],d['us_per_call_ll'],d['us_per_call_ll_graph'],d['bit_equal']) for d in map(json.loads,open('gpurun_out/ll_sweep_$proto.jsonl'))]"
done
