#!/bin/bash
# ll kernel grid-cap sweep (two processes on one GPU)
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
for cap in 8 32 64 128 256; do
  timeout -k 10 200 python tools/ll_sweep.py --grid-cap $cap --out gpurun_out/ll_sweep_cap$cap.jsonl > gpurun_out/ll_sweep_cap$cap.log 2>&1 || exit $?
  echo "cap $cap"; cat gpurun_out/ll_sweep_cap$cap.jsonl | python3 -c "import sys,json;[print(d['bucket_bytes'],d['us_per_call_p2p'],d['us_per_call_ll'],d['bit_equal']) for d in map(json.loads,sys.stdin)]"
done
