#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 3
export TMPDIR=/tmp
cp container_inc_amd/libinccl_amd.so /tmp/keep.so
for G in ${VARIANTS:-v20 v21 v41 v20 v21 v41}; do
  cp container_inc_amd/libinccl_amd_$G.so container_inc_amd/libinccl_amd.so
  timeout -k 10 200 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -q --timeout 100 --timeout-method thread  > gpurun_out/ab_g$G.log 2>&1 || { tail gpurun_out/ab_g$G.log; exit 4; }
  echo "G=$G tests: $(tail -1 gpurun_out/ab_g$G.log)"
  bash tools/gpu_switch_acks.sh _g$G > /dev/null || exit 5
  for a in 0 1; do python3 - <<PY
import csv
rows=list(csv.DictReader(open('gpurun_out/swacks_g$G/kernel_stats_acks$a.csv')))
print("G=$G acks=$a", [(r["Name"].split("namespace)::")[1].split("(")[0], round(float(r["AverageNs"])/1e3,2)) for r in rows if "k_" in r["Name"] and "namespace)::" in r["Name"]])
PY
  cat gpurun_out/swacks_g$G/acks$a.jsonl | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('  batch us', r['us_per_batch'])"
  done
done
cp /tmp/keep.so container_inc_amd/libinccl_amd.so
