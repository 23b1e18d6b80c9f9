#!/bin/bash
# Round 3: ingress apply frames per wave (1 / 2 / 4) after the recycle change.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03z
mkdir -p $O
export TMPDIR=/tmp
for v in 2 1 4 2 1 4; do
  INCCL_APPLY_FRAMES=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 tools/switch_bench.py > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 6; }
  python3 - $O/prof_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "apply" in r["Name"]:
        print("frames/wave", sys.argv[2], r["Name"].split("::")[1].split("(")[0][:30], r["Calls"], r["AverageNs"])
PY
done
