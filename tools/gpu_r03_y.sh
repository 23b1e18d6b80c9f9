#!/bin/bash
# Round 3: k_egress_fixed at 2 vs 3 resident 8-wave blocks per CU (16 vs 24 waves).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03y
mkdir -p $O
export TMPDIR=/tmp
for v in 2 3 2 3 1; do
  INCCL_EGRESS_BLOCKS_PER_CU=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 tools/switch_bench.py > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 6; }
  python3 - $O/prof_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "egress" in r["Name"]:
        print("blocks/CU", sys.argv[2], r["Name"].split("::")[1].split("(")[0][:30], r["Calls"], r["AverageNs"])
PY
done
