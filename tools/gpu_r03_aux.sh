#!/bin/bash
# Round 3: egress output-store cache policy (aux 0 / sc1 16 / nt 2 / sc1|nt 18), twice each.
# (INCCL_EGRESS_AUX was a temporary hook of that experiment; the kept form is INCCL_EGRESS_NT.)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03aux
mkdir -p $O
export TMPDIR=/tmp
for v in 0 16 2 18 0 16 2 18; do
  INCCL_EGRESS_AUX=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 tools/switch_bench.py > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 6; }
  python3 - $O/prof_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "egress" in r["Name"]:
        print("aux", sys.argv[2], r["Name"].split("(")[0][-40:], r["Calls"], r["AverageNs"])
PY
  grep -m1 "ms per batch" $O/bench_$v.log || true
done
