#!/bin/bash
# Round 3: k_icrc_pair (two frames per wave, 32-lane halves) vs k_icrc, after the
# switch/ICRC tests with each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03pair
mkdir -p $O
export TMPDIR=/tmp
for v in 1 0; do
  INCCL_ICRC_PAIR=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_switch_w$v.log 2>&1 || { echo "tests waves=$v failed"; tail -5 $O/pytest_switch_w$v.log; exit 5; }
done
echo "switch + ICRC tests ok paired and unpaired"
for v in 1 0 1 0; do
  INCCL_ICRC_PAIR=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 tools/switch_bench.py > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 6; }
  python3 - $O/prof_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "icrc" in r["Name"]:
        print("pair", sys.argv[2], r["Name"].split("::")[1].split("(")[0][:30], r["Calls"], r["AverageNs"])
PY
done
