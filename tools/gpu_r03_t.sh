#!/bin/bash
# Round 3: ingress apply waves per workgroup (1 / 2 / 4) -- kernel stats of
# tools/switch_bench.py per setting, after the switch tests at the non-default ones.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03t
mkdir -p $O
export TMPDIR=/tmp
for v in 8 16; do
  INCCL_APPLY_WPB=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_switch_wpb$v.log 2>&1 || { echo "tests wpb=$v failed"; tail -5 $O/pytest_switch_wpb$v.log; exit 5; }
done
echo "switch tests ok at 8 and 16 waves per workgroup"
for v in 4 8 16 4 8 16; do
  INCCL_APPLY_WPB=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 tools/switch_bench.py > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 6; }
  python3 - $O/prof_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "apply" in r["Name"]:
        print("wpb", sys.argv[2], r["Name"].split("::")[1].split("(")[0][:30], r["Calls"], r["AverageNs"])
PY
done
