#!/bin/bash
# Round 3: ICRC kernel A/B -- nibble tables (product) vs byte tables -- with the
# ICRC tests under each, and a kernel trace of the switch bench for each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03l
mkdir -p $O
for b in 0 1; do
  INCCL_ICRC_BYTE_TABLES=$b timeout -k 10 200 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -q --timeout 200 --timeout-method thread -k icrc > $O/pytest_icrc_b$b.log 2>&1
  rc=$?; echo "icrc tests byte_tables=$b rc=$rc"; tail -1 $O/pytest_icrc_b$b.log; [ $rc -eq 0 ] || exit $rc
  INCCL_ICRC_BYTE_TABLES=$b timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_b$b -o run --output-format csv -- python3 tools/switch_bench.py > $O/prof_b$b.log 2>&1 || exit 6
  python3 - $O/prof_b$b/run_kernel_stats.csv $b <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_icrc" in r["Name"]:
        print("byte_tables", sys.argv[2], r["Name"].split("::")[1].split("(")[0][:30], r["Calls"], r["AverageNs"])
PY
done
