#!/bin/bash
# Round 3: switch tests and kernel trace after the packed nibble-index lookups
# (CRC segment lookups in k_icrc and k_egress).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_switch.log 2>&1
rc=$?; echo "switch tests rc=$rc"; tail -1 $O/pytest_switch.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_switch.log | head; exit $rc; }
for i in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$i -o run --output-format csv -- python3 tools/switch_bench.py > $O/prof_$i.log 2>&1 || exit 6
  python3 - $O/prof_$i/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "namespace" in r["Name"]:
        print(r["Name"].split("::")[1].split("(")[0][:30], r["Calls"], r["AverageNs"])
PY
done
grep '"what"' $O/prof_1.log | head -2
