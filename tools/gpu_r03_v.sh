#!/bin/bash
# Round 3: k_egress_fixed at 14 waves per block (2 per CU = 28 waves) vs 8 (3 per
# CU = 24 waves), after the switch tests at both; SDWA + v_bitop3 in seg16_crc.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03v
mkdir -p $O
export TMPDIR=/tmp
for v in 7 8; do
  INCCL_EGRESS_WAVES=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_switch_w$v.log 2>&1 || { echo "tests waves=$v failed"; tail -5 $O/pytest_switch_w$v.log; exit 5; }
done
echo "switch tests ok at 7 and 8 waves per block"
for v in 7 8 7 8; do
  INCCL_EGRESS_WAVES=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 tools/switch_bench.py > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 6; }
  python3 - $O/prof_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "egress" in r["Name"]:
        print("waves", sys.argv[2], r["Name"].split("::")[1].split("(")[0][:30], r["Calls"], r["AverageNs"])
PY
done
