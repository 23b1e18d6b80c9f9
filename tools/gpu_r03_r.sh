#!/bin/bash
# Round 3: straight-line egress (k_egress_fixed) -- switch tests, then kernel
# stats of tools/switch_bench.py with it and with the generic k_egress (A/B).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_switch.log 2>&1
rc=$?; echo "switch tests rc=$rc"; tail -1 $O/pytest_switch.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_switch.log | head -20; exit $rc; }
for v in fixed generic fixed generic; do
  if [ $v = generic ]; then export INCCL_EGRESS_GENERIC=1; else unset INCCL_EGRESS_GENERIC; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 tools/switch_bench.py > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 6; }
  echo "== $v: $(grep -m1 '"what": "GPU switch' $O/bench_$v.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms"])') ms per batch"
  python3 - $O/prof_$v/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "egress" in r["Name"]:
        print("  ", r["Name"].split("::")[1].split("(")[0][:40], r["Calls"], r["AverageNs"])
PY
done
