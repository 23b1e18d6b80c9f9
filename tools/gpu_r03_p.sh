#!/bin/bash
# Round 3: the fused switch pass (inccl_switch_process) -- switch tests in both
# modes, then kernel stats of tools/switch_bench.py (separate and fused).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_switch.log 2>&1
rc=$?; echo "switch tests rc=$rc"; tail -1 $O/pytest_switch.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_switch.log | head -20; exit $rc; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/switch_bench.py > $O/switch_bench.log 2>&1 || { tail -20 $O/switch_bench.log; exit 6; }
grep '"what"' $O/switch_bench.log
python3 - $O/prof/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "namespace" in r["Name"]:
        print(r["Name"].split("::")[1].split("(")[0][:30], r["Calls"], r["AverageNs"])
PY
