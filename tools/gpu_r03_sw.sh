#!/bin/bash
# Round 3: switch GPU tests + switch_bench under rocprofv3 on the current defaults.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03sw
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_switch.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 5; }
tail -2 $O/pytest.log
for i in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$i -o run --output-format csv -- python3 tools/switch_bench.py > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 6; }
  python3 - $O/prof_$i/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("claim", "apply", "commit", "egress", "icrc")):
        print("%-40s %5s %8.1f us" % (n.split("(")[0][-40:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  grep -m3 "ms per batch\|GB/s" $O/bench_$i.log || true
done
