#!/bin/bash
# Round 3: switch tests + variant tests, then two switch_bench runs under rocprofv3, on the current defaults.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03sw2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_switch.py tests/test_gpu_switch_variants.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 5; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$i -o run --output-format csv -- python3 tools/switch_bench.py > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 6; }
  python3 - $O/prof_$i/run_kernel_stats.csv <<'PY'
import csv, sys, re
out = []
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_\w+)", r["Name"])
    if m:
        out.append("%s=%.1f" % (m.group(1), float(r["AverageNs"]) / 1e3))
print(" ".join(out))
PY
  grep -h '"ms"' $O/bench_$i.log | cut -c1-200 || true
done
