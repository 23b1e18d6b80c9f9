#!/bin/bash
# Round 3: ICRC without LDS staging (k_icrc_direct, INCCL_ICRC_DIRECT=1; 1 or 2 pairs per
# pass, INCCL_ICRC_PAIRS_PER_PASS): the switch/ICRC GPU tests on each, then the ICRC leg of
# switch_bench A/B against k_icrc_pair, twice each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03direct
mkdir -p $O
export TMPDIR=/tmp
for pp in 2 1; do
  INCCL_ICRC_DIRECT=1 INCCL_ICRC_PAIRS_PER_PASS=$pp timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_switch.py > $O/pytest_direct_pp$pp.log 2>&1 || { tail -30 $O/pytest_direct_pp$pp.log; exit 5; }
  tail -1 $O/pytest_direct_pp$pp.log
done
i=0
for v in "INCCL_ICRC_DIRECT=0" "INCCL_ICRC_DIRECT=1 INCCL_ICRC_PAIRS_PER_PASS=1" "INCCL_ICRC_DIRECT=1 INCCL_ICRC_PAIRS_PER_PASS=2" "INCCL_ICRC_DIRECT=1 INCCL_ICRC_PAIRS_PER_PASS=2 INCCL_ICRC_BLOCKS_PER_CU=3" \
         "INCCL_ICRC_DIRECT=0" "INCCL_ICRC_DIRECT=1 INCCL_ICRC_PAIRS_PER_PASS=1" "INCCL_ICRC_DIRECT=1 INCCL_ICRC_PAIRS_PER_PASS=2" "INCCL_ICRC_DIRECT=1 INCCL_ICRC_PAIRS_PER_PASS=2 INCCL_ICRC_BLOCKS_PER_CU=3"; do
  i=$((i+1))
  env $v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$i -o run --output-format csv -- python3 tools/switch_bench.py > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 6; }
  python3 - $O/prof_$i/run_kernel_stats.csv "$v" <<'PY'
import csv, sys, re
out = []
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_icrc\w*)", r["Name"])
    if m:
        out.append("%s=%.1f" % (m.group(1), float(r["AverageNs"]) / 1e3))
print(sys.argv[2], " ".join(out))
PY
done
