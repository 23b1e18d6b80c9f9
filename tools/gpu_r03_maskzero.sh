#!/bin/bash
# Round 3: ICRC mask + leading-byte zeroing from one 32-entry (AND, OR) LDS table (INCCL_ICRC_MASK_LDS=2) vs the mask table alone (1):
# the variant child against the oracle, then the ICRC leg of switch_bench, three runs each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03maskzero
mkdir -p $O
export TMPDIR=/tmp
INCCL_ICRC_MASK_LDS=2 timeout -k 10 240 python3 -u tests/switch_variant_child.py > $O/child.log 2>&1 || { tail -30 $O/child.log; exit 5; }
tail -1 $O/child.log
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_switch.py tests/test_gpu_switch_variants.py > $O/pytest_default.log 2>&1 || { tail -30 $O/pytest_default.log; exit 5; }
tail -1 $O/pytest_default.log
i=0
for v in "INCCL_ICRC_MASK_LDS=1" "INCCL_ICRC_MASK_LDS=2" "INCCL_ICRC_MASK_LDS=1" "INCCL_ICRC_MASK_LDS=2" "INCCL_ICRC_MASK_LDS=1" "INCCL_ICRC_MASK_LDS=2"; do
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
