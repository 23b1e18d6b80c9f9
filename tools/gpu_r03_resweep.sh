#!/bin/bash
# Round 3: launch geometry re-swept after the non-temporal stores: apply waves per
# workgroup (INCCL_APPLY_WPB 2 / 4 / 8) and egress blocks per CU (INCCL_EGRESS_BLOCKS_PER_CU
# 2 / 3 / 4), each setting twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03resweep
mkdir -p $O
export TMPDIR=/tmp
i=0
for v in "X=0" "INCCL_APPLY_WPB=2" "INCCL_APPLY_WPB=8" "INCCL_EGRESS_BLOCKS_PER_CU=2" "INCCL_EGRESS_BLOCKS_PER_CU=4" \
         "X=0" "INCCL_APPLY_WPB=2" "INCCL_APPLY_WPB=8" "INCCL_EGRESS_BLOCKS_PER_CU=2" "INCCL_EGRESS_BLOCKS_PER_CU=4"; do
  i=$((i+1))
  env $v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$i -o run --output-format csv -- python3 tools/switch_bench.py > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 6; }
  python3 - $O/prof_$i/run_kernel_stats.csv "$v" <<'PY'
import csv, sys, re
out = []
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_(?:ingress_apply|egress_fixed))", r["Name"])
    if m:
        out.append("%s=%.1f" % (m.group(1), float(r["AverageNs"]) / 1e3))
print(sys.argv[2], " ".join(sorted(out)))
PY
done
