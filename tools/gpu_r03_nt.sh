#!/bin/bash
# Round 3: non-temporal loads/stores in the switch kernels, each variant twice:
# apply payload loads (INCCL_APPLY_NT bit 1) / aggregate stores (bit 2), ICRC frame
# loads (INCCL_ICRC_NT=1), egress aggregate load (INCCL_EGRESS_NT=2): temporary hooks of that experiment,
# removed after it; INCCL_APPLY_NT=0 and INCCL_EGRESS_NT=0 remain (plain stores).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03nt
mkdir -p $O
export TMPDIR=/tmp
i=0
for v in "X=0" "INCCL_APPLY_NT=1" "INCCL_APPLY_NT=2" "INCCL_APPLY_NT=3 INCCL_ICRC_NT=1 INCCL_EGRESS_NT=2" "INCCL_EGRESS_NT=0" \
         "X=0" "INCCL_APPLY_NT=1" "INCCL_APPLY_NT=2" "INCCL_APPLY_NT=3 INCCL_ICRC_NT=1 INCCL_EGRESS_NT=2" "INCCL_EGRESS_NT=0"; do
  i=$((i+1))
  env $v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$i -o run --output-format csv -- python3 tools/switch_bench.py > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 6; }
  python3 - $O/prof_$i/run_kernel_stats.csv "$v" <<'PY'
import csv, sys
out = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    for key in ("apply", "egress", "icrc_pair"):
        if key in n:
            out.append("%s=%.1f" % (key, float(r["AverageNs"]) / 1e3))
print(sys.argv[2], " ".join(sorted(out)))
PY
done
