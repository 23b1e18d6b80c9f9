#!/bin/bash
# temporary: egress prefetch-depth variants, kernel times by rocprofv3
cd "$GRAFT_REPO_ROOT" || exit 3
export TMPDIR=/tmp
O=gpurun_out/expF; mkdir -p $O
stats() { python3 -c "import csv,sys; [print(r['Name'].replace('(anonymous namespace)::','')[:40], r['AverageNs']) for r in csv.DictReader(open(sys.argv[1])) if 'k_' in r['Name']]" "$(find $1 -name '*kernel_stats.csv' | head -1)"; }
INCCL_T_APPLY_SPLIT=1 INCCL_T_EGRESS_X=163 timeout -k 10 300 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_163.log 2>&1
echo "163 pytest rc=$?"; tail -2 $O/pytest_163.log
for x in 0 16 162 163 322 323 324; do
  INCCL_T_APPLY_SPLIT=1 INCCL_T_EGRESS_X=$x timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/x$x -o run --output-format csv -- python3 tools/switch_bench.py > $O/x$x.log 2>&1 || exit 1
  echo "x=$x"; stats $O/x$x | grep egress
done
