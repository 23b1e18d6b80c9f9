#!/bin/bash
# The fused stream kernel k_stream_vec at the sizes and R where it sits below its
# 256 MiB R = 2 figure: kernel time per case (tools/kernel_probe.py), then one
# rocprofv3 --pmc pass per counter group per case ($CASES: name:args ...;
# $PASSES: comma-separated counter groups, one pass each).
# Usage: gpu_pmc_stream.sh [tag]; writes gpurun_out/pmcst<tag>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/pmcst${1:-}
mkdir -p $O
export TMPDIR=/tmp
CASES=${CASES:-"hot256:--R 2 --mib 256 hot1g:--R 2 --mib 1024 cold256:--R 2 --mib 256 --sets 4 r8hot:--R 8 --mib 256 r8cold:--R 8 --mib 256 --sets 2"}
PASSES=${PASSES:-"FETCH_SIZE WRITE_SIZE TCP_UTCL1_TRANSLATION_MISS_sum,TCP_UTCL1_TRANSLATION_HIT_sum,TCP_UTCL1_REQUEST_sum,TCP_UTCL1_STALL_MULTI_MISS_sum TA_BUSY_avr,TA_ADDR_STALLED_BY_TC_CYCLES_sum,GRBM_UTCL2_BUSY,GRBM_GUI_ACTIVE TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum,TCC_TAG_STALL_sum,TCC_HIT_sum,TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum,TCP_TCC_READ_REQ_sum,TCP_PENDING_STALL_CYCLES_sum,TCP_TCP_TA_DATA_STALL_CYCLES_sum"}
timeout -s KILL 60 rocprofv3 -L > $O/counters_available.txt 2>&1 || true
python3 - "$CASES" > $O/cases.txt <<'PY'
import sys, re
items = re.findall(r'(\w+):((?:--\w[\w-]* \S+ ?)+)', sys.argv[1])
for n, a in items: print(n + "|" + a.strip())
PY
while IFS='|' read -r name args; do
  timeout -k 10 120 python3 tools/kernel_probe.py --kernel fused --iters 50 $args > $O/time_$name.json 2> $O/time_$name.err || { tail $O/time_$name.err; exit 5; }
  echo "$name $(cat $O/time_$name.json)"
  i=0
  for grp in $PASSES; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc ${grp//,/ } --output-format csv -d $O/${name}_p$i -o pmc -- python3 tools/kernel_probe.py --kernel fused --iters 5 $args > $O/${name}_p$i.log 2>&1 || { echo "pmc $name $grp failed"; tail -5 $O/${name}_p$i.log; exit 7; }
  done
  python3 tools/pmc_summary.py $O/${name}_p*/pmc_counter_collection.csv | grep k_stream > $O/summary_$name.txt
  cat $O/summary_$name.txt | cut -c1-600
done < $O/cases.txt
