#!/bin/bash
# Counters of the switch kernels over tools/switch_bench.py, one rocprofv3 pass
# per counter group.  Usage: gpu_pmc_switch.sh [tag] [passes file]; a passes
# file (lines "name|counters ...", e.g. tools/pmc_passes/switch_mem.txt: the
# memory path) replaces the default groups: SQ issue and wait cycles,
# instruction mix, LDS bank conflicts, HBM traffic (FETCH_SIZE and WRITE_SIZE in
# passes of their own; gfx950: double FETCH_SIZE for wide streaming reads).
# Writes gpurun_out/pmcsw<tag>/ and its summary.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/pmcsw${1:-}
mkdir -p $O
export TMPDIR=/tmp
DEFAULT="pmc1|SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
pmc2|SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM
pmc3|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD
pmc4|FETCH_SIZE
pmc5|WRITE_SIZE"
while IFS='|' read -r n counters; do
  [ -n "$n" ] || continue
  timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d $O/$n -o pmc -- python3 tools/switch_bench.py > $O/$n.log 2>&1 || { tail $O/$n.log; exit 7; }
done <<< "$([ -n "$2" ] && cat "$2" || echo "$DEFAULT")"
python3 tools/pmc_summary.py $O/pmc*/pmc_counter_collection.csv | grep -v rocclr > $O/summary.txt
cat $O/summary.txt
