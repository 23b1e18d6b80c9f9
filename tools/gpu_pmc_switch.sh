#!/bin/bash
# Counters of the switch kernels over tools/switch_bench.py: SQ issue and wait
# cycles, instruction mix, LDS bank conflicts, and HBM traffic (FETCH_SIZE and
# WRITE_SIZE in passes of their own; gfx950: double FETCH_SIZE for wide
# streaming reads).  Usage: gpu_pmc_switch.sh [tag]; writes gpurun_out/pmcsw<tag>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/pmcsw${1:-}
mkdir -p $O
export TMPDIR=/tmp
run() {  # run <name> <counters...>
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o pmc -- python3 tools/switch_bench.py > $O/$n.log 2>&1 || { tail $O/$n.log; exit 7; }
}
run pmc1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
run pmc2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM
run pmc3 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD
run pmc4 FETCH_SIZE
run pmc5 WRITE_SIZE
python3 tools/pmc_summary.py $O/pmc*/pmc_counter_collection.csv | grep -v rocclr > $O/summary.txt
cat $O/summary.txt
