#!/bin/bash
# Round 3: SQ counters of the fused switch kernel beside the separate passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03q
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  --output-format csv -d $O/pmc1 -o pmc -- python3 tools/switch_bench.py > $O/pmc1.log 2>&1 || { tail $O/pmc1.log; exit 7; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD \
  --output-format csv -d $O/pmc2 -o pmc -- python3 tools/switch_bench.py > $O/pmc2.log 2>&1 || { tail $O/pmc2.log; exit 7; }
python3 tools/pmc_summary.py $O/pmc1/pmc_counter_collection.csv $O/pmc2/pmc_counter_collection.csv | grep -v rocclr
