#!/bin/bash
# Round 3: the switch dataplane after the egress rewrite -- its GPU tests, the
# batch benchmark, a rocprofv3 kernel-trace of every switch kernel (claim /
# apply / commit / egress / recycle / icrc), a PMC pass on k_egress (LDS and
# wait counters), then (last, since it may hang) the >2 GiB IPC engine probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_switch.log 2>&1
rc=$?; echo "switch tests rc=$rc"; tail -3 $O/pytest_switch.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_switch.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/switch_bench.py > $O/switch_bench.log 2>&1 || { echo bench failed; tail -20 $O/switch_bench.log; exit 5; }
grep -v amdgpu.ids $O/switch_bench.log | tail -4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_switch -o run --output-format csv -- python3 tools/switch_bench.py > $O/prof_switch.log 2>&1 || { echo prof failed; tail -20 $O/prof_switch.log; exit 6; }
find $O/prof_switch -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -c1-160 {}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_switch -o pmc -- python3 tools/switch_bench.py > $O/pmc_switch.log 2>&1 || { echo "pmc switch failed"; tail $O/pmc_switch.log; exit 7; }
echo "pmc ok"
# LDS-specific counters (names as in the gfx9 SQ block; a refused name only
# fails this pass)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/pmc_switch_lds -o pmc -- python3 tools/switch_bench.py > $O/pmc_switch_lds.log 2>&1
echo "pmc lds rc=$?"
timeout -k 10 180 python -u tools/ipc_big_engine_probe.py p2p 2304 > $O/ipc_big_p2p.log 2>&1
rc=$?; echo "ipc big p2p rc=$rc"; tail -4 $O/ipc_big_p2p.log
exit $rc
