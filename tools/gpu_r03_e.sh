#!/bin/bash
# Round 3: switch dataplane after the leader-wave ingress apply and the
# register-direct egress: GPU switch tests, the batch bench at 3 and 2 egress
# blocks per CU, a rocprofv3 kernel trace, and LDS / SQ counter passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/${OUTDIR:-r03e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_switch.log 2>&1
rc=$?; echo "switch tests rc=$rc"; tail -2 $O/pytest_switch.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_switch.log | head -20; exit $rc; }
for b in 3 2; do
  INCCL_EGRESS_BLOCKS_PER_CU=$b timeout -k 10 300 python -u tools/switch_bench.py > $O/switch_bench_b$b.log 2>&1 || { echo bench failed; tail -20 $O/switch_bench_b$b.log; exit 5; }
  echo "egress blocks/CU $b:"; grep '"what"' $O/switch_bench_b$b.log | head -2
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_switch -o run --output-format csv -- python3 tools/switch_bench.py > $O/prof_switch.log 2>&1 || { echo prof failed; tail -20 $O/prof_switch.log; exit 6; }
python3 - $O/prof_switch/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r["Name"].split("(")[1 if "namespace" in r["Name"] else 0][:40], r["Calls"], r["AverageNs"])
PY
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_switch -o pmc -- python3 tools/switch_bench.py > $O/pmc_switch.log 2>&1 || { echo "pmc switch failed"; tail $O/pmc_switch.log; exit 7; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/pmc_switch_lds -o pmc -- python3 tools/switch_bench.py > $O/pmc_switch_lds.log 2>&1 || { echo "pmc lds failed"; exit 7; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_switch_$c -o pmc -- python3 tools/switch_bench.py > $O/pmc_switch_$c.log 2>&1 || { echo "pmc $c failed"; exit 7; }
done
echo "pmc ok"
# last, since the large case may hang: the torch-hosted symmetric IPC probe,
# first at 256 MiB (sanity), then at 2600 MiB
timeout -k 10 100 python -u tools/probes/ipc_torch_probe.py 256 > $O/ipc_torch_probe_256.log 2>&1
rc=$?; echo "ipc torch probe 256 rc=$rc"; grep -v amdgpu.ids $O/ipc_torch_probe_256.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python -u tools/probes/ipc_torch_probe.py 2600 > $O/ipc_torch_probe_2600.log 2>&1
rc=$?; echo "ipc torch probe 2600 rc=$rc"; grep -v amdgpu.ids $O/ipc_torch_probe_2600.log | tail -8
exit $rc
