#!/bin/bash
# Round 3: switch dataplane with wide apply loads (tests incl. unaligned rows,
# bench, kernel trace, counters), the N=2 one-GPU rehearsal with the N>1
# host_e2e key, then -- last, it may hang -- the C IPC probe with SIBLING
# processes at 2600 MiB.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_switch.log 2>&1
rc=$?; echo "switch tests rc=$rc"; tail -2 $O/pytest_switch.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_switch.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/switch_bench.py > $O/switch_bench.log 2>&1 || { echo bench failed; tail -20 $O/switch_bench.log; exit 5; }
grep '"what"' $O/switch_bench.log | head -2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_switch -o run --output-format csv -- python3 tools/switch_bench.py > $O/prof_switch.log 2>&1 || { echo prof failed; tail -20 $O/prof_switch.log; exit 6; }
python3 - $O/prof_switch/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r["Name"].split("(")[1 if "namespace" in r["Name"] else 0][:40], r["Calls"], r["AverageNs"])
PY
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_switch -o pmc -- python3 tools/switch_bench.py > $O/pmc_switch.log 2>&1 || { echo "pmc switch failed"; exit 7; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_switch_$c -o pmc -- python3 tools/switch_bench.py > $O/pmc_switch_$c.log 2>&1 || { echo "pmc $c failed"; exit 7; }
done
echo "pmc ok"
INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 420 python -u bench.py --gpus 2 --steps 10 --warmup 3 \
    --json-out $O/bench_n2_same_device.json > $O/bench_n2.log 2>&1
rc=$?; echo "n2 rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench_n2.log; exit $rc; }
timeout -k 10 100 tools/probes/ipc_size_probe 0 2600 sib > $O/ipc_probe_c_sib_2600.log 2>&1
rc=$?; echo "C sibling probe 2600 rc=$rc"; cat $O/ipc_probe_c_sib_2600.log
exit $rc
