#!/bin/bash
# Round 3 GPU call: the self-launched N=2 rehearsal (both ranks on GPU 0), the
# watchdog rehearsal (rank 0 stuck after the headline), then the IPC probe.
# Stops at the first unexpected status.
set -u
O=gpurun_out/r03b
mkdir -p $O
INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 420 python -u bench.py --gpus 2 --steps 10 --warmup 3 \
    --json-out $O/bench_n2_same_device.json > $O/bench_n2.log 2>&1
rc=$?; echo "n2 rc=$rc"
[ $rc -eq 0 ] || exit $rc
INCCL_BENCH_SAME_DEVICE=1 INCCL_BENCH_TEST_HANG=1 INCCL_BENCH_BUDGET=75 timeout -k 10 200 python -u bench.py \
    --gpus 2 --steps 10 --warmup 3 > $O/bench_hang.out 2> $O/bench_hang.err
rc=$?; echo "hang rehearsal rc=$rc (expected non-zero, from the watchdog's 3)"
grep -q '"error"' $O/bench_hang.out || { echo "no JSON line with error"; exit 1; }
[ $rc -ne 124 ] && [ $rc -ne 137 ] || exit $rc
bash tools/probes/ipc_runtime_probe.sh $O/ipc_runtime_probe > $O/probe_stdout.txt 2>&1
rc=$?; echo "probe rc=$rc"; cat $O/ipc_runtime_probe/log.txt
exit $rc
