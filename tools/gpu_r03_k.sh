#!/bin/bash
# Round 3: the apply frames-per-wave sweep (1, 2) with tests, then the IPC
# engines on a 2.25 GiB bucket in C processes (/opt/rocm's HSA runtime) --
# last, since it may hang if the HSA finding were wrong.
set -u
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03k
mkdir -p $O
for k in 1 2; do
  INCCL_APPLY_FRAMES=$k timeout -k 10 200 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -q --timeout 200 --timeout-method thread -k "batches or serial" > $O/pytest_switch_apply$k.log 2>&1
  rc=$?; echo "switch tests apply frames $k rc=$rc"; tail -1 $O/pytest_switch_apply$k.log; [ $rc -eq 0 ] || exit $rc
  INCCL_APPLY_FRAMES=$k timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_apply$k -o run --output-format csv -- python3 tools/switch_bench.py > $O/prof_apply$k.log 2>&1 || exit 6
  python3 - $O/prof_apply$k/run_kernel_stats.csv $k <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "namespace" in r["Name"]:
        print("apply_frames", sys.argv[2], r["Name"].split("::")[1].split("(")[0][:30], r["Calls"], r["AverageNs"])
PY
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_comm.py -m gpu -x -v --timeout 300 --timeout-method thread -k over_2gib > $O/pytest_big_ipc.log 2>&1
rc=$?; echo "big IPC C-hosted rc=$rc"; grep -E "PASS|FAIL|passed|failed|rank" $O/pytest_big_ipc.log | tail -12
exit $rc
