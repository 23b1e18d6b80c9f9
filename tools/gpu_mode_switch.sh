#!/bin/bash
# tools/mode_switch_probe.py with W ranks on one GPU, REPEATS times.
# Usage: gpu_mode_switch.sh W LOG2 REPEATS
cd "$GRAFT_REPO_ROOT" || exit 3
W=$1; LG=$2; REP=$3
mkdir -p gpurun_out/mode_switch
for ((i = 0; i < REP; i++)); do
  PORT=$((30000 + RANDOM % 20000))
  pids=()
  for ((r = 0; r < W; r++)); do
    timeout -k 10 240 python3 tools/mode_switch_probe.py $r $PORT $W $LG \
      > gpurun_out/mode_switch/${W}_${LG}_${i}_r$r.log 2> gpurun_out/mode_switch/${W}_${LG}_${i}_r$r.err &
    pids+=($!)
  done
  rc=0
  for p in "${pids[@]}"; do wait $p || rc=$?; done
  echo "repeat $i rc=$rc"
  cat gpurun_out/mode_switch/${W}_${LG}_${i}_r*.log
  [ $rc -eq 0 ] || exit $rc
done
