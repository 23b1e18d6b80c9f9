#!/bin/bash
# tools/mesh_stress_probe.py with W ranks on one GPU, once per mode listed.
# Usage: gpu_mesh_stress.sh W CALLS "MODES" LOG2 [LOG2 ...]
cd "$GRAFT_REPO_ROOT" || exit 3
W=$1; CALLS=$2; MODES=$3; shift 3
mkdir -p gpurun_out/mesh_stress
for m in $MODES; do
  PORT=$((30000 + RANDOM % 20000))
  pids=()
  for ((r = 0; r < W; r++)); do
    timeout -k 10 240 python3 tools/mesh_stress_probe.py $r $PORT $W $m $CALLS "$@" \
      > gpurun_out/mesh_stress/${W}_${m}_r$r.log 2> gpurun_out/mesh_stress/${W}_${m}_r$r.err &
    pids+=($!)
  done
  rc=0
  for p in "${pids[@]}"; do wait $p || rc=$?; done
  echo "mode $m rc=$rc"
  cat gpurun_out/mesh_stress/${W}_${m}_r*.log
  [ $rc -eq 0 ] || exit $rc
done
