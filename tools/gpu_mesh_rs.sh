#!/bin/bash
# Round 6: the mesh engines' reduce-scatter route on the configurations that
# failed in round 5 (profiles/r05/mesh_rs_investigation), once, on the rebuilt
# kernel.  W rank processes on one GPU, each under its own rocprofv3
# --kernel-trace --stats (started from this shell, so no process forks after
# the profiler initialised the GPU).  Usage: gpu_mesh_rs.sh W ENGINE LOG2 [LOG2 ...]
cd "$GRAFT_REPO_ROOT" || exit 3
export TMPDIR=/tmp
W=$1; ENGINE=$2; shift 2
OUT=gpurun_out/mesh_rs_${W}_${ENGINE}_$(echo "$@" | tr ' ' _)
mkdir -p $OUT
PORT=$((30000 + RANDOM % 20000))
pids=()
for ((r = 0; r < W; r++)); do
  INCCL_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r$r -o run -- \
    python3 tools/mesh_rs_probe.py --rank $r $PORT $W $ENGINE "$@" > $OUT/rank$r.log 2> $OUT/rank$r.err &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
echo "mesh rs W=$W $ENGINE $* rc=$rc"
grep -h '"rank"' $OUT/rank*.log
exit $rc
