#!/bin/bash
# Kernel-level profile of an N = 2 engine step on ONE GPU: two rank processes,
# each under its own rocprofv3 --kernel-trace --stats (started from this shell,
# no launcher that forks after GPU init).  Usage: gpu_engine_profile.sh ENGINE [MIB]
cd "$GRAFT_REPO_ROOT" || exit 3
export TMPDIR=/tmp
ENGINE=${1:-p2p}
MIB=${2:-256}
OUT=gpurun_out/engprof_${ENGINE}_${MIB}
mkdir -p $OUT
PORT=$((30000 + RANDOM % 20000))
pids=()
for r in 0 1; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r$r -o run -- \
    python3 tools/engine_rank.py $r 2 $PORT $ENGINE $MIB 20 > $OUT/rank$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
echo "engine $ENGINE $MIB MiB rc=$rc"
grep -h '"rank"' $OUT/rank*.log
exit $rc
