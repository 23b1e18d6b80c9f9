#!/bin/bash
# tools/rs_sequence_probe.py with W ranks on one GPU, started from this shell
# (no launcher that forks after GPU init).  Usage: [EXTRA="--rccl --random"] gpu_rs_sequence.sh W [MIB] [tag]
cd "$GRAFT_REPO_ROOT" || exit 3
W=${1:-8}; MIB=${2:-256}; TAG=${3:-}; EXTRA=${EXTRA:-}
OUT=gpurun_out/rs_seq_${W}_${MIB}${TAG}
mkdir -p $OUT
PORT=$((30000 + RANDOM % 20000))
pids=()
for ((r = 0; r < W; r++)); do
  INCCL_TRACE=1 timeout -k 10 400 python3 tools/rs_sequence_probe.py $r $PORT $W $MIB $EXTRA > $OUT/rank$r.log 2> $OUT/rank$r.err &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
echo "rs sequence W=$W $MIB MiB rc=$rc"
grep -h '"bad_total"' $OUT/rank*.log
grep -h '"bad": \[[^]]*[1-9]' $OUT/rank*.log | head -20
grep -h '"error"' $OUT/rank*.log | head -5
exit $rc
