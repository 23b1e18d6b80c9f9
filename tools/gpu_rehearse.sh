#!/bin/bash
# The driver's N-rank bench command, rehearsed with all N ranks on ONE GPU:
# `python3 bench.py --gpus N --steps K --warmup W`, self-launched (no
# WORLD_SIZE), INCCL_BENCH_SAME_DEVICE=1.  Usage: gpu_rehearse.sh N [K] [W] [tag]
# Writes gpurun_out/rehearse_n<N><tag>.{json,log}; extra env (INCCL_BENCH_*) passes through.
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
N=${1:-2}; K=${2:-20}; W=${3:-5}; TAG=${4:-}
OUT=gpurun_out/rehearse_n${N}${TAG}
START=$(date +%s)
INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 560 python3 bench.py --gpus "$N" --steps "$K" --warmup "$W" \
  --json-out "$OUT.json" > "$OUT.line" 2> "$OUT.log"
rc=$?
echo "rehearse n=$N rc=$rc wall=$(( $(date +%s) - START ))s"
cat "$OUT.line"
[ $rc -eq 0 ] || tail -40 "$OUT.log"
exit $rc
