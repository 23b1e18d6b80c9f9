#!/bin/bash
# N-rank bench rehearsal on ONE GPU (engine auto + sweep) with a stack-dump
# watchdog.  Usage: gpu_rehearse_n2_sweep.sh [N=2] (N <= 4 here; the N = 8 case
# is the driver's, on a whole node).
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
N=${1:-2}
[ "$N" -le 4 ] || { echo "N=$N: rehearse at most 4 ranks"; exit 2; }
INCCL_BENCH_WATCHDOG=60 INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $N --steps 10 --warmup 3 \
  --json-out gpurun_out/bench_n${N}_rehearsal.json 2>&1 | grep --line-buffered -v "ncclCommInitRank: invalid usage" > gpurun_out/bench_n${N}_rehearsal.log
rc=$?; echo "bench n$N rc=$rc"
tail -5 gpurun_out/bench_n${N}_rehearsal.log
exit $rc
