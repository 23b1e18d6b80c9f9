#!/bin/bash
# 2-rank bench rehearsal on one GPU (engine auto + sweep) with a stack-dump watchdog.
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
INCCL_BENCH_WATCHDOG=60 INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 \
  --json-out gpurun_out/bench_n2_rehearsal.json 2>&1 | grep --line-buffered -v "ncclCommInitRank: invalid usage" > gpurun_out/bench_n2_rehearsal.log
rc=$?; echo "bench n2 rc=$rc"
tail -5 gpurun_out/bench_n2_rehearsal.log
exit $rc
