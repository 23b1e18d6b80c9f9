#!/bin/bash
# Four-process bench.py on ONE GPU with --engine auto: the N=4 launch, bootstrap,
# engine selection (rccl / ar / a2a are refused on a shared GPU and must drop
# out cleanly), IPC mapping for W = 4, the p2p / mesh / ll engines and the sweep.
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 10 --warmup 3 --engine auto \
  --bucket-mib 256 --json-out gpurun_out/bench_n4_rehearsal_256.json > gpurun_out/bench_n4_rehearsal_256.log 2>&1
rc=$?; echo "bench n4 256MiB rc=$rc"; cat gpurun_out/bench_n4_rehearsal_256.json 2>/dev/null
if [ $rc -ne 0 ]; then tail -40 gpurun_out/bench_n4_rehearsal_256.log; exit $rc; fi
