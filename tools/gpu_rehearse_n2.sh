#!/bin/bash
# Two-process bench.py on ONE GPU over the p2p engine (RCCL refuses two ranks on
# one GPU): rehearses the N>1 launch, bootstrap, IPC mapping, barriers and timing.
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
for mib in 64 256; do
  INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --engine p2p \
    --bucket-mib $mib --json-out gpurun_out/bench_n2_rehearsal_$mib.json > gpurun_out/bench_n2_rehearsal_$mib.log 2>&1
  rc=$?; echo "bench n2 ${mib}MiB rc=$rc"; cat gpurun_out/bench_n2_rehearsal_$mib.json 2>/dev/null
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_n2_rehearsal_$mib.log; exit $rc; fi
done
