#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
for i in $(seq 1 ${RUNS:-20}); do
echo "== run $i" >> gpurun_out/sweep_check.log
INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 100 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 tools/sweep_oracle_check.py 2>&1 | grep -E "^rank|^\[inccl ll" | grep -v "failed: inccl_allreduce_f32 failed (rc=-3)" >> gpurun_out/sweep_check.log
done
grep -v " 0 wrong" gpurun_out/sweep_check.log | grep -v "^=="
rocm-smi --showserial 2>/dev/null | grep -i serial | head -2
