#!/bin/bash
# Round-2 check pass: GPU suite -> bench N=1 (all keys) -> 2-rank bench rehearsal on one GPU.
# Every GPU step has its own time limit; the script stops at the first abnormal exit.
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -5
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 600 python -u bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench_n1.json > gpurun_out/bench_n1.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_n1.log; exit 5; }
cat gpurun_out/bench_n1.json
INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 \
  --json-out gpurun_out/bench_n2_rehearsal.json > gpurun_out/bench_n2_rehearsal.log 2>&1
rc=$?; echo "bench n2 rc=$rc"
if [ $rc -ne 0 ]; then tail -30 gpurun_out/bench_n2_rehearsal.log; exit $rc; fi
head -c 3000 gpurun_out/bench_n2_rehearsal.json
echo done
