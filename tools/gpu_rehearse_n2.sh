#!/bin/bash
# full GPU suite (incl. multi-process p2p) -> N=2 bench rehearsal on one GPU (p2p engine)
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --engine p2p --bucket-mib 64 > gpurun_out/bench_n2_rehearsal.log 2>&1
rc=$?; echo "bench n2 rc=$rc"; tail -5 gpurun_out/bench_n2_rehearsal.log
