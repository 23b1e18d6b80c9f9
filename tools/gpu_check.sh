#!/bin/bash
# Full GPU test suite -> switch dataplane bench + its rocprofv3 stats -> W = 8
# multi-process rehearsal of the IPC engines -> two-process bench over the mesh
# engines on ONE GPU.  Each GPU step has its own time limit; the script stops at
# the first abnormal exit.
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python tools/switch_bench.py > gpurun_out/switch_bench.log 2>&1 || { echo switch bench failed; tail -20 gpurun_out/switch_bench.log; exit 5; }
grep '^{' gpurun_out/switch_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profsw -o run --output-format csv -- python tools/switch_bench.py > gpurun_out/profsw.log 2>&1 || { echo prof failed; tail gpurun_out/profsw.log; exit 7; }
timeout -k 10 400 python -u tools/mp_engines.py 8 meshw p2p > gpurun_out/mp8.log 2>&1 || { echo mp8 failed; grep -v amdgpu.ids gpurun_out/mp8.log | tail -20; exit 8; }
grep world gpurun_out/mp8.log
for eng in mesh meshw; do
  INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 3 --engine $eng --no-sweep \
    --bucket-mib 256 --json-out gpurun_out/bench_n2_${eng}_256.json > gpurun_out/bench_n2_${eng}_256.log 2>&1
  rc=$?; echo "bench n2 $eng rc=$rc"; cut -c1-400 gpurun_out/bench_n2_${eng}_256.json 2>/dev/null
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/bench_n2_${eng}_256.log; exit $rc; fi
done
echo done
