#!/bin/bash
# mesh engine on ONE GPU: its GPU tests (multi-process, world-1, peer timeout),
# then two-process bench.py runs over the mesh engine (INCCL_BENCH_SAME_DEVICE=1)
# at 64 and 256 MiB, the second with the N>1 size sweep.
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  -k "mesh or world1 or timeout" > gpurun_out/pytest_mesh.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_mesh.log | tail -20
if [ $rc -ne 0 ]; then tail -60 gpurun_out/pytest_mesh.log; exit $rc; fi
for mib in 64 256; do
  extra="--no-sweep"; [ $mib = 256 ] && extra=""
  INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --engine mesh $extra \
    --bucket-mib $mib --json-out gpurun_out/bench_n2_mesh_$mib.json > gpurun_out/bench_n2_mesh_$mib.log 2>&1
  rc=$?; echo "bench n2 mesh ${mib}MiB rc=$rc"; cat gpurun_out/bench_n2_mesh_$mib.json 2>/dev/null
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/bench_n2_mesh_$mib.log; exit $rc; fi
done
