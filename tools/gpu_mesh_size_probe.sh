#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
for eng in mesh meshw; do
  INCCL_TRACE=1 timeout -k 10 90 python -u tools/mesh_size_probe.py $eng ${SIZES:-256 1024} > gpurun_out/mesh_probe_$eng.log 2>&1
  rc=$?; echo "$eng rc=$rc"; grep -v amdgpu.ids gpurun_out/mesh_probe_$eng.log | grep -v "^\[inccl" | tail -12
  [ $rc -eq 0 ] || exit $rc
done
