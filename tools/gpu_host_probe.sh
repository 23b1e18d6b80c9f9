#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
for cs in default recreate priority; do
  for pre in allocfirst none; do
    echo "copy streams: $cs"
    INCCL_COPY_STREAMS=$cs PRE=$pre VARIANTS=lib,lib,copies timeout -k 10 120 python -u tools/host_pipe_probe.py 2>&1 | grep -v amdgpu | tee -a gpurun_out/host_probe5.jsonl
  done
done
