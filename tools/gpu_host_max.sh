#!/bin/bash
# Auto-scale max exchange of the IPC engines: shared-memory segment vs the TCP
# allgather (INCCL_HOST_MAX_TCP=1), two ranks on one GPU, p2p engine, 200 calls
# per size.  Writes gpurun_out/host_max.jsonl (rank 0's lines).
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
: > gpurun_out/host_max.jsonl
port=29611
for mib in 0.25 4; do
  for tcp in 0 1; do
    port=$((port + 7))
    for r in 0 1; do
      SCALE=auto INCCL_HOST_MAX_TCP=$tcp timeout -k 10 120 python tools/engine_rank.py $r 2 $port p2p $mib 200 > gpurun_out/host_max_r$r.log 2>&1 &
    done
    wait || exit 5
    grep -h '^{' gpurun_out/host_max_r0.log >> gpurun_out/host_max.jsonl || exit 6
  done
done
cat gpurun_out/host_max.jsonl
