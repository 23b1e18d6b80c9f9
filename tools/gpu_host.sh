#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "allreduce_write or host or edges or comm" > gpurun_out/pytest_host.log 2>&1 || { echo tests failed; tail -30 gpurun_out/pytest_host.log; exit 4; }
tail -2 gpurun_out/pytest_host.log
timeout -k 10 600 python tools/host_bench.py > gpurun_out/host_bench.log 2>&1 || { echo host_bench failed; tail -20 gpurun_out/host_bench.log; exit 5; }
cat gpurun_out/host_bench.log
