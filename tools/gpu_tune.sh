#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
TUNE_POLICY=1 timeout -k 10 300 ./tools/tune/tune_stream > gpurun_out/tune_policy.log 2>&1 || { echo tune failed; tail gpurun_out/tune_policy.log; exit 5; }
cat gpurun_out/tune_policy.log
