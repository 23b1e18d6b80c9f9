#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
timeout -k 10 400 ./tools/tune/tune_stream > gpurun_out/tune_stream2.log 2>&1 || { echo tune failed; tail gpurun_out/tune_stream2.log; exit 5; }
cat gpurun_out/tune_stream2.log
