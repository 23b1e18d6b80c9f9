#!/bin/bash
# GPU test suite only (optionally a -k filter as $1)
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
if [ -n "$1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x -k "$1" > gpurun_out/pytest_gpu.log 2>&1
else
  timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
fi
rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
exit $rc
