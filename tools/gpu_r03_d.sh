#!/bin/bash
# Round 3: the whole GPU suite, then the line-keeper rehearsal (rank 0 killed
# after the N=2 headline), then -- last, it may hang -- the torch-hosted
# symmetric IPC probe at 2600 MiB.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; exit $rc; }
INCCL_BENCH_SAME_DEVICE=1 INCCL_BENCH_TEST_DIE=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 3 \
    --no-sweep > $O/bench_die.out 2> $O/bench_die.err
rc=$?; echo "die rehearsal rc=$rc (expected non-zero)"; cut -c1-300 $O/bench_die.out
grep -q '"error"' $O/bench_die.out || { echo "no JSON line with error"; exit 1; }
[ $rc -ne 124 ] && [ $rc -ne 137 ] || exit $rc
timeout -k 10 120 python -u tools/probes/ipc_torch_probe.py 2600 > $O/ipc_torch_probe.log 2>&1
rc=$?; echo "ipc torch probe rc=$rc"; cat $O/ipc_torch_probe.log | grep -v amdgpu.ids
exit $rc
