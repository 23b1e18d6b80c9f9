#!/bin/bash
# GPU switch dataplane: tests, the batch benchmark, and its rocprofv3 kernel
# stats.  Usage: gpu_switch.sh [tag] [pytest -k filter]; env passes through.
# Writes gpurun_out/switch<tag>/.
cd "$GRAFT_REPO_ROOT" || exit 3
export TMPDIR=/tmp
OUT=gpurun_out/switch${1:-}
mkdir -p "$OUT"
K=${2:+-k "$2"}
timeout -k 10 400 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -v --timeout 200 --timeout-method thread $K \
  > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" "$OUT/pytest.log" | tail -5
[ $rc -eq 0 ] || { grep -E "FAIL|assert|Error" "$OUT/pytest.log" | head -30; exit $rc; }
timeout -k 10 300 python -u tools/switch_bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.jsonl"
[ $rc -eq 0 ] || { tail -20 "$OUT/bench.err"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 tools/switch_bench.py \
  > "$OUT/bench_prof.jsonl" 2> "$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv" && cut -d, -f1-8 "$OUT/kernel_stats.csv" | head -14
exit $rc
