#!/bin/bash
# Round 3: whole GPU suite with durations on the final tree, then the 4-rank
# self-launched bench rehearsal (two-phase headline, sweep) on one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=25 > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -32 $O/pytest_gpu.log | grep -E "passed|s call|s setup" | head -30
[ $rc -eq 0 ] || exit $rc
INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 500 python -u bench.py --gpus 4 --steps 10 --warmup 3 --json-out $O/bench_n4.json > $O/bench_n4.log 2>&1
rc=$?; echo "bench n4 rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench_n4.log; exit $rc; }
python3 - $O/bench_n4.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("n", d["n_gpus"], "value", d["value"], "engine", d["config"]["engine"], "parity", d["parity_vs_oracle"]["mismatches"],
      "verified", d.get("verified_vs_reference_engine"), "elapsed", d.get("elapsed_s"))
print("candidates", d.get("headline_candidates"))
rows = [r for r in d.get("sweep", []) if r.get("ok")]
print("sweep rows ok", len(rows), "mismatches", sum((r.get("parity_vs_oracle") or {}).get("mismatches") or 0 for r in rows))
PY
