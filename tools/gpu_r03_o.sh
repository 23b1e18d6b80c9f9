#!/bin/bash
# Round 3: the two-phase N > 1 headline (bench.py) rehearsed on one GPU.
#  a) phase 1 = p2p (INCCL_BENCH_SAFE_ENGINES; RCCL refuses two ranks on one
#     GPU), phase 2 = the rest: one line, headline_candidates listed
#  b) the same with rank 0 SIGKILLed at the start of phase 2: the line keeper
#     prints the phase-1 headline with the stage, non-zero exit
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03o
mkdir -p $O
export TMPDIR=/tmp
INCCL_BENCH_SAME_DEVICE=1 INCCL_BENCH_SAFE_ENGINES=p2p timeout -k 10 400 python -u bench.py --gpus 2 --steps 10 \
  --warmup 3 --no-sweep --json-out $O/two_phase_n2.json > $O/two_phase_n2.log 2>&1
rc=$?; echo "two-phase rc=$rc"; [ $rc -eq 0 ] || { tail -30 $O/two_phase_n2.log; exit $rc; }
python3 - $O/two_phase_n2.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value", d["value"], "engine", d["config"]["engine"], "parity", d["parity_vs_oracle"]["mismatches"],
      "verified", d.get("verified_vs_reference_engine"))
for c in d.get("headline_candidates", []):
    print("  candidate", c)
for t in d["config"]["engine_tuning"]:
    print("  tune", t["phase"], t["engine"], t["env"], t["verified"], t["ms"])
PY
INCCL_BENCH_SAME_DEVICE=1 INCCL_BENCH_SAFE_ENGINES=p2p INCCL_BENCH_TEST_DIE=phase2 timeout -k 10 300 python -u bench.py \
  --gpus 2 --steps 10 --warmup 3 --no-sweep > $O/die_phase2_n2.json 2> $O/die_phase2_n2.stderr.txt
rc=$?; echo "die-in-phase-2 rc=$rc (non-zero expected)"
grep -c '"metric"' $O/die_phase2_n2.json
python3 -c "import json;d=json.loads(open('$O/die_phase2_n2.json').read().strip().splitlines()[-1]);print('kept value',d['value'],'engine',d['config']['engine'],'error',d['error'])"
