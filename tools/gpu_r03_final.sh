#!/bin/bash
# Round 3 final tree: smoke() and the default bench line (N = 1), as the driver runs them.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 5; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 6; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("value", d["value"], d["unit"], "ms", d["ms_per_step"], "frac", r["frac"], "frac_cold", r.get("frac_cold"), "traffic", r.get("traffic"),
      "cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["unit"])
PY
