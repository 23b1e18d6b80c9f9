#!/bin/bash
# Round 3 (re-entry): the whole GPU suite, smoke() and the default bench on the
# restored tree, before any further change.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 4; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py --json-out $O/bench.json > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 5; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('value',d['value'],'frac',r['frac'],'cold',r.get('frac_cold'),'parity',d['parity_vs_oracle'])"
