#!/bin/bash
# The switch batch at other fan-ins (P = the largest power of two with
# fan_in x P <= 131 072 ingress frames: the bench's batches alternate between
# the two halves of a 2P-slot ring, which needs P to be a power of two):
# switch_bench.py under rocprofv3 kernel stats per fan-in.  Usage:
# gpu_switch_fans.sh [tag] [fan-ins...]; writes gpurun_out/fans<tag>/.
cd "$GRAFT_REPO_ROOT" || exit 3
export TMPDIR=/tmp
O=gpurun_out/fans${1:-}; mkdir -p $O; shift
for f in ${@:-2 3 4 5 8 16}; do
  P=1; while [ $(( P * 2 * f )) -le 131072 ]; do P=$(( P * 2 )); done
  SW_FAN_IN=$f SW_PSNS=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/f$f -o run --output-format csv -- python3 tools/switch_bench.py > $O/f$f.jsonl 2> $O/f$f.err || { tail -20 $O/f$f.err; exit 1; }
  echo "fan_in=$f psns=$P"
  python3 -c "import csv,sys; [print('  ', r['Name'].replace('(anonymous namespace)::','')[:40], r['AverageNs']) for r in csv.DictReader(open(sys.argv[1])) if 'k_' in r['Name'] and 'icrc' not in r['Name']]" "$(find $O/f$f -name '*kernel_stats.csv' | head -1)"
  grep eager $O/f$f.jsonl | python3 -c "import sys,json; [print('  ', json.loads(l)['mode'], json.loads(l)['ms']) for l in sys.stdin]"
done
