#!/bin/bash
# Per-call overhead of small eager calls: Python layers,
# C, and a rocprofv3 HIP API + kernel trace of each.  Writes gpurun_out/calls<tag>/.
cd "$GRAFT_REPO_ROOT" || exit 3
export TMPDIR=/tmp
O=gpurun_out/calls${1:-}
mkdir -p $O
timeout -k 10 120 python3 -u tools/call_overhead.py > $O/python.jsonl 2> $O/python.err || { tail $O/python.err; exit 4; }
cat $O/python.jsonl
timeout -k 10 60 ./tools/call_overhead > $O/c.jsonl 2> $O/c.err || { tail $O/c.err; exit 5; }
cat $O/c.jsonl
timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --stats -d $O/prof_c -o run --output-format csv -- ./tools/call_overhead 2000 \
  > $O/c_prof.jsonl 2> $O/c_prof.err || { tail $O/c_prof.err; exit 6; }
ITERS=1000 timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --stats -d $O/prof_py -o run --output-format csv -- python3 tools/call_overhead.py \
  > $O/py_prof.jsonl 2> $O/py_prof.err || { tail $O/py_prof.err; exit 7; }
for d in prof_c prof_py; do
  for f in $(find $O/$d -name "*_stats.csv"); do echo "== $f"; cut -d, -f1-4 $f | head -12; done
done
