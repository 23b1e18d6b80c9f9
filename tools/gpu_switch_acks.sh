#!/bin/bash
# Kernel stats of the switch batch without and with reflected ACKs
# (tools/switch_ack_probe.py).  Writes gpurun_out/swacks<tag>/.
cd "$GRAFT_REPO_ROOT" || exit 3
export TMPDIR=/tmp
O=gpurun_out/swacks${1:-}
mkdir -p $O
for a in 0 1; do
  SW_ACKS=$a timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_acks$a -o run --output-format csv -- python3 tools/switch_ack_probe.py \
    > $O/acks$a.jsonl 2> $O/acks$a.err || { tail $O/acks$a.err; exit 4; }
  cat $O/acks$a.jsonl
  f=$(find $O/prof_acks$a -name "*kernel_stats.csv" | head -1)
  cp "$f" $O/kernel_stats_acks$a.csv && cut -d, -f1-4,6 $O/kernel_stats_acks$a.csv | grep -E "k_|Name" | cut -c1-160
done
