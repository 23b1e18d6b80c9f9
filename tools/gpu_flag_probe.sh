#!/bin/bash
# tools/flag_probe.hip (built in-tree beforehand: tools/bin/flag_probe) over the
# three memory kinds, a writer on another XCD and on the same XCD, then the two-
# process IPC form.  Usage: gpu_flag_probe.sh TRIALS LIMIT_US DELAY_US
cd "$GRAFT_REPO_ROOT" || exit 3
T=${1:-2000}; L=${2:-1000}; D=${3:-2}
B=tools/bin/flag_probe
for mem in uncached finegrained coarse; do
  for wb in 1 8; do
    timeout -k 5 60 $B $mem $T $L $D $wb || exit $?
  done
done
F=$(mktemp -u /tmp/flagprobe.XXXXXX)
timeout -k 5 90 $B ipc-owner $F $T $L $D & p1=$!
timeout -k 5 90 $B ipc-peer $F $T $L $D & p2=$!
rc=0
wait $p1 || rc=$?
wait $p2 || rc=$?
rm -f $F
exit $rc
