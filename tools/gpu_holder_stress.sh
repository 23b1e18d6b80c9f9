#!/bin/bash
# tools/gpu_mesh_stress.sh twice: alone, then beside a fifth process that holds a
# GPU context with four streams (as the pytest process that spawns the one-GPU
# multi-process tests does).  Usage: gpu_holder_stress.sh W CALLS "MODES" LOG2
cd "$GRAFT_REPO_ROOT" || exit 3
W=$1; CALLS=$2; MODES=$3; LG=$4
echo "== alone"
bash tools/gpu_mesh_stress.sh $W $CALLS "$MODES" $LG || exit $?
mkdir -p gpurun_out/holder
for m in $MODES; do cp gpurun_out/mesh_stress/${W}_${m}_r0.log gpurun_out/holder/alone_${m}_r0.log; done
timeout -k 5 600 python3 -c '
import time, torch
ss = [torch.cuda.Stream() for _ in range(4)]
xs = []
for s in ss:
    with torch.cuda.stream(s):
        xs.append(torch.ones(1 << 20, device="cuda") * 2)
torch.cuda.synchronize()
print("holder ready", flush=True)
time.sleep(590)
' > gpurun_out/holder/holder.log 2>&1 &
H=$!
for i in $(seq 60); do grep -q "holder ready" gpurun_out/holder/holder.log 2>/dev/null && break; sleep 2; done
echo "== beside a holder"
bash tools/gpu_mesh_stress.sh $W $CALLS "$MODES" $LG; rc=$?
kill $H; wait $H
exit $rc
