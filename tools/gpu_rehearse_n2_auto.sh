#!/bin/bash
# Two-process bench.py on ONE GPU with the driver's flags (engine auto): RCCL
# drops out (ranks share a GPU), the IPC engines are tuned, the sweep runs.
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 \
  --json-out gpurun_out/bench_n2_auto.json > gpurun_out/bench_n2_auto.log 2>&1
rc=$?; echo "bench n2 auto rc=$rc"
if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_n2_auto.log; exit $rc; fi
python - <<'P'
import json
d = json.load(open("gpurun_out/bench_n2_auto.json"))
print(d["value"], d["ms_per_step"], d["config"]["engine"])
print([(t["engine"], t["ok"], t["ms"]) for t in d["config"]["engine_tuning"]])
sw = d.get("sweep") or []
print(len(sw), "sweep rows; bit-identical:", all(r["bit_identical"] for r in sw if r["ok"]))
P
