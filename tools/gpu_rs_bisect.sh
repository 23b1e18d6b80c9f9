#!/bin/bash
# Which part of the N = 8 bench run precedes the p2p reduce-scatter row's first
# call going wrong (profiles/r06/rehearse_n8): the bench with every rank on one
# GPU, (A) without the size sweep (INCCL_BENCH_SWEEP_ENGINES=none), (B) without
# the sweep and with the p2p engine only.  Each prints its reduce_scatter rows.
cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
py='import json,sys
d=json.load(open(sys.argv[1]))
for r in d.get("reduce_scatter") or []:
    print(json.dumps({k: r.get(k) for k in ("engine", "bucket_mib", "ok", "bit_identical", "parity_vs_oracle", "parity_vs_oracle_call3")}))'
INCCL_BENCH_SWEEP_ENGINES=none INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 400 python3 bench.py --gpus 8 --steps 5 --warmup 2 \
  --json-out gpurun_out/bisect_A.json > gpurun_out/bisect_A.line 2> gpurun_out/bisect_A.log || exit 5
echo "A (no sweep)"; python3 -c "$py" gpurun_out/bisect_A.json
INCCL_BENCH_SWEEP_ENGINES=none INCCL_BENCH_SAME_DEVICE=1 timeout -k 10 400 python3 bench.py --gpus 8 --steps 5 --warmup 2 --engine p2p \
  --json-out gpurun_out/bisect_B.json > gpurun_out/bisect_B.line 2> gpurun_out/bisect_B.log || exit 6
echo "B (no sweep, p2p only)"; python3 -c "$py" gpurun_out/bisect_B.json
