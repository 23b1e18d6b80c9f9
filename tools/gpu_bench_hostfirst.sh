cd $GRAFT_REPO_ROOT && timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --json-out gpurun_out/bench_hb.json > gpurun_out/bench_hb.log 2>&1 && python3 -c "
import json; d=json.load(open('gpurun_out/bench_hb.json')); print(d['host_e2e']); print(d['sizes']); print(d['roofline']['frac'], d['roofline_cold'])"
