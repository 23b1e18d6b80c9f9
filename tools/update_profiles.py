"""Copy a GPU evidence pass (tools/gpu_round_profile.sh, plus a smoke.log if one
was written) from gpurun_out/ into profiles/rNN/round_profile/ (tracked): bench
JSON, rocprofv3 kernel stats, PMC counter CSVs, the GPU test log, the 2-rank
rehearsal line; and rebuild the per-launch HBM traffic summary
profiles/pmc_traffic.json that bench.py reads.

    python tools/update_profiles.py --round 4 [--src gpurun_out]

Traffic correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide coalesced streaming
read, so hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import argparse
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# probe kind -> (traffic key's kernel name, substring of the mangled name, bytes per element)
KERNELS = {"fused": ("k_stream_vec<F32,F32,R>", "k_stream_vec", 4), "quant_sum": ("k_stream_vec<F32,Q32,R>", "k_stream_vec", 4),
           "bf16": ("k_stream16<BF16,BF16,R>", "k_stream16", 2), "f16": ("k_stream16<F16,F16,R>", "k_stream16", 2)}


def mean_counter(path, needle):
    rows = [r for r in csv.DictReader(open(path)) if needle in r["Kernel_Name"]]
    vals = [float(r["Counter_Value"]) for r in rows]
    return sum(vals) / len(vals), len(vals)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--round", type=int, required=True)
    p.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    p.add_argument("--mib", type=int, default=256)
    p.add_argument("--R", type=int, default=2)
    a = p.parse_args()
    prof = os.path.join(ROOT, "profiles")
    dest = os.path.join(prof, f"r{a.round:02d}", "round_profile")
    os.makedirs(dest, exist_ok=True)
    src = a.src
    for name, out in (("bench.json", "bench.json"), (os.path.join("prof", "run_kernel_stats.csv"), "bench_kernel_stats.csv"),
                      ("bench_profiled.json", "bench_profiled.json"),
                      (os.path.join("prof_bf16", "run_kernel_stats.csv"), "bf16_kernel_stats.csv"),
                      # the rotated-set (cold) run: k_stream_vec's average here reproduces frac_cold
                      (os.path.join("prof_cold", "run_kernel_stats.csv"), "cold_kernel_stats.csv"),
                      ("prof_cold.log", "cold_probe.log"),
                      ("pytest_gpu.log", "pytest_gpu.log"), ("rehearse_n2.json", "rehearse_n2.json"), ("smoke.log", "smoke.log")):
        if os.path.exists(os.path.join(src, name)):
            shutil.copy(os.path.join(src, name), os.path.join(dest, out))
    traffic_path = os.path.join(prof, "pmc_traffic.json")
    traffic = json.load(open(traffic_path)) if os.path.exists(traffic_path) else {}
    for k, (kname, needle, esize) in KERNELS.items():
        n = a.mib * (1 << 20) // esize
        f_csv = os.path.join(src, f"pmc_{k}_FETCH_SIZE", "pmc_counter_collection.csv")
        w_csv = os.path.join(src, f"pmc_{k}_WRITE_SIZE", "pmc_counter_collection.csv")
        if not (os.path.exists(f_csv) and os.path.exists(w_csv)):
            continue
        f, nf = mean_counter(f_csv, needle)
        w, nw = mean_counter(w_csv, needle)
        shutil.copy(f_csv, os.path.join(dest, f"pmc_{k}_FETCH_SIZE.csv"))
        shutil.copy(w_csv, os.path.join(dest, f"pmc_{k}_WRITE_SIZE.csv"))
        alg = (a.R + 1) * esize * n
        hbm = (2 * f + w) * 1024
        traffic[f"{kname} R={a.R} n={n}"] = {
            "hbm_bytes_per_launch": int(round(hbm)), "fetch_size_kib_raw": f, "write_size_kib": w,
            "launches_averaged": [nf, nw],
            "correction": "gfx950: FETCH_SIZE counts half the bytes of a wide coalesced stream -> x2 "
                          "(MI355X_MICROARCH.md HBM); units KiB",
            "alg_bytes_per_launch": alg, "ratio_to_alg": round(hbm / alg, 5),
            "command": f"rocprofv3 --pmc <FETCH_SIZE|WRITE_SIZE> --output-format csv -- python tools/kernel_probe.py "
                       f"--kernel {k} --R {a.R} --mib {a.mib} --iters 5",
            "round": a.round}
    json.dump(traffic, open(traffic_path, "w"), indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
