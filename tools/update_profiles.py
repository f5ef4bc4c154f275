"""Copy a tools/gpu_profile.sh run (gpurun_out/<tag>/) into profiles/ under a round prefix, write a
per-kernel summary (<prefix>_kernels.json: average duration from the kernel trace, FETCH_SIZE and
WRITE_SIZE bytes per dispatch from the separate --pmc passes) and regenerate profiles/pmc_traffic.json
(the HBM bytes per validate launch that bench.py reports as roofline.traffic).
Usage: python tools/update_profiles.py <tag> <prefix>, e.g. r2prof r2."""
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
from pmc_summary import summarise  # noqa: E402

BENCH_KERNEL = "fixed_kernel<6, false"
# kernels of tools/bench_configs.py --only varlen,shard,seal,parse (name substrings)
CFG_KERNELS = {
    "varlen (config 3): 8-lane sorted-runs kernel (runs sorted in the kernel)": "frame_crc_varlen8_kernel<false, false",
    "seal (config 2 encode side), pass 2: non-temporal trailer stores": "seal_scatter_kernel",
    "validate, fixed 1500 B (config 2 in bench; config-4 shard and the seal's pass 1 in bench_configs)":
        "fixed_kernel<6, false",
    "parse: walk": "parse_walk",
    "parse: emit": "parse_emit",
}


def kernel_stats(path):
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            out[r["Name"]] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                              "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3}
    return out


def pick(stats, sub):
    hits = {k: v for k, v in stats.items() if sub in k}
    return next(iter(hits.items())) if len(hits) == 1 else (None, None)


def last_json(path):
    with open(path) as f:
        lines = [l for l in f if l.startswith("{")]
    return json.loads(lines[-1])


def main():
    tag, prefix = sys.argv[1], sys.argv[2]
    src = os.path.join(REPO, "gpurun_out", tag)
    dst = os.path.join(REPO, "profiles")
    copies = {"bench_ktrace/run_kernel_stats.csv": "bench_kernel_stats.csv",
              "bench_fetch/run_counter_collection.csv": "bench_pmc_fetch.csv",
              "bench_write/run_counter_collection.csv": "bench_pmc_write.csv",
              "cfg_ktrace/run_kernel_stats.csv": "configs_kernel_stats.csv",
              "cfg_fetch/run_counter_collection.csv": "configs_pmc_fetch.csv",
              "cfg_write/run_counter_collection.csv": "configs_pmc_write.csv",
              "configs.log": "configs.jsonl"}
    for s, d in copies.items():
        if os.path.exists(os.path.join(src, s)):
            shutil.copy(os.path.join(src, s), os.path.join(dst, f"{prefix}_{d}"))
    # the bench kernel's dispatches of the timed steps (the trace's last `steps` dispatches: the
    # settle and warmup launches before them include cold-GPU ones)
    tr = os.path.join(src, "bench_ktrace", "run_kernel_trace.csv")
    if os.path.exists(tr):
        with open(tr) as f:
            durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(f)
                    if BENCH_KERNEL in r["Kernel_Name"]]
        steps = 20  # tools/gpu_profile.sh: bench.py --steps 20
        timed = durs[-steps:]
        with open(os.path.join(dst, f"{prefix}_bench_timed_dispatches.json"), "w") as f:
            json.dump({"kernel": BENCH_KERNEL, "dispatches_in_trace": len(durs), "timed_steps": steps,
                       "timed_avg_us": round(sum(timed) / len(timed), 2), "all_avg_us": round(sum(durs) / len(durs), 2),
                       "timed_us": [round(x, 1) for x in timed],
                       "source": "rocprofv3 --kernel-trace of `python3 bench.py --steps 20 --warmup 5 "
                                 "--no-cpu-baseline` (tools/gpu_profile.sh), End - Start per dispatch"}, f, indent=1)
    bench_path = os.path.join(src, "bench.json")
    bench = last_json(bench_path if os.path.exists(bench_path) else os.path.join(src, "bench_ktrace.log"))
    with open(os.path.join(dst, f"{prefix}_bench.json"), "w") as f:
        f.write(json.dumps(bench) + "\n")

    # per-kernel summary of the configs run
    summary = {}
    kst = kernel_stats(os.path.join(src, "cfg_ktrace", "run_kernel_stats.csv"))
    for label, sub in CFG_KERNELS.items():
        name, st = pick(kst, sub)
        if name is None:
            continue
        fe = summarise(os.path.join(src, "cfg_fetch"), sub).get("FETCH_SIZE", {})
        wr = summarise(os.path.join(src, "cfg_write"), sub).get("WRITE_SIZE", {})
        summary[label] = {"kernel": name, **st,
                          "fetch_bytes_per_dispatch": round(fe["fetch_bytes_x2"]) if fe else None,
                          "write_bytes_per_dispatch": round(wr["write_bytes"]) if wr else None,
                          "pmc_dispatches": {"FETCH_SIZE": fe.get("dispatches"), "WRITE_SIZE": wr.get("dispatches")}}
    summary["_note"] = ("avg/min/max from rocprofv3 --kernel-trace --stats of tools/bench_configs.py --only "
                        "varlen,shard,seal,parse --reps 10 (several workloads per kernel name are averaged "
                        "together: the fixed validate kernel runs config 4's shard there, 3 launches of 12.5M/3 "
                        "frames, and the seal's first pass, 1M frames); FETCH_SIZE KiB x1024 x2 (gfx950 correction), WRITE_SIZE KiB x1024, per dispatch, "
                        "from separate --pmc passes (--reps 3)")
    with open(os.path.join(dst, f"{prefix}_kernels.json"), "w") as f:
        json.dump(summary, f, indent=1)

    fetch = summarise(os.path.join(src, "bench_fetch"), BENCH_KERNEL)["FETCH_SIZE"]
    write = summarise(os.path.join(src, "bench_write"), BENCH_KERNEL)["WRITE_SIZE"]
    out = {
        "frames": bench["config"]["frames_per_gpu"],
        "frame_len": bench["config"]["frame_len"],
        "kernel": bench["roofline"]["kernel"].split(" (")[0],
        "fetch_bytes_per_launch": round(fetch["fetch_bytes_x2"]),
        "write_bytes_per_launch": round(write["write_bytes"]),
        "hbm_bytes_per_launch": round(fetch["fetch_bytes_x2"] + write["write_bytes"]),
        "dispatches_averaged": {"FETCH_SIZE": fetch["dispatches"], "WRITE_SIZE": write["dispatches"]},
        "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) of `python3 bench.py "
                  "--steps 5 --warmup 2 --no-cpu-baseline` (tools/gpu_profile.sh); FETCH_SIZE KiB x1024 x2 "
                  "(gfx950 half-count correction, MI355X_MICROARCH.md HBM section), WRITE_SIZE KiB x1024; "
                  f"raw CSVs in profiles/{prefix}_bench_pmc_*.csv",
    }
    with open(os.path.join(dst, "pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(summary, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
