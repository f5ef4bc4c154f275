"""profiles/ from a tools/profile_workloads.sh run: copies every workload's kernel-trace stats as
profiles/<prefix>_<workload>_kernel_stats.csv (the raw per-dispatch counter CSVs stay under
gpurun_out/<tag>/, untracked: rerun tools/profile_workloads.sh <tag> to regenerate them), and writes
(merges into) profiles/<prefix>_summary.json: per workload, the kernel(s) it times, the average and
median dispatch duration from the trace (warm dispatches only), the algorithmic bytes per dispatch,
the roofline fraction recomputed from them, and FETCH/WRITE bytes per dispatch (FETCH_SIZE KiB x1024
x2, the gfx950 correction of MI355X_MICROARCH.md; WRITE_SIZE KiB x1024).  Also regenerates
profiles/pmc_traffic.json (bench.py's roofline.traffic) from the bench workload.
Usage: python tools/profile_summary.py <tag> <prefix>, e.g. r3prof r3."""
import csv
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
from pmc_summary import summarise  # noqa: E402

PEAK_GBS = 8000.0
N2, L2 = 1_000_000, 1500
N3, BYTES3 = 10_000_000, None  # config 3's byte count comes from the workload's JSON line
SHARD = 12_500_000
# workload -> [(label, kernel-name substring, algorithmic bytes per dispatch or None, dispatches per op)]
WORKLOADS = {
    "bench": [("config 2 validate (bench line)", "frame_crc_fixed_kernel<6, false", N2 * (L2 + 5)),
              ("read-only streaming ceiling probe over the same 1.5 GB", "read_stream_kernel", N2 * L2 // 1024 * 1024)],
    "varlen": [("config 3 validate", "frame_crc_varlen8_kernel<false, false", "varlen"),
               ("config 3 validate, second launch (frames over 13 lines: none here, each workgroup reads its "
                "count and returns)", "frame_crc_long8_kernel<false, false", None)],
    "gate_tg": [("gate on the test-generator batch, first launch", "frame_crc_varlen8_kernel<false, false", None),
                ("gate on the test-generator batch, second launch (the 38 % of frames over 13 lines)",
                 "frame_crc_long8_kernel<false, false", None)],
    "shard": [("config 4 per-GPU shard validate (3 launches of 4.17M frames)", "frame_crc_fixed_kernel<6, false",
               SHARD // 3 * (L2 + 5))],
    "seal": [("config 2 seal, one kernel (product: each workgroup's trailers after its reads)",
              "frame_crc_fixed_kernel<6, true", N2 * (L2 + 4)),
             ("config 2 seal, two passes (comparison): pass 1 (CRC words)", "frame_crc_fixed_kernel<6, false",
              N2 * (L2 + 4)),
             ("config 2 seal, two passes (comparison): pass 2 (trailer stores)", "seal_scatter_kernel", N2 * 8)],
    "seal_varlen": [("config 3 seal", "frame_crc_varlen8_kernel<true, false", "seal_varlen"),
                    ("config 3 seal, second launch (none over 13 lines)", "frame_crc_long8_kernel<true, false", None)],
    "parse": [("parse walk (test-generator workload)", "parse_walk", None),
              ("parse emit (test-generator workload)", "parse_emit", None)],
    "parse_mtu": [("parse walk (frames <= MAX_FRAME_SIZE)", "parse_walk", None),
                  ("parse emit (frames <= MAX_FRAME_SIZE)", "parse_emit", None)],
}


def trace_durations(path, sub):
    with open(path) as f:
        return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(f)
                if sub in r["Kernel_Name"]]


def last_json(path):
    try:
        with open(path) as f:
            lines = [ln for ln in f if ln.startswith("{")]
        return json.loads(lines[-1]) if lines else {}
    except OSError:
        return {}


def main():
    tag, prefix = sys.argv[1], sys.argv[2]
    src = os.path.join(REPO, "gpurun_out", tag)
    dst = os.path.join(REPO, "profiles")
    # (merged into an existing summary: a run over some workloads refreshes only their entries)
    path = os.path.join(dst, f"{prefix}_summary.json")
    summary = json.load(open(path)) if os.path.exists(path) else {}
    for w, kernels in WORKLOADS.items():
        kt = os.path.join(src, f"{w}_ktrace")
        if not os.path.isdir(kt):
            continue
        for sfx, name in (("run_kernel_stats.csv", "kernel_stats.csv"),):
            for root, _, files in os.walk(kt):
                if sfx in files:
                    shutil.copy(os.path.join(root, sfx), os.path.join(dst, f"{prefix}_{w}_{name}"))
        line = last_json(os.path.join(src, f"{w}_ktrace.log"))
        trace = None
        for root, _, files in os.walk(kt):
            if "run_kernel_trace.csv" in files:
                trace = os.path.join(root, "run_kernel_trace.csv")
        for label, sub, algo in kernels:
            d = trace_durations(trace, sub) if trace else []
            warm = d[5:] if len(d) > 10 else d  # (the first dispatches of a process run on a cold GPU)
            if algo == "varlen":
                algo = line.get("algorithmic_bytes")
            elif algo == "seal_varlen":
                algo = line.get("algorithmic_bytes")
            fe = summarise(os.path.join(src, f"{w}_fetch"), sub).get("FETCH_SIZE", {})
            wr = summarise(os.path.join(src, f"{w}_write"), sub).get("WRITE_SIZE", {})
            ent = {"workload": w, "run_tag": tag, "kernel_substring": sub, "dispatches": len(d),
                   "avg_us": round(statistics.mean(warm), 2) if warm else None,
                   "median_us": round(statistics.median(warm), 2) if warm else None,
                   "min_us": round(min(warm), 2) if warm else None,
                   "algorithmic_bytes_per_dispatch": algo,
                   "fetch_bytes_per_dispatch": round(fe["fetch_bytes_x2"]) if fe else None,
                   "write_bytes_per_dispatch": round(wr["write_bytes"]) if wr else None}
            if algo and warm:
                ent["frac_of_8TBs_from_avg"] = round(algo / (statistics.mean(warm) * 1e-6) / 1e9 / PEAK_GBS, 4)
                ent["frac_of_8TBs_from_median"] = round(algo / (statistics.median(warm) * 1e-6) / 1e9 / PEAK_GBS, 4)
            if fe and wr and algo:
                ent["traffic_over_algorithmic"] = round((fe["fetch_bytes_x2"] + wr["write_bytes"]) / algo, 4)
            if line:
                ent["workload_line"] = {k: line[k] for k in ("kernel_ms", "ms_per_step", "ceiling_GBs",
                                                             "frac_of_ceiling", "hbm_frac", "value") if k in line}
                if "roofline" in line:
                    ent["workload_line"].update({k: line["roofline"].get(k) for k in
                                                 ("kernel_avg_ms", "frac", "ceiling_GBs", "frac_of_ceiling")})
            summary[label] = ent
    summary["_note"] = ("one process per workload (tools/profile_workloads.sh): <w>_ktrace = rocprofv3 --kernel-trace "
                        "--stats; avg/median over the trace's dispatches of that kernel after the first 5; FETCH/WRITE "
                        "from separate --pmc passes, per dispatch; algorithmic bytes per dispatch as DESIGN.md section 5")
    with open(path, "w") as f:
        json.dump(summary, f, indent=1)
    b = summary.get("config 2 validate (bench line)")
    if b and b["fetch_bytes_per_dispatch"] and b["write_bytes_per_dispatch"]:
        out = {"frames": N2, "frame_len": L2, "kernel": "ufc_dev::frame_crc_fixed_kernel<6, false, 2, 2, 8, 4224>",
               "fetch_bytes_per_launch": b["fetch_bytes_per_dispatch"],
               "write_bytes_per_launch": b["write_bytes_per_dispatch"],
               "hbm_bytes_per_launch": b["fetch_bytes_per_dispatch"] + b["write_bytes_per_dispatch"],
               "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) of `python3 bench.py "
                         "--steps 5 --warmup 2 --no-cpu-baseline --settle-ms 50 --no-ceiling` "
                         "(tools/profile_workloads.sh); FETCH_SIZE KiB x1024 x2 (gfx950 half-count correction, "
                         f"MI355X_MICROARCH.md HBM section), WRITE_SIZE KiB x1024; raw CSVs: gpurun_out/{tag}/bench_{{fetch,write}} "
                         "(untracked; tools/profile_workloads.sh regenerates them)"}
        with open(os.path.join(dst, "pmc_traffic.json"), "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
