"""Copy a tools/gpu_profile.sh run (gpurun_out/<tag>/) into profiles/ under a round prefix and
regenerate profiles/pmc_traffic.json (the HBM bytes per validate launch that bench.py reports
as roofline.traffic).  Usage: python tools/update_profiles.py <tag> <prefix>, e.g. r1c r1."""
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
from pmc_summary import summarise  # noqa: E402

KERNEL = "fixed_kernel<6, false"


def main():
    tag, prefix = sys.argv[1], sys.argv[2]
    src = os.path.join(REPO, "gpurun_out", tag)
    dst = os.path.join(REPO, "profiles")
    shutil.copy(os.path.join(src, "ktrace", "run_kernel_stats.csv"), os.path.join(dst, f"{prefix}_kernel_stats.csv"))
    shutil.copy(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), os.path.join(dst, f"{prefix}_pmc_fetch.csv"))
    shutil.copy(os.path.join(src, "pmc_write", "run_counter_collection.csv"), os.path.join(dst, f"{prefix}_pmc_write.csv"))
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"{prefix}_bench.json"))
    fetch = summarise(os.path.join(src, "pmc_fetch"), KERNEL)["FETCH_SIZE"]
    write = summarise(os.path.join(src, "pmc_write"), KERNEL)["WRITE_SIZE"]
    bench = json.load(open(os.path.join(src, "bench.json")))
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
                  f"raw CSVs in profiles/{prefix}_pmc_*.csv",
    }
    with open(os.path.join(dst, "pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
