"""profiles/<prefix>_sq_counters.json from tools/pmc_sq.sh runs: per workload, the mean of every SQ counter
per dispatch of the workload's kernel, per wave (SQ_WAVES) and per set of 8 frames (config 3's 10M-frame
batch: 1.25M sets), and the fractions the DESIGN quotes.  Usage:
    python tools/sq_counters.py <tag> <prefix> <workload>:<kernel substring> ..."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
from pmc_summary import summarise  # noqa: E402

SETS = 10_000_000 // 8


def main():
    tag, prefix = sys.argv[1], sys.argv[2]
    out = {"_note": f"rocprofv3 --pmc passes of tools/pmc_sq.sh (gpurun_out/{tag}, untracked); per dispatch means; "
                    "per_set = per dispatch / 1.25M sets of 8 frames (config 3)"}
    for spec in sys.argv[3:]:
        w, sub = spec.split(":", 1)
        d = {}
        for g in ("p1", "p2"):
            path = os.path.join(REPO, "gpurun_out", tag, f"{w}_{g}")
            if os.path.isdir(path):
                d.update({k: v["mean"] for k, v in summarise(path, sub).items()})
        if not d:
            continue
        ent = dict(d)
        ent["kernel_substring"] = sub
        waves = d.get("SQ_WAVES", 0)
        if waves:
            ent["per_wave"] = {k: round(v / waves, 1) for k, v in d.items() if k != "SQ_WAVES"}
        ent["per_set"] = {k: round(v / SETS, 1) for k, v in d.items() if k != "SQ_WAVES"}
        if "SQ_WAVE_CYCLES" in d:
            if "SQ_INSTS_VALU" in d:
                ent["valu_issue_frac_of_wave_cycles"] = round(d["SQ_INSTS_VALU"] / d["SQ_WAVE_CYCLES"], 4)
            if "SQ_WAIT_INST_ANY" in d:
                ent["wait_inst_any_frac_of_wave_cycles"] = round(d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"], 4)
        if "SQ_LDS_BANK_CONFLICT" in d and "SQ_ACTIVE_INST_LDS" in d:
            ent["lds_bank_conflict_frac_of_lds_active"] = round(d["SQ_LDS_BANK_CONFLICT"] / d["SQ_ACTIVE_INST_LDS"], 4)
        out[w] = ent
    with open(os.path.join(REPO, "profiles", f"{prefix}_sq_counters.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v.get("per_set") for k, v in out.items() if not k.startswith("_")}, indent=1))


if __name__ == "__main__":
    main()
