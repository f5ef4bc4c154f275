"""Per-wave SQ counter summary of the last dispatch of a kernel in rocprofv3 --pmc CSVs.
Usage: python tools/probes/pmc_summary.py <dir with pmc*/run_counter_collection.csv> [kernel substring]"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "varlen2"
for f in sorted(glob.glob(root + "/pmc*/run_counter_collection.csv")):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
    if not agg:
        continue
    d = max(k for k, _ in agg)
    vals = {c: v for (k, c), v in agg.items() if k == d}
    waves = vals.get("SQ_WAVES") or None
    print(f.split("/")[-2], {c: (round(v / waves) if waves and c != "SQ_WAVES" else v) for c, v in sorted(vals.items())})
