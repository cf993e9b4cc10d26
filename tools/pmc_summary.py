"""Summarise rocprofv3 counter CSVs: python tools_pmc_summary.py <dir>..."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    for f in sorted(glob.glob(f"{d}/pmc*/run_counter_collection.csv")):
        agg = collections.defaultdict(float)
        dur = {}
        for r in csv.DictReader(open(f)):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        ms = sum(dur.values()) / 1e6
        print(f.split("/")[-2], f"dispatches={len(dur)} kernel_ms={ms:.2f}",
              " ".join(f"{k}={v:.4g}" for k, v in sorted(agg.items())))
