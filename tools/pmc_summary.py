"""Summarise rocprofv3 counter CSVs per kernel: python tools/pmc_summary.py <dir>...

Each <dir>/pmc*/run_counter_collection.csv is one counter pass
(tools/profile.sh); values are summed over the dispatches of each kernel.
"""
import collections
import csv
import glob
import re
import sys


def short(n):
    m = re.search(r"::(k[A-Z]\w*(?:<[^>]*>)?)\(", n)
    return m.group(1) if m else n[:40]


for d in sys.argv[1:]:
    for f in sorted(glob.glob(f"{d}/pmc*/run_counter_collection.csv")):
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        dur = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for k in sorted(agg):
            ms = sum(dur[k].values()) / 1e6
            print(f.split("/")[-2], k, f"dispatches={len(dur[k])} kernel_ms={ms:.2f}",
                  " ".join(f"{c}={v:.4g}" for c, v in sorted(agg[k].items())))
