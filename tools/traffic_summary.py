"""Summarise tools/traffic.sh output: per-kernel average duration (kernel
trace), FETCH_SIZE per dispatch (PMC pass) and the FETCH_SIZE calibration on
random 64-B line gathers (tools/gather_bench).

usage: python tools/traffic_summary.py <traffic dir> <out.json> [summary.txt]

FETCH_SIZE (KB) = TCC_EA0_RDREQ x 64 B / 1024. MI355X_MICROARCH.md: for wide
coalesced streaming reads it reports half the bytes; for random 64-B line
gathers the calibration below measures the factor directly (bytes per line
reported / 64), and that factor is applied to the search kernels, whose HBM
traffic is random 64-B lines (Occ lines, SA entries, text windows).
"""
import collections
import csv
import json
import os
import re
import sys


def short(n):
    m = re.search(r"::(k[A-Z]\w*(?:<[^>]*>)?)\(", n)
    return m.group(1) if m else n[:40]


def lib_build_id():
    """The build id of the library the profiled command loaded (sahara_build_id)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import sahara_amd
    return sahara_amd.build_id()


def main(d, out, txt=None):
    lines = []
    stats = {}
    for r in csv.DictReader(open(f"{d}/trace/run_kernel_stats.csv")):
        k = short(r["Name"])
        if k.startswith(("kSearch", "kSeed", "kResolve", "kLocate")):
            stats[k] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3)
    # calibration: kGroup<U, G> dispatches: lines = 2048 blocks * 256 / G * 64 iters * U
    cal = []
    per = collections.defaultdict(float)
    names = {}
    if os.path.exists(f"{d}/calib/run_counter_collection.csv"):
        for r in csv.DictReader(open(f"{d}/calib/run_counter_collection.csv")):
            per[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
            names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
        for disp, kb in sorted(per.items()):
            U, G = map(int, re.search(r"kGroup<(\d+), (\d+)>", names[disp]).groups())
            cal.append(kb * 1024 / (2048 * 256 / G * 64 * U))
        big = cal[len(cal) // 3:]  # the 6.75 and 24 GB footprints (beyond the 256 MB MALL)
        factor = 64.0 / (sum(big) / len(big))
        lines.append(f"calibration: random 64-B line gathers report {sum(big)/len(big):.2f} B/line in FETCH_SIZE "
                     f"-> factor {factor:.3f}")
    else:  # no calibration pass in this run: the factor measured before (profiles/traffic_c3.json)
        factor = float(os.environ.get("FETCH_FACTOR", "1.0"))
        lines.append(f"calibration: not rerun, factor {factor:.3f}")
    fetch = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{d}/pmc_fetch/run_counter_collection.csv")):
        fetch[(short(r["Kernel_Name"]), int(r["Dispatch_Id"]))].append(
            (float(r["Counter_Value"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    agg = collections.defaultdict(list)
    for (k, _), v in fetch.items():
        agg[k].append((sum(x[0] for x in v), v[0][1]))
    res = {}
    for k, v in sorted(agg.items()):
        kb = sum(x[0] for x in v) / len(v)
        b = kb * 1024 * factor
        calls, avg_us = stats.get(k, (len(v), sum(x[1] for x in v) / len(v) / 1e3))
        res[k.split("<")[0]] = {"bytes_per_launch": round(b), "avg_launch_us": round(avg_us, 1),
                                "traffic_GBs": round(b / (avg_us / 1e6) / 1e9, 1), "dispatches": len(v)}
        lines.append(f"{k:28s} launches={len(v):3d} avg={avg_us:9.1f} us  FETCH_SIZE={kb/1024/1024:8.3f} GiB/launch "
                     f"-> {b/1e9:7.3f} GB/launch = {b/(avg_us/1e6)/1e9:7.1f} GB/s")
    res["calibration_factor"] = round(factor, 4)
    res["build_id"] = lib_build_id()
    if os.environ.get("STEPS"):  # timed steps of the profiled command (no warmup): launches per step
        res["steps"] = int(os.environ["STEPS"])
    json.dump(res, open(out, "w"), indent=1)
    text = "\n".join(lines)
    print(text)
    if txt:
        open(txt, "w").write(text + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
