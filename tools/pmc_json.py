"""SQ counter passes (tools/pmc_text.sh) -> per-launch figures per kernel, as JSON.

usage: python tools/pmc_json.py <pmc dir> <out.json> [summary.txt]

Each <dir>/pmc*/run_counter_collection.csv is one rocprofv3 --pmc pass over
the same bench command; a counter's value per launch is its sum over the rows
of one dispatch, averaged over the kernel's dispatches. bench.py reads
SQ_INSTS_VALU of its dominant kernel from the output (roofline.valu_issue).
Derived ratios (SQ_WAVE_CYCLES, SQ_ACTIVE_INST_*, SQ_WAIT_* all count
quad-cycles on gfx950, MI355X_MICROARCH.md):
  issue_active   = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES  (share of wave time issuing)
  wait_any       = SQ_WAIT_ANY / SQ_WAVE_CYCLES          (waiting on memory / LDS counters)
  lds_conflict   = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(n):
    m = re.search(r"::(k[A-Z]\w*)", n) or re.search(r"(k[A-Z]\w*)", n)
    return m.group(1) if m else n[:40]


def lib_build_id():
    """The build id of the library the profiled command loaded (sahara_build_id)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import sahara_amd
    return sahara_amd.build_id()


def main(d, out, txt=None):
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for f in sorted(glob.glob(f"{d}/pmc*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            per[short(r["Kernel_Name"])][r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    res, lines = {}, []
    for k, counters in sorted(per.items()):
        avg = {c: sum(v.values()) / len(v) for c, v in counters.items()}
        disp = max(len(v) for v in counters.values())
        e = {c: round(v) for c, v in sorted(avg.items())}
        e["dispatches"] = disp
        if avg.get("SQ_WAVE_CYCLES"):
            for name, num in (("issue_active", "SQ_ACTIVE_INST_ANY"), ("wait_any", "SQ_WAIT_ANY"),
                              ("valu_active", "SQ_ACTIVE_INST_VALU")):
                if num in avg:
                    e[name] = round(avg[num] / avg["SQ_WAVE_CYCLES"], 3)
        if avg.get("SQ_ACTIVE_INST_LDS") and "SQ_LDS_BANK_CONFLICT" in avg:
            e["lds_conflict"] = round(avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_ACTIVE_INST_LDS"], 3)
        res[k] = e
        lines.append(f"{k:16s} " + " ".join(f"{c}={v:.4g}" for c, v in e.items()))
    res["build_id"] = lib_build_id()
    json.dump(res, open(out, "w"), indent=1)
    print("\n".join(lines))
    if txt:
        open(txt, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
