#!/bin/bash
# The default bench line and a rocprofv3 kernel trace (--stats) of the same
# command, so that roofline.launch_ms can be checked against the profile:
# tools/bench_profiled.sh <outdir> [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -5 "$OUT/bench.err"; exit 1; }
cp "$OUT"/trace/run_kernel_stats.csv "$OUT/kernel_stats.csv"
python3 - "$OUT" <<'PY'
import csv, json, re, sys
out = sys.argv[1]
d = json.load(open(f"{out}/bench.json"))
rl = d["roofline"]
# the dominant kernel's launches in trace order: the timed call's are the ones
# after its two warmup calls (bench.py runs the packed calls first)
dom = rl["kernel"]
rows = []
for x in csv.DictReader(open(f"{out}/trace/run_kernel_trace.csv")):
    m = re.search(r"(k[A-Z]\w+)<(.*)>", x["Kernel_Name"])
    if m and m.group(1) == dom and [t.strip() for t in m.group(2).split(",")][2] == "false":
        rows.append((int(x["Start_Timestamp"]), int(x["End_Timestamp"])))
rows.sort()
with open(f"{out}/{dom}_launches.csv", "w") as f:
    f.write("start_ns,end_ns,duration_us\n")
    for a, b in rows:
        f.write(f"{a},{b},{(b - a) / 1e3:.1f}\n")
per = round(d["config"]["timed_launches"][dom]["launches_per_step"])
lo, hi = 2 * per, (2 + d["steps"]) * per
timed = rows[lo:hi]
avg_timed = sum(b - a for a, b in timed) / max(1, len(timed)) / 1e6
print(f"{dom}: timed launches {lo}..{hi} of {len(rows)}: rocprof avg {avg_timed:.3f} ms vs bench launch_ms "
      f"{rl['launch_ms']} (ratio {rl['launch_ms'] / avg_timed:.3f})")
ks = {}
for x in csv.DictReader(open(f"{out}/kernel_stats.csv")):
    m = re.search(r"(k[A-Z]\w+)<(.*)>", x["Name"])
    if not m:
        continue
    targs = [t.strip() for t in m.group(2).split(",")]
    if m.group(1).startswith("kSearch") and len(targs) >= 3 and targs[2] == "true":
        continue  # count-mode instantiations (the bench's instrumented runs)
    k = ks.setdefault(m.group(1), [0, 0.0])
    k[0] += int(x["Calls"]); k[1] += float(x["TotalDurationNs"])
n, tot = ks[dom]
avg = tot / n / 1e6
print(f"bench {d['value']/1e6:.1f}M reads/s; {dom}: all {n} launches (timed, warmup, device-resident, "
      f"PCIe-inclusive calls) average {avg:.3f} ms")
json.dump({"kernel": dom, "build_id": d["config"].get("build_id"), "bench_value": d["value"],
           "bench_launch_ms": rl["launch_ms"], "rocprof_timed_avg_ms": round(avg_timed, 4),
           "timed_launches": len(timed), "ratio": round(rl["launch_ms"] / avg_timed, 4),
           "rocprof_all_avg_ms": round(avg, 4), "all_launches": n}, open(f"{out}/summary.json", "w"), indent=1)
PY
rm -f "$OUT"/trace/run_kernel_trace.csv
