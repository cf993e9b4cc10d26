"""Timeline of the last search step in a rocprofv3 kernel trace: one line per
kernel dispatch (start/end relative to the step's first seed kernel, in us).
With a third argument "gap": the step before the last one instead, from the
dispatches before its first seed kernel (the previous step's tail) through the
last step's first seed kernel, so that the idle time between steps shows."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
def short(n):
    if "rocprim" in n:
        return "rp:" + ",".join(re.findall(r"detail::(\w+)<", n)[1:2])
    m = re.search(r"(k[A-Z]\w+)", n)
    return m.group(1) if m else n[:30]
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Stream_Id"], r["Queue_Id"]) for r in rows]
ev.sort()
seeds = [i for i, e in enumerate(ev) if e[2] == "kSeedItems"]
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 5
gap = len(sys.argv) > 3 and sys.argv[3] == "gap"
first = seeds[-2 * nb] if gap else seeds[-nb]
t0 = ev[first][0]
for s, e, n, st, q in ev[max(0, first - 12) if gap else first:seeds[-nb] + 1 if gap else None]:
    if n.startswith("kDigest"):
        break
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q} {n}")
