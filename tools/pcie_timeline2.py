"""Device timeline of the last sahara_gpu_search_reads[_compact] call of a
rocprofv3 --kernel-trace --memory-copy-trace run (tools/pcie_sweep.py): kernels
and copies relative to the call's first upload DMA, the busy time of each copy
direction, and per kernel name the count and summed duration.

usage: python tools/pcie_timeline2.py <dir with *_kernel_trace.csv, *_memory_copy_trace.csv> [--all]
"""
import collections
import csv
import glob
import re
import sys

d = sys.argv[1]


def short(n):
    if "rocprim" in n:
        return "rp:" + ",".join(re.findall(r"detail::(\w+)<", n)[1:2])
    m = re.search(r"(k[A-Z]\w+)", n)
    return m.group(1) if m else n[:30]


kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
ct = glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True)
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), "q" + r.get("Queue_Id", "?"))
      for r in csv.DictReader(open(kt))]
cp = []
if ct:
    for r in csv.DictReader(open(ct[0])):
        cp.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Operation", "copy")),
                   int(r.get("Bytes", r.get("Size", 0)) or 0)))
ev.sort()
pk = [e for e in ev if e[2] == "kPackFrom2"]
starts = [pk[0][0]] + [b[0] for a, b in zip(pk, pk[1:]) if b[0] - a[0] > 5_000_000]
t0 = starts[-1]
t0 = max([s for s, e, k, b in cp if s <= t0] or [t0 - 1_000_000])
t1 = max(e for s, e, k, q in ev if s >= t0)
win = sorted([e for e in ev if t0 <= e[0] <= t1] + [(s, e, f"COPY {k} {b/1e6:.1f}MB", "dma") for s, e, k, b in cp
                                                     if t0 <= s <= t1])
if "--all" in sys.argv:
    for s, e, n, q in win:
        print(f"{(s - t0) / 1e3:9.2f} {(e - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f}  {q:5s} {n}")
else:
    for s, e, n, q in win:
        if n.startswith(("kSearchText", "kSearchFM", "kSeedItems", "kCountRows", "kCompactHits", "kSortDecode",
                         "kLocate")) or (n.startswith("COPY") and e - s > 200_000):
            print(f"{(s - t0) / 1e3:9.2f} {(e - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f}  {q:5s} {n}")


def busy(iv):
    iv = sorted(iv)
    tot, cur = 0, None
    for s, e in iv:
        if cur is None or s > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    return (tot + (cur[1] - cur[0] if cur else 0)) / 1e3


print(f"window {(t1 - t0) / 1e3:.2f} ms")
for k in sorted({c[2] for c in cp}):
    sel = [(s, e) for s, e, kk, b in cp if kk == k and t0 <= s <= t1]
    print(f"copies {k}: {len(sel)} busy {busy(sel):.2f} ms, "
          f"{sum(b for s, e, kk, b in cp if kk == k and t0 <= s <= t1) / 1e9:.3f} GB")
agg = collections.defaultdict(lambda: [0, 0.0])
for s, e, n, q in win:
    if q != "dma":
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e3
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"  {n:40s} {c:5d} {t:8.2f} ms")
print(f"kernels busy {busy([(s, e) for s, e, n, q in win if q != 'dma']):.2f} ms")
