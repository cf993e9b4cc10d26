"""Timeline of one sahara_gpu_search_reads call (bench.py's PCIe-inclusive
path) from a rocprofv3 --kernel-trace --memory-copy-trace run: kernels and
copies relative to the call's first kInterleaveRC, and the busy time of each
copy direction and of the search kernels.

usage: python tools/pcie_timeline.py <dir with run_kernel_trace.csv, run_memory_copy_trace.csv>
"""
import csv
import re
import sys

d = sys.argv[1]


def short(n):
    if "rocprim" in n:
        return "rp:" + ",".join(re.findall(r"detail::(\w+)<", n)[1:2])
    m = re.search(r"(k[A-Z]\w+)", n)
    return m.group(1) if m else n[:30]


ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), "q" + r["Queue_Id"])
      for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv"))]
cp = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Operation", "copy")),
       int(r.get("Bytes", r.get("Size", 0)) or 0)) for r in csv.DictReader(open(f"{d}/run_memory_copy_trace.csv"))]
ev.sort()
rc = [e for e in ev if e[2] == "kInterleaveRC"]
# calls = clusters of kInterleaveRC dispatches; the last call (warm) is shown
starts = [rc[0][0]] + [b[0] for a, b in zip(rc, rc[1:]) if b[0] - a[0] > 5_000_000]
t0 = starts[-1]
last_rc = max(e[0] for e in rc if e[0] >= t0)
# the call's first upload DMA precedes its first kInterleaveRC
t0 = max([s for s, e, k, b in cp if s <= t0] or [t0])
t1 = next((e[0] for e in ev if e[0] > last_rc and e[2] == "kUnpackNibbles"), ev[-1][1])
win = sorted([e for e in ev if t0 <= e[0] < t1] + [(s, e, f"COPY {k} {b/1e6:.1f}MB", "dma") for s, e, k, b in cp
                                                    if t0 <= s < t1])
for s, e, n, q in win:
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


end = max(e for s, e, n, q in win)
print(f"window {(end - t0) / 1e3:.2f} ms")
for k in sorted({c[2] for c in cp}):
    sel = [(s, e) for s, e, kk, b in cp if kk == k and t0 <= s < t1]
    print(f"copies {k}: {len(sel)} busy {busy(sel):.2f} ms, {sum(b for s, e, kk, b in cp if kk == k and t0 <= s < t1)/1e9:.3f} GB")
print(f"search kernels busy {busy([(s, e) for s, e, n, q in win if q != 'dma']):.2f} ms")
