"""Per call of a kernel trace (rocprofv3 kernel_trace.csv): how much of the
call the FM, text and locate kernels overlap, and the gaps between them.

usage: python tools/thread_trace.py <kernel_trace.csv>
"""
import csv
import sys


def kname(full):
    """kSearchTextBatch from 'void sahara::(anonymous namespace)::kSearchTextBatch<...>(...)'."""
    for k in ("kSearchTextBatch", "kSearchFM", "kSeedItems", "kLocate"):
        if k in full:
            return k
    return full.split("(")[0]


def union(iv):
    tot, cur = 0, None
    for a, b in sorted(iv):
        if cur is None or a > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    return tot + (cur[1] - cur[0] if cur else 0)


def main(path):
    ev = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kname(r["Kernel_Name"]),
                       r.get("Queue_Id", "")))
    ev.sort()
    calls, cur, last = [], [], None
    for e in ev:
        if last is not None and e[0] > last + 500_000:
            calls.append(cur)
            cur = []
        cur.append(e)
        last = e[1] if last is None else max(last, e[1])
    calls.append(cur)
    for c in calls:
        text = [(a, b) for a, b, n, _ in c if n.startswith("kSearchText")]
        if not text:
            continue
        fm = [(a, b) for a, b, n, _ in c if n.startswith("kSearchFM")]
        t0, t1 = c[0][0], max(b for _, b, _, _ in c)
        both = union(text) + union(fm) - union(text + fm)
        queues = sorted({q for _, _, _, q in c})
        print(f"call {(t1 - t0) / 1e6:7.2f} ms: text {union(text) / 1e6:5.2f} ms ({len(text)}), "
              f"FM {union(fm) / 1e6:5.2f} ms ({len(fm)}, summed {sum(b - a for a, b in fm) / 1e6:5.2f}), "
              f"FM beside text {both / 1e6:5.2f} ms, any kernel {union([(a, b) for a, b, _, _ in c]) / 1e6:5.2f} ms, "
              f"queues {queues}")


if __name__ == "__main__":
    main(sys.argv[1])
