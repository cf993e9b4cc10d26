"""Fill / overlap / drain of each call in a device timeline (tools/pcie_timeline2.py
output: one event per line, `start end duration queue name...` in microseconds
from the call's first event).

usage: python tools/timeline_split.py <timeline.txt>

  fill    first event (the first chunk's DMA) -> first kSearchText start
  text    union of the kSearchText launches (the bound of the pipelined pass)
  gaps    time between kSearchText launches inside the text span
  drain   last kSearchText end -> the call's last event (locate, sort, records)
"""
import sys


def main(path):
    ev = []
    for line in open(path):
        f = line.split()
        if len(f) < 5:
            continue
        try:
            t0, t1 = float(f[0]), float(f[1])
        except ValueError:
            continue
        ev.append((t0, t1, " ".join(f[4:])))
    if not ev:
        raise SystemExit("no events")
    # several calls in the window (short calls, C2): a call begins after 500 us
    # in which nothing ran
    ev.sort()
    calls, cur, last = [], [], None
    for e in ev:
        if last is not None and e[0] > last + 500.0:
            calls.append(cur)
            cur = []
        cur.append(e)
        last = e[1] if last is None else max(last, e[1])
    calls.append(cur)
    for c in calls:
        if any(n.startswith("kSearchText") for _, _, n in c):
            split(c)


def split(ev):
    start = min(e[0] for e in ev)
    end = max(e[1] for e in ev)
    text = sorted((a, b) for a, b, n in ev if n.startswith("kSearchText"))
    busy, gaps, cur = 0.0, 0.0, None
    for a, b in text:
        if cur is None:
            cur = [a, b]
        elif a <= cur[1]:
            cur[1] = max(cur[1], b)
        else:
            busy += cur[1] - cur[0]
            gaps += a - cur[1]
            cur = [a, b]
    if cur:
        busy += cur[1] - cur[0]
    fill = text[0][0] - start if text else 0.0
    drain = end - max(b for _, b in text) if text else 0.0
    tot = end - start
    print(f"call {tot:.0f} us: fill {fill:.0f} ({fill / tot:.1%}), text {busy:.0f} ({busy / tot:.1%}), "
          f"gaps between text launches {gaps:.0f} ({gaps / tot:.1%}), drain {drain:.0f} ({drain / tot:.1%})")


if __name__ == "__main__":
    main(sys.argv[1])
