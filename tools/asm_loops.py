#!/usr/bin/env python3
"""List the loops of one kernel in a gfx950 device assembly listing and the
memory waits inside each: a `s_waitcnt vmcnt(..)` inside a hot loop that
issues no load of its own means a value from outside the loop is awaited on
every trip (how the r5 text kernel lost 4.5x: a returning atomic's register
pending across the micro-step loop).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Isahara_amd/csrc \\
        --cuda-device-only -S sahara_amd/csrc/search.hip -o /tmp/search.s
    python3 tools/asm_loops.py /tmp/search.s kSearchTextILi5ELb0ELb0ELi1E

A loop is a backward branch to a label of the same function; nested loops
are listed separately (innermost first by size)."""
import re
import sys


def main(path, pattern):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^\S*%s\S*:" % re.escape(pattern), l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    label_at = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            label_at[m.group(1)] = i
    loops = []
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_(?:c)?branch\S*\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in label_at and label_at[m.group(1)] <= i:
            loops.append((label_at[m.group(1)], i))
    for a, b in sorted(loops, key=lambda x: x[1] - x[0]):
        seg = body[a:b + 1]
        waits = [l.strip() for l in seg if "s_waitcnt" in l and "vmcnt" in l]
        loads = sum(1 for l in seg if re.search(r"\b(global|buffer|flat)_(load|atomic)", l))
        print("%s..+%d  insts %d  vm-waits %d  vm-ops %d  %s" %
              (body[a].split(":")[0], b - a, sum(1 for l in seg if l.startswith("\t") and not l.strip().startswith(";")),
               len(waits), loads, "; ".join(sorted(set(waits)))[:120]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
