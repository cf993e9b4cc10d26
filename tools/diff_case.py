"""Debug helper: run one golden case on the GPU and print the hit rows that
differ from tests/golden (missing / extra). usage: python tools/diff_case.py <case>"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import sahara_amd as sa  # noqa: E402
from helpers import hits_as_rows  # noqa: E402
from test_golden import CASES, GOLD, IDX, expected, patterns  # noqa: E402

name = sys.argv[1]
c = CASES[name]
I = sa.BiFMIndex.load(os.path.join(GOLD, IDX[c["fixture"]]))
pats = patterns(c["fixture"], c["reverse"])
m = pats.shape[1]
edit = c["metric"] == "lev"
sch = sa.search_scheme(c["generator"], 0, c["k"], m, hamming=not edit)
got = hits_as_rows(sa.search(I, pats, sch, edit=edit))
want = expected(name)
g = collections.Counter(map(tuple, got.tolist()))
w = collections.Counter(map(tuple, want.tolist()))
print("got", len(got), "want", len(want))
print("missing", sorted((w - g).elements())[:40])
print("extra", sorted((g - w).elements())[:40])
pi, l, u = sch
for s in range(min(len(pi), 0)):
    print("search", s, "pi", pi[s][:5], "...", "l", "".join(map(str, l[s])), "u", "".join(map(str, u[s])))
