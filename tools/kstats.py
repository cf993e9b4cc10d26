"""Per-kernel summary of a rocprofv3 kernel_stats.csv (short names)."""
import csv
import re
import sys

for x in csv.DictReader(open(sys.argv[1])):
    n = x["Name"]
    if "rocprim" in n:
        short = "rocprim:" + ",".join(re.findall(r"detail::(\w+)<", n)[1:3])
    else:
        m = re.search(r"(k[A-Z]\w+)", n)
        short = m.group(1) if m else n[:40]
    print(f"{short[:70]:70s} {x['Calls']:>5} {float(x['AverageNs']) / 1e3:10.1f}us {float(x['TotalDurationNs']) / 1e6:8.2f}ms")
