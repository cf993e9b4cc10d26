#!/bin/bash
# HBM traffic (FETCH_SIZE) and SQ counter passes of the search kernels for the
# given configs (default c5 c2), each pass a rocprofv3 run of its own; the
# per-launch summaries land in $1/traffic_<cfg>.json and $1/pmc_<cfg>.json
# (copied to profiles/ by hand; bench.py reads them from there).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
CFGS=${*:-c5 c2}
mkdir -p "$OUT"
for c in $CFGS; do
  bash "$R/tools/traffic.sh" "$OUT/traffic_$c" --config $c || { echo "traffic $c failed"; exit 1; }
  python3 "$R/tools/traffic_summary.py" "$OUT/traffic_$c" "$OUT/traffic_$c.json" "$OUT/traffic_$c.txt" || exit 1
  rm -f "$OUT/traffic_$c/trace/run_kernel_trace.csv"
  bash "$R/tools/pmc_text.sh" "$OUT/pmc_$c" --config $c || { echo "pmc $c failed"; exit 1; }
  cp "$OUT/pmc_$c/pmc.json" "$OUT/pmc_$c.json"; cp "$OUT/pmc_$c/pmc.txt" "$OUT/pmc_$c.txt"
  echo "== $c"; cat "$OUT/traffic_$c.txt" "$OUT/pmc_$c.txt" | head -40
done
