#!/bin/bash
# Device timeline of the headline call's last step (kernel + memory-copy trace)
# and its fill / text / gaps / drain split: tools/call_timeline.sh <outdir> [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --no-device-resident --no-ingest --steps 3 --warmup 1 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "trace failed"; tail -5 "$OUT/bench.err"; exit 1; }
python3 "$R/tools/pcie_timeline2.py" "$OUT/trace" > "$OUT/timeline.txt" || exit 1
python3 "$R/tools/pcie_timeline2.py" "$OUT/trace" --all > "$OUT/timeline_all.txt" || exit 1
python3 "$R/tools/timeline_split.py" "$OUT/timeline.txt" | tee "$OUT/split.txt"
rm -f "$OUT"/trace/*_trace.csv
