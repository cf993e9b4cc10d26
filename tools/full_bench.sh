#!/bin/bash
# Default bench (with the CPU baseline) + rocprofv3 kernel trace + FETCH_SIZE pass; outputs in $1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
timeout -k 10 600 python3 "$R/bench.py" "$@" > "$OUT/bench.json" 2> "$OUT/bench.log" || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
cat "$OUT/bench.json"
bash "$R/tools/traffic.sh" "$OUT/traffic" || exit 1
python3 "$R/tools/traffic_summary.py" "$OUT/traffic" "$OUT/traffic_c3.json" "$OUT/traffic_c3.txt"
