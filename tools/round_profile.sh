#!/bin/bash
# Round evidence on the GPU box, outputs in $1 (under gpurun_out/):
# GPU tests, kernel trace + FETCH_SIZE pass (tools/traffic.sh), their summary,
# then the default bench (CPU baseline included) with the fresh traffic figure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -5 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
bash "$R/tools/traffic.sh" "$OUT/traffic" "$@" || exit 1
python3 "$R/tools/traffic_summary.py" "$OUT/traffic" "$OUT/traffic_c3.json" "$OUT/traffic_c3.txt" || exit 1
cp "$OUT/traffic/trace/run_kernel_stats.csv" "$OUT/kernel_stats.csv"
python3 "$R/tools/timeline.py" "$OUT/traffic/trace/run_kernel_trace.csv" 5 > "$OUT/timeline.txt"
rm -rf "$OUT/traffic/trace/run_kernel_trace.csv"
timeout -k 10 600 python3 "$R/bench.py" --traffic-json "$OUT/traffic_c3.json" "$@" > "$OUT/bench.json" 2> "$OUT/bench.log" || { tail -5 "$OUT/bench.log"; exit 1; }
cat "$OUT/bench.json"
