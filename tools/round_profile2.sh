#!/bin/bash
# Profile evidence for one build on the GPU box, outputs in $1 (under gpurun_out/):
#   traffic/   kernel trace + FETCH_SIZE (+ calibration) of the default bench -> traffic.json
#   pmc/       SQ counter passes of the search kernels -> pmc.json (roofline.valu_issue)
#   ref/       kernel trace + FETCH_SIZE of the reference execution model -> traffic_ref.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
bash "$R/tools/traffic.sh" "$OUT/traffic" "$@" || exit 1
python3 "$R/tools/traffic_summary.py" "$OUT/traffic" "$OUT/traffic.json" "$OUT/traffic.txt" || exit 1
cp "$OUT/traffic/trace/run_kernel_stats.csv" "$OUT/kernel_stats.csv"
python3 "$R/tools/timeline.py" "$OUT/traffic/trace/run_kernel_trace.csv" 5 > "$OUT/timeline.txt"
rm -f "$OUT/traffic/trace/run_kernel_trace.csv"
bash "$R/tools/pmc_text.sh" "$OUT/pmc" "$@" || exit 1
bash "$R/tools/traffic_ref.sh" "$OUT/ref" "$@" || exit 1
cp "$OUT/ref/trace/run_kernel_stats.csv" "$OUT/kernel_stats_ref.csv"
echo done
