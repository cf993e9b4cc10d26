#!/bin/bash
# Round evidence at one build (GPU box): the default bench traced by rocprofv3
# (tools/bench_profiled.sh: roofline.launch_ms against the trace), the traffic
# and SQ counter passes (tools/round_profile2.sh). Outputs under $1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
bash "$R/tools/round_profile2.sh" "$OUT/prof" "$@" || exit 1
bash "$R/tools/bench_profiled.sh" "$OUT/bench_traced" --no-cpu "$@" || exit 1
echo evidence done
