#!/bin/bash
# Round-4 evidence, part 1 (GPU box): GPU tests, then the kernel trace,
# FETCH_SIZE and SQ counter passes of the default bench's timed call
# (tools/round_profile2.sh). Outputs under $1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
grep "contexts\] before" "$OUT/pytest_gpu.log" || true
bash "$R/tools/round_profile2.sh" "$OUT/prof" "$@" || exit 1
cat "$OUT/prof/traffic.txt" "$OUT/prof/pmc/pmc.txt"
