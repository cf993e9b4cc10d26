#!/bin/bash
# GPU box: device timeline of the bench's timed call (packed reads in, hits
# out): a rocprofv3 kernel + memory-copy trace of three calls
# (bench.py --no-device-resident) and the last call's timeline
# (tools/pcie_timeline2.py). Outputs under $1. Extra args go to bench.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT/trace"
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --no-device-resident --no-ingest --warmup 2 --steps 3 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "trace failed"; tail -5 "$OUT/bench.err"; exit 1; }
cd "$R" && python3 tools/pcie_timeline2.py "$OUT/trace" > "$OUT/timeline.txt" && python3 tools/pcie_timeline2.py "$OUT/trace" --all > "$OUT/timeline_all.txt"
tail -30 "$OUT/timeline.txt"
find "$OUT/trace" -name "*_trace.csv" -delete
