#!/bin/bash
# Kernel trace + FETCH_SIZE of the reference's execution model (kSearchFM
# ranking every node from the root, kLocate's LF walk to the samples):
# `bench.py --execution reference`, two timed steps, no warmup, so that
# dispatches / 2 = launches per step. Summary: <outdir>/traffic_ref.json.
# Usage (on the GPU box): tools/traffic_ref.sh <outdir> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--execution reference --no-cpu --no-verify --no-e2e --no-ingest --warmup 0 --steps 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" $ARGS "$@" > "$OUT/trace.json" 2> "$OUT/trace.err" || { echo "trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "kSearch|kSeed|kLocate" -d "$OUT/pmc_fetch" -o run \
    --output-format csv -- python3 "$R/bench.py" $ARGS "$@" > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err" || { echo "pmc failed"; exit 1; }
STEPS=2 python3 "$R/tools/traffic_summary.py" "$OUT" "$OUT/traffic_ref.json" "$OUT/traffic_ref.txt"
rm -f "$OUT/trace/run_kernel_trace.csv"
