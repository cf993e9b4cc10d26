#!/bin/bash
# HBM traffic (FETCH_SIZE) per kernel + kernel-trace stats for the default bench,
# plus a FETCH_SIZE calibration on random 64-B line gathers (tools/gather_bench).
# Usage (on the GPU box): tools/traffic.sh <outdir> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --no-device-resident --no-ingest "$@" > "$OUT/trace.json" 2> "$OUT/trace.err" || { echo "trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "kSearch|kSeed|kResolve|kLocate" -d "$OUT/pmc_fetch" -o run \
    --output-format csv -- python3 "$R/bench.py" --no-device-resident --no-ingest "$@" > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err" || { echo "pmc failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "kGroup" -d "$OUT/calib" -o run \
    --output-format csv -- "$R/tools/gather_bench" > "$OUT/calib.txt" 2> "$OUT/calib.err" || { echo "calib failed"; exit 1; }
echo done
