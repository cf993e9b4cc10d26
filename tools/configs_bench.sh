#!/bin/bash
# C2 and C5 bench lines (with CPU baseline), plus a serial (unpipelined) C3
# kernel trace for standalone kernel durations. Outputs in $1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
for c in c2 c5; do
  timeout -k 10 400 python3 "$R/bench.py" --config $c "$@" > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.log" || { echo "bench $c failed"; tail -5 "$OUT/bench_$c.log"; exit 1; }
  cat "$OUT/bench_$c.json"
done
mkdir -p "$OUT/serial"
cd /tmp && export TMPDIR=/tmp
SAHARA_PIPELINE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/serial" -o run --output-format csv -- \
   python3 "$R/bench.py" --no-cpu --no-count --no-e2e --steps 2 --warmup 1 > "$OUT/serial/b.json" 2> "$OUT/serial/b.err" || { echo "serial trace failed"; exit 1; }
cd "$R" && python3 tools/timeline.py "$OUT/serial/run_kernel_trace.csv" 5 > "$OUT/serial/timeline.txt"
cat "$OUT/serial/b.json"
