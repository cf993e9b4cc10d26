#!/bin/bash
# Round evidence on the GPU box, outputs in $1 (under gpurun_out/): GPU test
# log, default C3 bench line (CPU baseline included), C2 / C5 / C6 bench
# lines, and a rocprofv3 kernel trace + stats of the C3 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT/trace"
cd "$R"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
fi
timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 > "$OUT/c3_bench.json" 2> "$OUT/c3_bench.log" || { tail -20 "$OUT/c3_bench.log"; exit 1; }
for c in c2 c5 c6; do
  # C2's step is ~1 ms: time more of them so the line is not one launch's jitter
  steps=5; [ $c = c2 ] && steps=20
  timeout -k 10 600 python -u bench.py --config $c --steps $steps > "$OUT/${c}_bench.json" 2> "$OUT/${c}_bench.log" || { echo "bench $c failed"; tail -10 "$OUT/${c}_bench.log"; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --no-device-resident --no-ingest --steps 5 > "$OUT/trace/b.json" 2> "$OUT/trace.err" || { echo "trace failed"; exit 1; }
cd "$R" && python3 tools/timeline.py "$OUT/trace/run_kernel_trace.csv" 5 > "$OUT/c3_timeline.txt" && cp "$OUT/trace/run_kernel_stats.csv" "$OUT/c3_kernel_stats.csv" && rm -f "$OUT/trace/run_kernel_trace.csv"
for f in "$OUT"/*_bench.json; do python3 -c "import json,sys; d=json.load(open('$f')); c=d['config']; print('$f', d['value'], d['ms_per_step'], (d.get('cpu_baseline') or {}).get('parity_on_sample'), c.get('origin_recall'), c.get('sa_probe_ok'), (c.get('pcie_inclusive') or {}).get('reads_per_s'))"; done
