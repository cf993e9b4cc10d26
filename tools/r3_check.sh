#!/bin/bash
# HEAD check on the GPU box, outputs in $1 (under gpurun_out/): GPU tests,
# the C3 bench line (20 timed steps, CPU baseline included), and a rocprofv3
# kernel trace + stats of the same bench command (per-kernel averages that
# the bench line's roofline.launch_ms must agree with).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT/trace"
cd "$R"
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
fi
timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 "$@" > "$OUT/bench.json" 2> "$OUT/bench.log" || { tail -20 "$OUT/bench.log"; exit 1; }
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --no-cpu --no-count --no-verify --no-e2e --no-ref-path --steps 20 --warmup 2 "$@" > "$OUT/trace/b.json" 2> "$OUT/trace.err" || { echo "trace failed"; tail -5 "$OUT/trace.err"; exit 1; }
cd "$R" && python3 tools/timeline.py "$OUT/trace/run_kernel_trace.csv" 5 > "$OUT/timeline.txt"; python3 tools/timeline.py "$OUT/trace/run_kernel_trace.csv" 5 gap > "$OUT/timeline_gap.txt"; cp "$OUT/trace/run_kernel_stats.csv" "$OUT/kernel_stats.csv" && rm -f "$OUT/trace/run_kernel_trace.csv"
python3 tools/kstats.py "$OUT/kernel_stats.csv" > "$OUT/kstats.txt"; head -30 "$OUT/kstats.txt"
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); c = d["config"]; r = d["roofline"] or {}
print("value", d["value"], "ms/step", d["ms_per_step"], "kernel", r.get("kernel"), "launch_ms", r.get("launch_ms"), "frac", r.get("frac"))
print("pcie", {k: (c.get(k) or {}).get("reads_per_s") for k in ("pcie_inclusive", "pcie_inclusive_full_records", "pcie_inclusive_patterns")},
      "same", (c.get("pcie_inclusive") or {}).get("same_hits"), "cpu", (d.get("cpu_baseline") or {}).get("value"),
      "recall", c.get("origin_recall"), "sa", c.get("sa_probe_ok"))
PY
