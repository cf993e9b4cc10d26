#!/bin/bash
# PCIe-inclusive path probe on the GPU box, outputs in $1 (under gpurun_out/):
# a knob sweep of sahara_gpu_search_reads_compact at C3 (settings as
# tools/pcie_sweep.py takes them) ending with two calls' host marks, then a
# rocprofv3 kernel + memory-copy trace of three default calls and its device
# timeline (tools/pcie_timeline2.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT/trace"
cd "$R"
timeout -k 10 500 python -u tools/pcie_sweep.py --rounds 2 --steps 10 --marks 2 "$@" > "$OUT/sweep.txt" 2>&1 || { tail -20 "$OUT/sweep.txt"; exit 1; }
grep -E "mean|compact call" "$OUT/sweep.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/tools/pcie_sweep.py" --rounds 1 --steps 3 base= > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$OUT/trace.log"; exit 1; }
cd "$R" && python3 tools/pcie_timeline2.py "$OUT/trace" > "$OUT/timeline.txt"; head -60 "$OUT/timeline.txt"
find "$OUT/trace" -name "*_trace.csv" -delete
