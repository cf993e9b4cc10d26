#!/bin/bash
# Kernel trace of tools/thread_probe.py --alive: the main-thread calls, then
# the helper-thread calls, in one process (tools/thread_trace.py splits them).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/thread_trace; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
(while true; do date +%T >> "$OUT/heartbeat"; sleep 20; done) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
    python3 -u "$R/tools/thread_probe.py" --alive --rounds 1 --steps 3 > "$OUT/probe.txt" 2>&1 || { tail -5 "$OUT/probe.txt"; exit 1; }
grep round "$OUT/probe.txt"
f=$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/thread_trace.py" "$f" > "$OUT/split.txt" && cat "$OUT/split.txt"
