#!/bin/bash
# One iteration on the GPU box: GPU tests, default bench, pipelined kernel
# trace (timeline of the last step) and a per-kernel summary.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && bash tools/gpu_test_bench.sh || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/b.json')); c=d['config']; print({k: c[k] for k in ('locate_ms','sort_ms','seed_ms','search_ms','text_ms')}, d['ms_per_step'])"
mkdir -p gpurun_out/kp
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kp" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --no-count --steps 2 --warmup 1 "$@" > "$R/gpurun_out/kp/b.json" 2>&1 || exit $?
cd "$R" && python3 tools/timeline.py gpurun_out/kp/run_kernel_trace.csv 5 > gpurun_out/kp/timeline.txt
python3 tools/kstats.py gpurun_out/kp/run_kernel_stats.csv | grep -v "kScatter\|kBwt\|kHeads\|kInit\|kSampled\|kPair\|kReverse\|kLines\|kPack\|kKmer\|kSamples\|onesweep\|lookback"
