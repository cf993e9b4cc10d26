#!/bin/bash
# HEAD check on the GPU box: GPU tests, then the default bench line (with CPU baseline).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log || { tail -20 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.json
