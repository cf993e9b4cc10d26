#!/bin/bash
# tools/thread_probe.py --alive under HIP runtime settings, one process each:
# is the helper-thread slowdown a loss of stream concurrency in the runtime?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
OUT=gpurun_out/thread_env; mkdir -p $OUT
run() {
  name=$1; shift
  echo "## $name" | tee -a $OUT/all.txt
  env SAHARA_TIMING=1 "$@" timeout -k 10 240 python3 -u tools/thread_probe.py --alive --rounds 1 > $OUT/$name.txt 2>&1 \
    || { tail -5 $OUT/$name.txt; exit 1; }
  grep -E "round|\(" $OUT/$name.txt | tee -a $OUT/all.txt
}
run hwq8 GPU_MAX_HW_QUEUES=8
run hwq4 GPU_MAX_HW_QUEUES=4
run nodirect GPU_MAX_HW_QUEUES=8 AMD_DIRECT_DISPATCH=0
