#!/bin/bash
# The bench line and the two-context thread probe under GPU_MAX_HW_QUEUES=4
# (the box's default) and 8, one process each, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
OUT=gpurun_out/hwq_ab; mkdir -p $OUT
for q in 8 4; do
  echo "## probe hwq$q" | tee -a $OUT/all.txt
  GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python3 -u tools/thread_probe.py --alive --rounds 1 > $OUT/probe_$q.txt 2>&1 \
    || { tail -5 $OUT/probe_$q.txt; exit 1; }
  grep round $OUT/probe_$q.txt | tee -a $OUT/all.txt
done
for i in 1 2; do
  for q in 8 4; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 -u bench.py --no-cpu > $OUT/bench_${q}_$i.txt 2>&1 || { tail -5 $OUT/bench_${q}_$i.txt; exit 1; }
    echo "bench hwq$q $i: $(tail -1 $OUT/bench_${q}_$i.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), "M", d["ms_per_step"], "ms launch", d["roofline"]["launch_ms"])')" | tee -a $OUT/all.txt
  done
done
