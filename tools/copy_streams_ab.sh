#!/bin/bash
# SAHARA_COPY_STREAMS=shared (4 streams per context) against own copy
# streams (6): the thread probe (a second context in the process) and the
# bench line, alternating, one process each.
# (SAHARA_COPY_STREAMS lived in capi.cpp newCtx for the r6 experiment and was removed
# again; profiles/r06_copy_streams_ab.txt holds the results)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
OUT=gpurun_out/copy_streams; mkdir -p $OUT
for v in high low own; do
  echo "## probe $v" | tee -a $OUT/all.txt
  SAHARA_COPY_STREAMS=$v timeout -k 10 240 python3 -u tools/thread_probe.py --alive --rounds 1 > $OUT/probe_$v.txt 2>&1 \
    || { tail -5 $OUT/probe_$v.txt; exit 1; }
  grep round $OUT/probe_$v.txt | tee -a $OUT/all.txt
done
for i in 1 2; do
  for v in high low own; do
    SAHARA_COPY_STREAMS=$v timeout -k 10 300 python3 -u bench.py > $OUT/bench_${v}_$i.txt 2>&1 || { tail -5 $OUT/bench_${v}_$i.txt; exit 1; }
    echo "bench $v $i: $(tail -1 $OUT/bench_${v}_$i.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), "M", d["ms_per_step"], "ms")')" | tee -a $OUT/all.txt
  done
done
