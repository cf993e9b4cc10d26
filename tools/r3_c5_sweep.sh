#!/bin/bash
# C5 (k = 3, 250 bp) patterns per batch: one 2M-pattern batch (default) against
# 1M / 0.5M / 0.25M, so that neighbouring batches' seeds, FM, locate and sort
# overlap the text phase; two alternating rounds. Lines in $1/c5_b<batch>_<round>.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
cd "$R"
for round in 1 2; do
  for b in default 1000000 500000 250000; do
    if [ $b = default ]; then unset SAHARA_BATCH; else export SAHARA_BATCH=$b; fi
    timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu --no-e2e --no-ref-path --no-verify "$@" \
      > "$OUT/c5_b${b}_$round.json" 2> "$OUT/c5_b${b}_$round.log" || { echo "c5 $b failed"; tail -5 "$OUT/c5_b${b}_$round.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c5_b${b}_$round.json')); c=d['config']; print('$b', $round, d['value'], d['ms_per_step'], c.get('text_lane_util'), c.get('text_ms'), c.get('text_launches_per_step'))"
  done
done
