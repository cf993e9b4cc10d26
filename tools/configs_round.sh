#!/bin/bash
# Bench lines of the other BASELINE configs at this build (C2, C5), without
# the CPU baseline: tools/configs_round.sh <outdir> [configs...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
for c in ${@:-c2 c5}; do
  timeout -k 10 500 python3 "$R/bench.py" --config $c --no-cpu --no-ingest > "$OUT/$c.json" 2> "$OUT/$c.err" \
      || { echo "$c failed"; tail -5 "$OUT/$c.err"; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('$OUT/$c.json')); dr=d['config'].get('device_resident',{})
print('$c', round(d['value']/1e6,1), 'M packed;', round(dr.get('reads_per_s',0)/1e6,1), 'M device-resident; ratio', dr.get('timed_call_over_device_resident'))"
done
