#!/bin/bash
# Kernel-trace summaries of the headline call for this tree's library and
# another build (SAHARA_HIP_LIB), side by side: tools/kstats_ab.sh <outdir> <other lib> [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); OTHER=$(realpath "$2"); shift 2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for side in new old; do
  if [ $side == old ]; then export SAHARA_HIP_LIB=$OTHER; else unset SAHARA_HIP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$side" -o run --output-format csv -- \
      python3 "$R/bench.py" --no-cpu --no-count --no-e2e --no-verify --no-ref-path --no-device-resident --no-ingest \
      --steps 3 --warmup 1 "$@" > "$OUT/$side.json" 2> "$OUT/$side.err" || { echo "$side failed"; tail -5 "$OUT/$side.err"; exit 1; }
  f=$(find "$OUT/$side" -name "*kernel_stats.csv" | head -1)
  echo "== $side $(python3 -c "import json;d=json.load(open('$OUT/$side.json'));print(round(d['value']/1e6,1),'M', d['ms_per_step'],'ms')")"
  python3 "$R/tools/kstats.py" "$f" | sort -k4 -nr | head -12
done
