#!/bin/bash
# Kernel-trace summaries (search kernels) of the headline call per library
# build: tools/kstats_libs.sh <outdir> lib... (paths relative to the repo)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  n=$(echo "$L" | tr '/' '_' | sed 's/\.so$//')
  export SAHARA_HIP_LIB=$R/$L
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$n" -o run --output-format csv -- \
      python3 "$R/bench.py" --no-cpu --no-count --no-e2e --no-verify --no-ref-path --no-device-resident --no-ingest \
      --steps 3 --warmup 1 > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  f=$(find "$OUT/$n" -name "*kernel_stats.csv" | head -1)
  echo "== $n $(python3 -c "import json;d=json.load(open('$OUT/$n.json'));print(round(d['value']/1e6,1),'M', d['ms_per_step'],'ms')")"
  python3 "$R/tools/kstats.py" "$f" | grep -E "kSearch|kSeed|kLocate|kSort|kPack" 
done
