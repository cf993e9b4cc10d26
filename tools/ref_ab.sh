#!/bin/bash
# A/B of two library builds in the reference execution mode (every DFS node
# ranked from the root, LF locate), alternating processes:
#   tools/ref_ab.sh <lib A> <lib B> [rounds] [bench args, e.g. --config c5]
# One line per run: lib, reads/s, kSearchFM lane utilisation.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
A=$1; B=$2; N=${3:-2}
shift 3 2>/dev/null
mkdir -p "$R/gpurun_out"
for i in $(seq 1 $N); do
  for L in "$A" "$B"; do
    SAHARA_KMER=0 SAHARA_HIP_LIB="$R/$L" timeout -k 10 400 python3 "$R/bench.py" --execution reference --no-cpu --no-e2e \
        --no-verify --no-ingest "$@" > "$R/gpurun_out/ref_ab.json" 2> "$R/gpurun_out/ref_ab.log" \
      || { echo "FAIL $L"; tail -5 "$R/gpurun_out/ref_ab.log"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$R/gpurun_out/ref_ab.json')); print(sys.argv[1], round(d['value']/1e6,2), d['ms_per_step'])" "$L"
  done
done
