#!/bin/bash
# A/B in the reference execution mode (every DFS node ranked from the root,
# LF locate), alternating processes:
#   tools/ref_ab.sh <rounds> <spec A> <spec B> ... -- [bench args, e.g. --config c5]
# A spec is a library build (a path ending in .so) or NAME=VAR=VAL[,VAR=VAL]
# (environment settings over the default build). One line per run: spec,
# reads/s, ms per step.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
N=$1; shift
specs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do specs+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p "$R/gpurun_out"
for i in $(seq 1 $N); do
  for S in "${specs[@]}"; do
    envs=(SAHARA_KMER=0)
    if [[ "$S" == *.so ]]; then
      envs+=("SAHARA_HIP_LIB=$R/$S")
    elif [[ "$S" == *=* ]]; then
      IFS=',' read -ra kv <<< "${S#*=}"
      envs+=("${kv[@]}")
    fi
    env "${envs[@]}" timeout -k 10 400 python3 "$R/bench.py" --execution reference --no-cpu --no-e2e \
        --no-verify --no-ingest "$@" > "$R/gpurun_out/ref_ab.json" 2> "$R/gpurun_out/ref_ab.log" \
      || { echo "FAIL $S"; tail -5 "$R/gpurun_out/ref_ab.log"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$R/gpurun_out/ref_ab.json')); print(sys.argv[1], round(d['value']/1e6,2), d['ms_per_step'])" "${S%%=*}"
  done
done
