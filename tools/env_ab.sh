#!/bin/bash
# A/B of process-level environment settings (read when the HIP runtime starts,
# so not switchable inside one process), alternating bench processes:
#   tools/env_ab.sh <rounds> NAME=VAR=VAL[,VAR=VAL] ... -- [bench args]
# NAME= alone runs the defaults; a path ending in .so runs that library build.
# One line per run: name, reads/s (M).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
N=$1; shift
specs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do specs+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p "$R/gpurun_out"
for i in $(seq 1 $N); do
  for S in "${specs[@]}"; do
    envs=(SAHARA_ENV_AB=1)
    rest="${S#*=}"
    if [[ "$S" == *.so ]]; then envs+=("SAHARA_HIP_LIB=$R/$S"); rest=""; fi
    if [ -n "$rest" ]; then IFS=',' read -ra kv <<< "$rest"; envs+=("${kv[@]}"); fi
    env "${envs[@]}" timeout -k 10 400 python3 "$R/bench.py" --no-device-resident --no-ingest --no-cpu "$@" \
        > "$R/gpurun_out/env_ab.json" 2> "$R/gpurun_out/env_ab.log" \
      || { echo "FAIL $S"; tail -5 "$R/gpurun_out/env_ab.log"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$R/gpurun_out/env_ab.json')); print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'])" "${S%%=*}"
  done
done
