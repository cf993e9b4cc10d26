#!/bin/bash
# A/B of environment settings, alternating runs of the default bench line:
# tools/ab_env.sh <rounds> "VAR=val ..." "..." [-- bench args]   ("" = defaults)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
N=$1; shift
CFGS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do CFGS+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p "$R/gpurun_out"
for i in $(seq 1 "$N"); do
  for cfg in "${CFGS[@]}"; do
    env $cfg timeout -k 10 300 python3 "$R/bench.py" --no-cpu --no-count --no-e2e --no-verify --no-ref-path "$@" \
        > "$R/gpurun_out/ab.json" 2> "$R/gpurun_out/ab.log" || { echo "FAIL $cfg"; tail -3 "$R/gpurun_out/ab.log"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$R/gpurun_out/ab.json')); c=d['config']; print(repr(sys.argv[1]), round(d['value']/1e6,1), d['ms_per_step'], {k: c.get(k) for k in ('text_ms','search_ms','seed_ms','locate_ms','sort_ms')})" "$cfg"
  done
done
