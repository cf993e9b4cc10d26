#!/bin/bash
# A/B of two builds of the library, alternating runs: tools/ab_lib.sh <lib A> <lib B> [rounds] [bench args]
# Prints each run's `value` (the packed call) and its device-resident rate.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
A=$1; B=$2; N=${3:-3}
shift 3 2>/dev/null
mkdir -p "$R/gpurun_out"
for i in $(seq 1 $N); do
  for L in "$A" "$B"; do
    SAHARA_HIP_LIB="$R/$L" timeout -k 10 300 python3 "$R/bench.py" --no-cpu --no-count --no-e2e --no-verify --no-ref-path "$@" > "$R/gpurun_out/ab.json" 2> "$R/gpurun_out/ab.log" || { echo "FAIL $L"; tail -3 "$R/gpurun_out/ab.log"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$R/gpurun_out/ab.json')); dr=d['config'].get('device_resident',{}); print(sys.argv[1], round(d['value']/1e6,1), 'ms', d['ms_per_step'], 'device-resident', round(dr.get('reads_per_s',0)/1e6,1), 'ms', dr.get('ms_per_step'))" "$L"
  done
done
