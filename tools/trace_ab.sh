#!/bin/bash
# Kernel-trace timelines of the last bench step under environment variants:
# tools/trace_ab.sh "VAR=val ..." "..." [-- bench args]  -> gpurun_out/tl_<i>.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out"
CFGS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do CFGS+=("$1"); shift; done
[ "$1" = "--" ] && shift
i=0
for cfg in "${CFGS[@]}"; do
  i=$((i+1))
  D="$R/gpurun_out/tr$i"
  mkdir -p "$D"
  (cd /tmp && export TMPDIR=/tmp && env $cfg timeout -k 10 300 rocprofv3 --kernel-trace -d "$D" -o run --output-format csv -- \
      python3 "$R/bench.py" --no-cpu --no-count --no-e2e --no-verify --no-ref-path --steps 1 --warmup 1 "$@" > "$D/b.json" 2> "$D/b.log") || { echo "FAIL $cfg"; exit 1; }
  f=$(find "$D" -name "run_kernel_trace.csv" | head -1)
  python3 "$R/tools/timeline.py" "$f" 5 > "$R/gpurun_out/tl_$i.txt"
  echo "== $cfg: $(python3 -c "import json;d=json.load(open('$D/b.json'));print(round(d['value']/1e6,1),'M reads/s',d['ms_per_step'],'ms')")"
  rm -rf "$D"
done
