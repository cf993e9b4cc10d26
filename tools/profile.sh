#!/bin/bash
# PMC passes on the search kernel, one rocprofv3 run per counter group (the
# microarch guide's rule: counters in their own runs, kernel-trace only).
# Usage: tools_profile.sh <outdir> "<group1>" "<group2>" ... -- [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
groups=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do groups+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-kSearch}" -d "$OUT/pmc$i" -o run \
      --output-format csv -- python3 "$R/bench.py" --no-cpu --no-count --warmup 0 --steps 1 "$@" \
      > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.err" || { echo "pass $i failed rc=$?"; exit 1; }
done
