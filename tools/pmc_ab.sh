#!/bin/bash
# SQ counters of kSearchText for two builds of the same workload (this tree
# and another checkout of the repo, e.g. a worktree of an earlier commit), one
# rocprofv3 --pmc pass per build and counter group, summarised per launch
# (tools/pmc_json.py). Usage (GPU box): tools/pmc_ab.sh <outdir> <other repo dir> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); OTHER=$(realpath "$2"); shift 2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
G1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES"
G2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM"
for side in new old; do
  B=$R; [ $side == old ] && B=$OTHER
  i=0
  for grp in "$G1" "$G2"; do
    i=$((i+1))
    mkdir -p "$OUT/$side"
    timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex kSearchText -d "$OUT/$side/pmc$i" -o run \
        --output-format csv -- python3 "$B/bench.py" --no-device-resident --no-ingest --warmup 0 --steps 1 "$@" \
        > "$OUT/$side/pmc$i.json" 2> "$OUT/$side/pmc$i.err" || { echo "$side pass $i failed"; exit 1; }
  done
  python3 "$R/tools/pmc_json.py" "$OUT/$side" "$OUT/$side/pmc.json" "$OUT/$side/pmc.txt" || exit 1
done
