#!/bin/bash
# Round-3 evidence on the GPU box, outputs in $1 (under gpurun_out/): the
# round evidence (GPU tests, C3 / C2 / C5 / C6 bench lines, C3 kernel trace),
# then --max_hits 1 timed at C3 with one round and two. Stops after a GPU
# fault, abort or time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
cd "$R"
stop() { [ "$1" -ge 124 ] && { echo "stopping after exit $1"; exit "$1"; }; return 0; }
bash tools/round_evidence.sh "$OUT/ev"; rc=$?; stop $rc
[ $rc -ne 0 ] && exit $rc
for e in 2 0; do
  SAHARA_TIMING=1 timeout -k 10 300 python -u tools/pcie_sweep.py --rounds 2 --steps 3 --max-hits 1 --read-errors $e \
      two= one=SAHARA_MAXHITS_ROUNDS=1 > "$OUT/maxhits_e$e.txt" 2>&1; rc=$?; grep -E "mean|exact round" "$OUT/maxhits_e$e.txt" | tail -3; stop $rc
done
