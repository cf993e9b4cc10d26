#!/bin/bash
# The drop-in at full C3 scale through bin/sahara:
#   sahara index          on a 3 Gbp, 24-record FASTA (tools/make_ref_fasta.py)
#   sahara read_simulator 10M x 100 bp reads, -e 2, from that FASTA
#   sahara search         -e 2 of those reads against the .idx
# Each step's stdout (stats block) goes to <outdir>; the big files live in
# $SCALE_DIR (default /tmp/sahara_scale) and are removed at the end.
# Usage (on the GPU box): tools/cli_scale.sh <outdir> [reads]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); N=${2:-10000000}
W=${SCALE_DIR:-/tmp/sahara_scale}
mkdir -p "$OUT" "$W"
(while true; do date +%T >> "$OUT/heartbeat"; sleep 20; done) & HB=$!
trap 'kill $HB 2>/dev/null; rm -rf "$W"' EXIT
df -h /tmp > "$OUT/df.txt"; nproc >> "$OUT/df.txt"; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS" >> "$OUT/df.txt"
step() {  # step <name> <command...>: wall time into times.txt
  local name=$1; shift
  local t0=$(date +%s%N)
  "$@" || return 1
  echo "$name $(( ($(date +%s%N) - t0) / 1000000 )) ms" >> "$OUT/times.txt"
}
step make_ref_fasta timeout -k 10 300 python3 "$R/tools/make_ref_fasta.py" "$W/ref.fa" 3000000000 24 || { echo "fasta failed"; exit 1; }
step index timeout -k 10 600 "$R/bin/sahara" index "$W/ref.fa" > "$OUT/index.txt" 2> "$OUT/index.err" || { echo "index failed"; tail -5 "$OUT/index.err"; exit 1; }
step read_simulator timeout -k 10 600 "$R/bin/sahara" read_simulator -i "$W/ref.fa" -o "$W/reads.fa" -n "$N" -l 100 -e 2 \
    > "$OUT/read_simulator.txt" 2> "$OUT/read_simulator.err" || { echo "read_simulator failed"; tail -5 "$OUT/read_simulator.err"; exit 1; }
step search env SAHARA_TIMING=${SEARCH_TIMING:-1} timeout -k 10 600 "$R/bin/sahara" search -q "$W/reads.fa" -i "$W/ref.fa.idx" -e 2 -o "$W/out.txt" \
    > "$OUT/search.txt" 2> "$OUT/search.err" || { echo "search failed"; tail -5 "$OUT/search.err"; exit 1; }
md5sum < "$W/out.txt" > "$OUT/out_md5.txt"
# (optional) another build's CLI on the same files: its stats and output bytes
if [ -n "$CLI_B" ]; then
  step search_b env SAHARA_TIMING=1 timeout -k 10 600 "$R/$CLI_B" search -q "$W/reads.fa" -i "$W/ref.fa.idx" -e 2 -o "$W/out_b.txt" \
      > "$OUT/search_b.txt" 2> "$OUT/search_b.err" || { echo "search_b failed"; tail -5 "$OUT/search_b.err"; exit 1; }
  md5sum < "$W/out_b.txt" >> "$OUT/out_md5.txt"
  step search_again env SAHARA_TIMING=1 timeout -k 10 600 "$R/bin/sahara" search -q "$W/reads.fa" -i "$W/ref.fa.idx" -e 2 -o "$W/out.txt" \
      > "$OUT/search_again.txt" 2> "$OUT/search_again.err" || { echo "search again failed"; exit 1; }
fi
ls -la "$W" > "$OUT/files.txt"
head -3 "$W/out.txt" > "$OUT/out_head.txt"; wc -l < "$W/out.txt" >> "$OUT/out_head.txt"
echo done
