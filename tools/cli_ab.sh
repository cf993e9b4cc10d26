#!/bin/bash
# sahara search at C3 scale (files as tools/cli_scale.sh makes them), run
# alternately under environment settings: tools/cli_ab.sh <outdir> <rounds> NAME=VAR=VAL[,VAR=VAL] ...
# (NAME= alone: the defaults). Each run's stats block and SAHARA_TIMING lines go to <outdir>/<name>_<round>.txt.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); N=$2; shift 2
W=${SCALE_DIR:-/tmp/sahara_scale}
mkdir -p "$OUT" "$W"
(while true; do date +%T >> "$OUT/heartbeat"; sleep 20; done) & HB=$!
trap 'kill $HB 2>/dev/null; rm -rf "$W"' EXIT
timeout -k 10 300 python3 "$R/tools/make_ref_fasta.py" "$W/ref.fa" 3000000000 24 || { echo "fasta failed"; exit 1; }
timeout -k 10 600 "$R/bin/sahara" index "$W/ref.fa" > "$OUT/index.txt" 2> "$OUT/index.err" || { echo "index failed"; exit 1; }
timeout -k 10 600 "$R/bin/sahara" read_simulator -i "$W/ref.fa" -o "$W/reads.fa" -n 10000000 -l 100 -e 2 > /dev/null 2>&1 || { echo "read_simulator failed"; exit 1; }
for i in $(seq 1 $N); do
  for S in "$@"; do
    name=${S%%=*}; rest=${S#*=}; envs=(SAHARA_TIMING=1)
    if [ -n "$rest" ]; then IFS=',' read -ra kv <<< "$rest"; envs+=("${kv[@]}"); fi
    env "${envs[@]}" timeout -k 10 300 "$R/bin/sahara" search -q "$W/reads.fa" -i "$W/ref.fa.idx" -e 2 -o "$W/out.txt" \
        > "$OUT/${name}_$i.txt" 2>&1 || { echo "search $name failed"; tail -5 "$OUT/${name}_$i.txt"; exit 1; }
    sleep 5
    echo "$name $i: $(grep -E 'total time' "$OUT/${name}_$i.txt" | tr -s ' ') | $(grep -E 'ld queries|ld index|index load' "$OUT/${name}_$i.txt" | tr -s ' ' | tr '\n' ' ')"
    grep -h "\[sahara\] context" "$OUT/${name}_$i.txt"
  done
done
md5sum < "$W/out.txt" > "$OUT/out_md5.txt"
