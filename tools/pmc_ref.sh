#!/bin/bash
# SQ counters of kSearchFM in the reference execution mode (every DFS node
# ranked from the root; `bench.py --execution reference`), two passes, per
# launch into <outdir>/pmc.json (tools/pmc_json.py).
# Usage (on the GPU box): tools/pmc_ref.sh <outdir> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
SAHARA_KMER=0 KREGEX=kSearchFM bash "$R/tools/profile.sh" "$OUT" \
    "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES" \
    "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
    -- --execution reference --no-verify --no-e2e --no-ingest "$@" || exit 1
python3 "$R/tools/pmc_json.py" "$OUT" "$OUT/pmc.json" "$OUT/pmc.txt"
