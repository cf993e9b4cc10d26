#!/bin/bash
# SQ counters of the search kernels on the default bench, two passes of at
# most 8 SQ counters each (one rocprofv3 run per pass, kernel dispatches
# only), summarised per launch into <outdir>/pmc.json by tools/pmc_json.py.
# Usage (on the GPU box): tools/pmc_text.sh <outdir> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
KREGEX=${KREGEX:-kSearch} bash "$R/tools/profile.sh" "$OUT" \
    "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES" \
    "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
    -- --no-device-resident --no-ingest "$@" || exit 1
python3 "$R/tools/pmc_json.py" "$OUT" "$OUT/pmc.json" "$OUT/pmc.txt"
