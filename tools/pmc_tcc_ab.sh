#!/bin/bash
# L2 (TCC) and SQ counters of kSearchText for this tree's library and another
# build (e.g. the previous round's), serial passes (SAHARA_PIPELINE=0) so each
# launch runs alone: tools/pmc_tcc_ab.sh <outdir> <other libsahara_hip.so> [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); OTHER=$(realpath "$2"); shift 2
export SAHARA_PIPELINE=0 KREGEX=kSearchText
for side in new old; do
  if [ $side == old ]; then export SAHARA_HIP_LIB=$OTHER; else unset SAHARA_HIP_LIB; fi
  bash "$R/tools/profile.sh" "$OUT/$side" \
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
      "TCC_ATOMIC_sum TCC_REQ_sum TCC_READ_sum TCC_WRITE_sum" \
      "SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VALU" \
      -- --no-device-resident --no-ingest "$@" || exit 1
  python3 "$R/tools/pmc_json.py" "$OUT/$side" "$OUT/$side/pmc.json" "$OUT/$side/pmc.txt" || exit 1
done
