#!/bin/bash
# GPU box: text/packed parity tests, then the headline call and the device-
# resident pass A/B'd over SAHARA_* settings in one process (tools/ab_inproc.py).
# Usage: tools/ab_default.sh <outdir> NAME=VAR=VAL[,..] ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"; cd "$R"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_packed.py tests/test_compact.py -m gpu -x -q \
      --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
timeout -k 10 400 python -u tools/ab_inproc.py --rounds ${ROUNDS:-2} --steps ${STEPS:-5} "$@" > "$OUT/ab_dr.txt" 2>&1 || { tail "$OUT/ab_dr.txt"; exit 1; }
grep -v "^round" "$OUT/ab_dr.txt"
timeout -k 10 400 python -u tools/ab_inproc.py --packed --rounds ${ROUNDS:-2} --steps ${STEPS:-5} "$@" > "$OUT/ab_packed.txt" 2>&1 || { tail "$OUT/ab_packed.txt"; exit 1; }
grep -v "^round" "$OUT/ab_packed.txt"
