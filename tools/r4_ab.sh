#!/bin/bash
# GPU box: the parity tests of the text phase and the packed call, then an
# in-process A/B of the headline call over SAHARA_* settings. Outputs under $1.
# Usage: tools/r4_ab.sh <outdir> [--config c3] NAME=VAR=VAL ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
cd "$R"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_packed.py tests/test_compact.py \
      tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
      || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
timeout -k 10 900 python -u tools/ab_inproc.py --packed --rounds ${ROUNDS:-3} --steps ${STEPS:-10} "$@" > "$OUT/ab.txt" 2> "$OUT/ab.err" \
    || { tail -20 "$OUT/ab.err"; exit 1; }
cat "$OUT/ab.txt"
