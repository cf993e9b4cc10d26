# GPU box: serial / pipelined timing per library (no count mode): tools/text_timing.sh lib...
set -o pipefail
cd $GRAFT_REPO_ROOT
for L in "$@"; do
  n=$(echo "$L" | tr '/' '_' | sed 's/\.so$//')
  f=gpurun_out/tim_$n.txt
  SAHARA_HIP_LIB=$PWD/$L timeout -k 10 200 python -u tools/ab_inproc.py --rounds 1 --steps 5 ${TIMING_SETTINGS:-serial=SAHARA_PIPELINE=0 pipe=SAHARA_PIPELINE=1} > $f 2>&1 || { tail $f; exit 1; }
  grep -h "^round" $f | sed "s#^#$n #"
done
