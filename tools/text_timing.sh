# GPU box: serial / pipelined timing per library (no count mode): tools/text_timing.sh lib...
set -o pipefail
cd $GRAFT_REPO_ROOT
for L in "$@"; do
  n=$(basename $L .so)
  SAHARA_HIP_LIB=$PWD/$L timeout -k 10 200 python -u tools/ab_inproc.py --rounds 1 --steps 5 serial=SAHARA_PIPELINE=0 pipe=SAHARA_PIPELINE=1 > gpurun_out/tim_$n.txt 2>&1 || { tail gpurun_out/tim_$n.txt; exit 1; }
  grep "^round" gpurun_out/tim_$n.txt | sed "s/^/$n /"
done
