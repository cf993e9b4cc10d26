# GPU box: count-mode text-kernel cycle split (serial, pipelined) per library: tools/text_cycles.sh lib...
set -o pipefail
cd $GRAFT_REPO_ROOT
for L in "$@"; do
  n=$(basename $L .so)
  SAHARA_HIP_LIB=$PWD/$L timeout -k 10 240 python -u tools/ab_inproc.py --rounds 1 --steps 5 --count serial=SAHARA_PIPELINE=0 pipe=SAHARA_PIPELINE=1 > gpurun_out/cnt_$n.txt 2>&1 || { tail gpurun_out/cnt_$n.txt; exit 1; }
done
