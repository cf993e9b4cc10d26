# Carried nodes (SAHARA_CARRY_BELOW): the GPU suite with carrying on, then
# in-process A/Bs, device-resident and the packed call (tools/ab_inproc.py)
mkdir -p gpurun_out
SAHARA_CARRY_BELOW=${CARRY_TEST:-32} timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/carry_pytest.log 2>&1 || { tail -30 gpurun_out/carry_pytest.log; exit 1; }
tail -2 gpurun_out/carry_pytest.log
timeout -k 10 500 python3 tools/ab_inproc.py --rounds 3 --steps 10 --count off= c16=SAHARA_CARRY_BELOW=16 c32=SAHARA_CARRY_BELOW=32 c48=SAHARA_CARRY_BELOW=48 c64=SAHARA_CARRY_BELOW=64 > gpurun_out/carry_dr.txt 2>&1 || exit 1
timeout -k 10 500 python3 tools/ab_inproc.py --rounds 3 --steps 10 --packed off= c16=SAHARA_CARRY_BELOW=16 c32=SAHARA_CARRY_BELOW=32 c48=SAHARA_CARRY_BELOW=48 c64=SAHARA_CARRY_BELOW=64 > gpurun_out/carry_packed.txt 2>&1 || exit 1
tail -6 gpurun_out/carry_dr.txt; tail -6 gpurun_out/carry_packed.txt
