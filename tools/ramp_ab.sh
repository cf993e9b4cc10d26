mkdir -p gpurun_out
timeout -k 10 800 python3 tools/ab_inproc.py --rounds 5 --steps 10 --packed base= e2=SAHARA_RAMP_END=1048576:524288 e3=SAHARA_RAMP_END=1048576:524288:262144 > gpurun_out/ramp_packed3.txt 2>&1 || exit 1
tail -4 gpurun_out/ramp_packed3.txt
timeout -k 10 400 python3 tools/ab_inproc.py --rounds 3 --steps 10 --config c5 --packed base= e2=SAHARA_RAMP_END=1048576:524288 > gpurun_out/ramp_packed_c5.txt 2>&1 || exit 1
tail -3 gpurun_out/ramp_packed_c5.txt
