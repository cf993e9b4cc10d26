# Batch-size A/B, device-resident then the packed call (tools/ab_inproc.py)
mkdir -p gpurun_out
timeout -k 10 500 python3 tools/ab_inproc.py --rounds 3 --steps 10 b4m= b2m=SAHARA_BATCH=2097152 b1m=SAHARA_BATCH=1048576 > gpurun_out/batch_dr.txt 2>&1 || exit 1
timeout -k 10 500 python3 tools/ab_inproc.py --rounds 3 --steps 10 --packed b2m= b4m=SAHARA_BATCH=4194304 ramp=SAHARA_BATCH=4194304,SAHARA_RAMP=1048576:2097152,SAHARA_RAMP_END=2097152:1048576 b3m=SAHARA_BATCH=3145728 > gpurun_out/batch_packed.txt 2>&1 || exit 1
