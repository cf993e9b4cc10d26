# r6: GPU suite, index load phases (tools/load_probe.py), dry-steps A/B, C2, CLI at C3 scale
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python3 tools/load_probe.py --config c3 --reads 100000 > gpurun_out/load_probe.txt 2>&1 || { tail -5 gpurun_out/load_probe.txt; exit 1; }
grep -E "load|save|build" gpurun_out/load_probe.txt
bash tools/cli_scale.sh gpurun_out/r6_cli_scale || exit 1
tail -12 gpurun_out/r6_cli_scale/search.txt; grep sahara gpurun_out/r6_cli_scale/search.err | head -5
timeout -k 10 500 python3 tools/ab_inproc.py --rounds 3 --steps 10 --count d0= d4=SAHARA_TEXT_STEPS_DRY=4 d8=SAHARA_TEXT_STEPS_DRY=8 d16=SAHARA_TEXT_STEPS_DRY=16 > gpurun_out/dry_dr.txt 2>&1 || exit 1
timeout -k 10 500 python3 tools/ab_inproc.py --rounds 3 --steps 10 --packed d0= d4=SAHARA_TEXT_STEPS_DRY=4 d8=SAHARA_TEXT_STEPS_DRY=8 d16=SAHARA_TEXT_STEPS_DRY=16 > gpurun_out/dry_packed.txt 2>&1 || exit 1
tail -5 gpurun_out/dry_dr.txt; tail -5 gpurun_out/dry_packed.txt
timeout -k 10 300 python3 bench.py --config c2 --no-cpu > gpurun_out/c2.json 2> gpurun_out/c2.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/c2.json')); print('c2', d['value'], d['ms_per_step'], d['config']['device_resident']['reads_per_s'])"
