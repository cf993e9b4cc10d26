# r6: GPU suite, CLI at C3 scale, the default bench line
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash tools/cli_scale.sh gpurun_out/r6_cli_scale2 || exit 1
tail -12 gpurun_out/r6_cli_scale2/search.txt; grep sahara gpurun_out/r6_cli_scale2/search.err | head -5; cat gpurun_out/r6_cli_scale2/out_md5.txt
timeout -k 10 400 python3 bench.py > gpurun_out/b.json 2> gpurun_out/b.log || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/b.json')); print(d['value'], d['ms_per_step'], d['config']['device_resident']['reads_per_s'], d['cpu_baseline'])"
