mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 500 python3 bench.py > gpurun_out/b.json 2> gpurun_out/b.log || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/b.json')); print(d['value'], d['ms_per_step'], d['config']['device_resident']['reads_per_s'], d['config']['text_launches_per_step'], d['cpu_baseline']['value'])"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
