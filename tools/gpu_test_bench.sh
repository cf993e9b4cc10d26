mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/b.json 2> gpurun_out/b.log || exit $?
python -c "import json; d=json.load(open('gpurun_out/b.json')); c=d['config']; print(d['value'], {k: c[k] for k in ('text_ms','search_ms','text_nodes_per_read','text_lane_util','text_cycle_split','text_compare_steps_per_read','text_refill_frac','text_steps_per_read')})"
