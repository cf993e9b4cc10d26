# r6 final evidence: the default bench line (C3, with the CPU baseline) and C2 / C5 lines
mkdir -p gpurun_out/r6_final
timeout -k 10 500 python3 bench.py > gpurun_out/r6_final/c3_bench.json 2> gpurun_out/r6_final/c3_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r6_final/c3_bench.json')); r=d['roofline']; print('c3', d['value'], d['ms_per_step'], r['launch_ms'], r.get('traffic'), r.get('valu_issue',{}).get('frac'), r.get('traced'), [k for k in r if k.startswith('stale')])"
timeout -k 10 400 python3 bench.py --config c5 --no-cpu > gpurun_out/r6_final/c5_bench.json 2> gpurun_out/r6_final/c5_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r6_final/c5_bench.json')); print('c5', d['value'], d['config']['device_resident']['reads_per_s'])"
timeout -k 10 300 python3 bench.py --config c2 --no-cpu > gpurun_out/r6_final/c2_bench.json 2> gpurun_out/r6_final/c2_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r6_final/c2_bench.json')); print('c2', d['value'], d['config']['device_resident']['reads_per_s'])"
