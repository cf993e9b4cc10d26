#!/bin/bash
# Bench sweep over environment knobs: tools/sweep.sh "VAR=val VAR2=val" "..." ...
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu $BENCH_ARGS > gpurun_out/sweep.json 2> gpurun_out/sweep.log || { echo "FAIL $cfg"; tail -3 gpurun_out/sweep.log; exit 1; }
  python -c "
import json,sys; d=json.load(open('gpurun_out/sweep.json')); c=d['config']
print(sys.argv[1], round(d['value']/1e6,1), 'pcie', c.get('pcie_inclusive',{}).get('reads_per_s'), 'ref', c.get('reference_path',{}).get('reads_per_s'), 'M reads/s', d['ms_per_step'], 'ms', 'sort', c.get('sort_ms'), 'loc', c.get('locate_ms'), 'seed', c.get('seed_ms'), 'fm', c.get('search_ms'), 'text', c.get('text_ms'), 'grids', c.get('search_grid'), c.get('text_grid'), 'pipe', c.get('pipelined'))" "$cfg"
done
