# bench value of three library builds in alternating processes (sahara_amd/lib/ab/<name>.so)
mkdir -p gpurun_out
for i in 1 2 3; do for L in "$@"; do
  SAHARA_HIP_LIB=$GRAFT_REPO_ROOT/sahara_amd/lib/ab/$L.so timeout -k 10 300 python3 bench.py --no-cpu --no-count --no-e2e --no-verify --no-ref-path --no-device-resident --no-ingest > gpurun_out/ab.json 2> gpurun_out/ab.log || { tail -3 gpurun_out/ab.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'])" $L | tee -a gpurun_out/lib_ab3.txt
done; done
