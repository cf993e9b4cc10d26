mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash tools/cli_ab.sh gpurun_out/r6_cli_ab3 4 head= || exit 1
cat gpurun_out/r6_cli_ab3/out_md5.txt
