mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash tools/cli_ab.sh gpurun_out/r6_cli_ab2 3 pf8= pf0=SAHARA_CLI_PREFAULT=0 || exit 1
