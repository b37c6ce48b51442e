set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cli.py tests/test_downstream.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t13.log 2>&1 || { tail -30 gpurun_out/t13.log; exit 1; }
tail -1 gpurun_out/t13.log
timeout -k 10 900 python tools/e2e_probe.py --config c3 --preread --gap 25 --variants "MCAAT_PRELOAD=0;X=1;MCAAT_PRELOAD=0;X=1;HIP_ENABLE_DEFERRED_LOADING=0" > gpurun_out/defer.log 2>&1
grep variant gpurun_out/defer.log | sed 's/TIMING_GROW.*//' | cut -c1-250
