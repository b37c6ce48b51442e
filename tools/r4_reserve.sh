set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_downstream.py tests/test_cli.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t12.log 2>&1 || { tail -30 gpurun_out/t12.log; exit 1; }
tail -1 gpurun_out/t12.log
timeout -k 10 900 python tools/e2e_probe.py --config c3 --preread --gap 25 --variants "MCAAT_RESERVE=0;MCAAT_RESERVE=1;MCAAT_RESERVE=0;MCAAT_RESERVE=1" > gpurun_out/reserve.log 2>&1
cat gpurun_out/reserve.log | cut -c1-400
