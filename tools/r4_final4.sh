set -e
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || { tail -40 gpurun_out/gpu_suite.log; exit 1; }
tail -1 gpurun_out/gpu_suite.log
timeout -k 10 900 python tools/e2e_probe.py --config c3 --preread --settle 30 --gap 40 --variants "X=1;X=2" > gpurun_out/fq.log 2>&1
grep -E "variant" gpurun_out/fq.log | sed 's/TIMING_GROW.*//' | cut -c1-170
