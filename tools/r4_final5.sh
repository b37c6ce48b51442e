set -e
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || { tail -40 gpurun_out/gpu_suite.log; exit 1; }
tail -1 gpurun_out/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log
