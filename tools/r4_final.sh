set -e
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_gpu_suite.log 2>&1 || { tail -40 gpurun_out/r04_gpu_suite.log; exit 1; }
tail -1 gpurun_out/r04_gpu_suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> gpurun_out/r04_gpu_suite.log 2>&1
tail -1 gpurun_out/r04_gpu_suite.log
