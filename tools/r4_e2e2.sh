set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "keep_region or valid_subgraph or cli or downstream or planted or order" > gpurun_out/t4.log 2>&1 || { tail -30 gpurun_out/t4.log; exit 1; }
tail -1 gpurun_out/t4.log
bash tools/r4_e2e.sh
