set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_scale_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t10.log 2>&1 || { tail -30 gpurun_out/t10.log; exit 1; }
tail -1 gpurun_out/t10.log
CFG=c5 STEPS=2 bash tools/abq.sh default
CFG=c2 STEPS=3 bash tools/abq.sh default
CFG=c3 STEPS=3 bash tools/abq.sh default
