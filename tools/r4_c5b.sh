set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t6.log 2>&1 || { tail -30 gpurun_out/t6.log; exit 1; }
tail -1 gpurun_out/t6.log
CFG=c5 STEPS=2 bash tools/abq.sh default
MCAAT_KNOBS=cf.compact=1 CFG=c5 STEPS=2 bash tools/abq.sh default
CFG=c3 STEPS=3 bash tools/abq.sh default
MCAAT_KNOBS=cf.compact=1 CFG=c3 STEPS=3 bash tools/abq.sh default
