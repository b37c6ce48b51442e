set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_scale_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "grow or multi_group" > gpurun_out/t11.log 2>&1 || { tail -30 gpurun_out/t11.log; exit 1; }
tail -1 gpurun_out/t11.log
STEPS=3 CFG=c5 bash tools/abq.sh default
MCAAT_KNOBS=cf.dls_budget=16 CFG=c5 STEPS=3 bash tools/abq.sh default
MCAAT_KNOBS=cf.dls_budget=32 CFG=c5 STEPS=3 bash tools/abq.sh default
