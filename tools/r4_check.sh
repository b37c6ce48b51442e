# round-4 check on the GPU box: GPU suite, then C3 A/Bs (library variants and knobs)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || { tail -30 gpurun_out/gpu_suite.log; exit 1; }
tail -2 gpurun_out/gpu_suite.log
bash tools/abq.sh default ab/nocoop.so
MCAAT_KNOBS=cf.compact=0 bash tools/abq.sh default
MCAAT_KNOBS=cf.dls_persist=0 bash tools/abq.sh default
CFG=c5 bash tools/abq.sh default
CFG=c5 MCAAT_KNOBS=cf.compact=0,cf.dls_persist=0,nc.big_table=1 bash tools/abq.sh default
