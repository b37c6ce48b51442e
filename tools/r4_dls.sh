set -e
mkdir -p gpurun_out
STEPS=3 CFG=c5 bash tools/abq.sh default
MCAAT_KNOBS=cf.dls_budget=16 CFG=c5 STEPS=3 bash tools/abq.sh default
MCAAT_KNOBS=cf.dls_budget=32 CFG=c5 STEPS=3 bash tools/abq.sh default
