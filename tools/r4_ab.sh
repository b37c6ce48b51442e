set -e
mkdir -p gpurun_out
CFG=c5 STEPS=2 bash tools/abq.sh default ab/prep8.so
MCAAT_KNOBS=cf.scan_u=1 CFG=c5 STEPS=2 bash tools/abq.sh default
CFG=c3 STEPS=3 bash tools/abq.sh ab/prep8.so
MCAAT_KNOBS=cf.scan_u=1 CFG=c3 STEPS=3 bash tools/abq.sh default
