set -e
mkdir -p gpurun_out
MCAAT_KNOBS=nc.desc_cap=1536 CFG=c2 STEPS=3 bash tools/abq.sh default
MCAAT_KNOBS=nc.big_table=1 CFG=c2 STEPS=3 bash tools/abq.sh default
MCAAT_KNOBS=nc.group_budget=100000000 CFG=c2 STEPS=3 bash tools/abq.sh default
