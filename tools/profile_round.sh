# One round's profiles of a config: rocprofv3 kernel stats, then separate FETCH_SIZE and
# WRITE_SIZE passes (never combined with traces), summarised per kernel.
# usage: CFG=c3 bash tools/profile_round.sh r03   -> gpurun_out/kstats/<r>_<cfg>, gpurun_out/pmc_<cfg>
R=$PWD; TAG=${1:-r03}; CFG=${CFG:-c3}
CFG=$CFG bash tools/kstats.sh ${TAG}_${CFG} > gpurun_out/${TAG}_${CFG}_kstats.txt || exit $?
rm -rf gpurun_out/pmc && CFG=$CFG bash tools/pmc_c3.sh 0 "f w" || exit $?
rm -rf gpurun_out/pmc_$CFG && mv gpurun_out/pmc gpurun_out/pmc_$CFG
NB=$(python -c "import sys; sys.path.insert(0, '$R'); from mcaat_amd.configs import CONFIGS; s = CONFIGS['$CFG']['spec']; print(s.n_reads * s.read_len)")
python tools/traffic_summary.py gpurun_out/pmc_$CFG gpurun_out/traffic_$CFG.json $NB > gpurun_out/${TAG}_${CFG}_traffic.txt
