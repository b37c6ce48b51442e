# round-4 profiles on the GPU box: C3 bench line, kernel stats, FETCH/WRITE passes (traffic
# summary), SQ LDS/wait counters; C5 kernel stats and bench line
set -e
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r04_c3_bench.json 2> gpurun_out/r04_c3_bench.err
CFG=c3 bash tools/profile_round.sh r04
bash tools/pmc_c3.sh 0 "s5 s2"
CFG=c5 bash tools/kstats.sh r04_c5 > gpurun_out/r04_c5_kstats.txt
timeout -k 10 500 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/r04_c5_bench.json 2> gpurun_out/r04_c5_bench.err
echo prof-done
