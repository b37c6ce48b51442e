# round-4 final profiles on the GPU box: the C3 bench line, kernel stats and FETCH/WRITE
# traffic, SQ LDS/wait counters, C5 kernel stats and bench line, one-rank RCCL sharded build
set -e
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r04_c3_bench.json 2> gpurun_out/r04_c3_bench.err
tail -1 gpurun_out/r04_c3_bench.json | cut -c1-300
CFG=c3 bash tools/profile_round.sh r04
rm -rf gpurun_out/pmc && bash tools/pmc_c3.sh 0 "s5 s2" && rm -rf gpurun_out/pmc_c3_sq && mv gpurun_out/pmc gpurun_out/pmc_c3_sq
CFG=c5 bash tools/kstats.sh r04_c5 > gpurun_out/r04_c5_kstats.txt
timeout -k 10 500 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/r04_c5_bench.json 2> gpurun_out/r04_c5_bench.err
timeout -k 10 400 python tools/native_multi_check.py --world 1 --rank 0 --comm rccl --name /mcaat_r4r1 --uid-file /tmp/mcaat_r4_uid --config c3 --digest gpurun_out/w1r.json > gpurun_out/w1r.log 2>&1
grep "rank 0" gpurun_out/w1r.log | sed 's/.*build_stages_ms/build_stages_ms/'
echo prof-done
