# Round-end measurement on one GPU box: GPU suite, kernel stats, FETCH/WRITE PMC passes, bench.
# Usage: bash tools/final_c3.sh <tag>   (outputs under gpurun_out/)
T=${1:-final}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 &&
bash tools/kstats.sh $T > gpurun_out/kstats_$T.txt 2>&1 &&
bash tools/pmc_c3.sh 300000000 "f w" > gpurun_out/pmc_$T.txt 2>&1 &&
timeout -k 10 420 python bench.py > gpurun_out/bench_$T.log 2>&1
