set -e
mkdir -p gpurun_out
MCAAT_VERBOSE=1 timeout -k 10 400 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-post --ingest-reads 0 --no-e2e > gpurun_out/c5v.json 2> gpurun_out/c5v.err
grep -c . gpurun_out/c5v.err
CFG=c5 bash tools/kstats.sh r04_c5b > gpurun_out/r04_c5b_kstats.txt
head -30 gpurun_out/r04_c5b_kstats.txt
