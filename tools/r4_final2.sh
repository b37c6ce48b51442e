set -e
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || { tail -40 gpurun_out/gpu_suite.log; exit 1; }
tail -1 gpurun_out/gpu_suite.log
CFG=c5 bash tools/kstats.sh r04_c5 > gpurun_out/r04_c5_kstats.txt
timeout -k 10 500 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/r04_c5_bench.json 2> gpurun_out/r04_c5_bench.err
tail -1 gpurun_out/r04_c5_bench.json | cut -c1-200
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log
