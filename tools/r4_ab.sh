set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "building_blocks or two_owners or bad_keys or valid_subgraph" > gpurun_out/t7.log 2>&1 || { tail -30 gpurun_out/t7.log; exit 1; }
tail -1 gpurun_out/t7.log
CFG=c3 STEPS=3 bash tools/abq.sh default ab/wpipe2.so default ab/wpipe2.so
MCAAT_PROF_A=1 MCAAT_LIB=$PWD/ab/wpipe2.so timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-post --no-e2e --ingest-reads 0 2> gpurun_out/pa2.err > /dev/null
grep "pass A" gpurun_out/pa2.err | tail -1
