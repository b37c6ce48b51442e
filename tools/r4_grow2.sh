set -e
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_scale_parity.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/grow2_t.log 2>&1 || { tail -30 gpurun_out/grow2_t.log; exit 1; }
tail -1 gpurun_out/grow2_t.log
MCAAT_VERBOSE=1 timeout -k 10 400 python bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-post --ingest-reads 0 --no-e2e > gpurun_out/grow.log 2> gpurun_out/grow.err
grep -E "node_counter" gpurun_out/grow.err | tail -8
timeout -k 10 400 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-post --ingest-reads 0 --no-e2e > gpurun_out/grow_b.log 2> gpurun_out/grow_b.err
tail -1 gpurun_out/grow_b.log | cut -c1-160
