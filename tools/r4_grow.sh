mkdir -p gpurun_out
MCAAT_VERBOSE=1 timeout -k 10 400 python bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-post --ingest-reads 0 --no-e2e > gpurun_out/grow.log 2> gpurun_out/grow.err || { tail -20 gpurun_out/grow.err; exit 1; }
grep -E "node_counter" gpurun_out/grow.err | tail -40
