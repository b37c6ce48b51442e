set -e
mkdir -p gpurun_out
MCAAT_PROF_C=1 MCAAT_KNOBS=nc.overlap=0 timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-post --ingest-reads 0 --no-e2e > gpurun_out/c5p.json 2> gpurun_out/c5p.err
grep -a "pass C" gpurun_out/c5p.err | tail -1
tail -1 gpurun_out/c5p.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms'], d['roofline']['kernels_ms_per_step'])"
