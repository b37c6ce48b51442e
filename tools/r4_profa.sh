set -e
mkdir -p gpurun_out
MCAAT_PROF_A=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-post --no-e2e > gpurun_out/pa.json 2> gpurun_out/pa.err
grep "pass A" gpurun_out/pa.err | tail -3
python3 -c "import json; d=json.loads(open('gpurun_out/pa.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms'], d['roofline']['kernels_ms_per_step'])"
