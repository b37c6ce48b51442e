set -e
mkdir -p gpurun_out
MCAAT_E2E_LOG=gpurun_out/e2e_cli.log timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-post --ingest-reads 0 > gpurun_out/b3.json 2> gpurun_out/b3.err
tail -1 gpurun_out/b3.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']); print(d['e2e'].get('T_s'), d['e2e'].get('cli_phases_s'))"
grep TIMING gpurun_out/e2e_cli.log
