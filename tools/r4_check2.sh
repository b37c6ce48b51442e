set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || { tail -30 gpurun_out/gpu_suite.log; exit 1; }
tail -2 gpurun_out/gpu_suite.log
MCAAT_E2E_LOG=gpurun_out/e2e_cli.log timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b2.json 2> gpurun_out/b2.err
tail -1 gpurun_out/b2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms']); print(d['e2e'].get('T_s'), d['e2e'].get('cli_phases_s'))"
