# quick A/B of library builds on C3 (plain timing, no profiling ticks): bash tools/abq.sh <lib.so|default>...
# CFG=c2 / c5 for another config; prints ms/step, stage times and the dominant kernels' ms per step
mkdir -p gpurun_out
for L in "$@"; do
  if [ "$L" = default ]; then unset MCAAT_LIB; else export MCAAT_LIB=$PWD/$L; fi
  timeout -k 10 300 python bench.py --config ${CFG:-c3} --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-post --ingest-reads 0 --no-e2e > gpurun_out/abq.log 2>&1 || { tail -5 gpurun_out/abq.log; exit 1; }
  echo "== $L"
  tail -1 gpurun_out/abq.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step %.1f D %d cycles %d' % (d['ms_per_step'], d['config']['sdbg_edges_D'], d['config']['cycles']), d['stages_ms'], d['roofline'].get('kernels_ms_per_step'))"
done
