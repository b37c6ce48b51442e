# A/B timing of library builds: bash tools/ab.sh <lib.so>... (default lib when "default")
mkdir -p gpurun_out
for L in "$@"; do
  if [ "$L" = default ]; then unset MCAAT_LIB; else export MCAAT_LIB=$PWD/$L; fi
  MCAAT_PROF_A=1 MCAAT_PROF_C=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-post --ingest-reads 0 --no-e2e > gpurun_out/ab.log 2>&1 || exit $?
  echo "== $L"; grep -a "pass [AC]" gpurun_out/ab.log | tail -2; tail -1 gpurun_out/ab.log | grep -o "kernels_ms_per_step.\{100\}"
  tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step %.1f D %d cycles %d' % (d['ms_per_step'], d['config']['sdbg_edges_D'], d['config']['cycles']), d['stages_ms'])"
done
