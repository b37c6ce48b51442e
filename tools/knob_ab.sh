# A/B of an environment knob on the C3 bench: bash tools/knob_ab.sh VAR "v1 v2 ..." ("-" = unset)
mkdir -p gpurun_out
VAR=$1
for v in $2; do
  if [ "$v" = "-" ]; then unset $VAR; else export $VAR=$v; fi
  MCAAT_PROF_A=1 MCAAT_PROF_C=1 timeout -k 10 300 python bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --no-post --ingest-reads 0 --no-e2e > gpurun_out/knob.log 2>&1 || exit $?
  echo "== $VAR=$v"; grep -a "pass [AC]" gpurun_out/knob.log | tail -2
  tail -1 gpurun_out/knob.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('ms/step %.1f D %d cycles %d' % (d['ms_per_step'], d['config']['sdbg_edges_D'], d['config']['cycles']), r['kernels_ms_per_step'], d['stages_ms']['node_counter'])"
done
