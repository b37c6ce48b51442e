# A/B with pass A / pass C phase ticks: bash tools/abp.sh <lib.so|default>...  (CFG=c2 / c5 for another config)
mkdir -p gpurun_out
for L in "$@"; do
  if [ "$L" = default ]; then unset MCAAT_LIB; else export MCAAT_LIB=$PWD/$L; fi
  MCAAT_PROF_C=1 timeout -k 10 300 python bench.py --config ${CFG:-c3} --steps 2 --warmup 1 --no-cpu-baseline --no-post --ingest-reads 0 --no-e2e > gpurun_out/abp.log 2>&1 || { tail -5 gpurun_out/abp.log; exit 1; }
  echo "== $L"; grep -a "pass C" gpurun_out/abp.log | tail -1
done
