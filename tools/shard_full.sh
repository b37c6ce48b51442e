# Full-size datasets through shared-memory ranks on the one GPU, one config after another; the
# first failure ends the job (each run's rank logs are kept per config).
#   bash tools/shard_full.sh c3:8 c5:2
set -e
mkdir -p gpurun_out
for cw in "$@"; do
  cfg=${cw%%:*}; w=${cw##*:}
  rc=0
  VERB=1 WORLD=$w bash tools/shard_compare.sh $cfg > gpurun_out/shard_${cfg}_w${w}.txt 2>&1 || rc=$?
  for f in gpurun_out/shard_rank*.log gpurun_out/shard_rank*.json; do
    [ -e "$f" ] && mv "$f" "gpurun_out/${cfg}_w${w}_$(basename $f)"
  done
  tail -12 gpurun_out/shard_${cfg}_w${w}.txt
  [ $rc -eq 0 ] || exit $rc
done
