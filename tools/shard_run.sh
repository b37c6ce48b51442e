# Two (or $WORLD) shared-memory ranks of tools/native_multi_check.py on one GPU, each logging to
# gpurun_out/shard_rank<r>.log (MCAAT_VERBOSE stage marks; PROF=1: each rank under rocprofv3 --kernel-trace
# --stats into gpurun_out/prof_shard). Usage: bash tools/shard_run.sh <config> [extra args]
set -e
mkdir -p gpurun_out
W=${WORLD:-2}
NAME=/mcaat_sr_$$
pids=()
for r in $(seq 0 $((W-1))); do
  PRE=""
  if [ -n "$PROF" ]; then PRE="rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_shard -o rank$r --"; fi
  MCAAT_VERBOSE=${VERB:-1} timeout -k 10 ${TLIM:-800} $PRE python -u tools/native_multi_check.py --world $W --rank $r --comm shm \
     --name $NAME --config $1 --digest gpurun_out/shard_rank{rank}.json --slot 0 "${@:2}" > gpurun_out/shard_rank$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
tail -3 gpurun_out/shard_rank0.log
exit $rc
