# The full C3 (or $1) dataset: the one-GPU path's digest, then WORLD shm ranks' (tools/shard_run.sh);
# prints both (graph + CycleFinder checksums, stage times, CycleFinder device memory).
set -e
mkdir -p gpurun_out
CFG=${1:-c3}
PRE=""
if [ -n "$PROF" ]; then PRE="rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_shard -o single --"; fi
timeout -k 10 600 $PRE python -u tools/native_multi_check.py --world 1 --rank 0 --single --config $CFG \
   --digest gpurun_out/shard_single.json > gpurun_out/shard_single.log 2>&1
tail -2 gpurun_out/shard_single.log
bash tools/shard_run.sh $CFG "${@:2}"
python3 - <<PY
import json
a = json.load(open("gpurun_out/shard_single.json"))
for r in range(${WORLD:-2}):
    b = json.load(open(f"gpurun_out/shard_rank{r}.json"))
    same = {k: a[k] == b[k] for k in ("D", "keys", "mult", "valid", "stats", "results", "entries", "cycles")}
    print("rank", r, "equal to one GPU:", all(same.values()), same)
    print("  cf hbm", b.get("cf_hbm_GB"), "one GPU", a.get("cf_hbm_GB"), "build peak", b.get("build_hbm_peak_GB"))
    print("  collectives", b.get("collectives"), "queued", b.get("collectives_queued"))
    print("  build ms", b.get("build_stages_ms"))
    print("  cf ms", b.get("cf_stages_ms"))
PY
# keep the kernel statistics only (the traces exceed what gpurun copies back)
if [ -n "$PROF" ]; then find gpurun_out/prof_shard -name "*kernel_trace*" -delete; fi
exit 0
