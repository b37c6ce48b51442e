# Parameterised GPU job (replaces round 4's one-off tools/r4_*.sh wrappers).
#   bash tools/gpu_check.sh tests "<pytest -k expr>"   selected GPU tests
#   bash tools/gpu_check.sh suite                       the whole GPU suite + smoke
#   bash tools/gpu_check.sh abq [c3|c2|c5] [steps]      quick timing (tools/abq.sh)
#   bash tools/gpu_check.sh bench                       the driver's default bench line
#   bash tools/gpu_check.sh rccl1 [c3]                  the sharded build's stages at one RCCL rank
#                                                       (second build; the exchanges are local copies)
#   bash tools/gpu_check.sh shard2 [c3]                 2 shm ranks vs one GPU, kernels profiled per rank
#   bash tools/gpu_check.sh shardn [c3] [world]         world shm ranks vs one GPU (digests, peaks, collectives)
# Every GPU step has its own time limit; the first failure ends the job.
set -e
mkdir -p gpurun_out
what=$1; shift || true
case "$what" in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$1" \
      > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
    tail -3 gpurun_out/gpu_tests.log ;;
  suite)
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --durations=30 --timeout 600 --timeout-method thread \
      > gpurun_out/gpu_suite.log 2>&1 || { tail -40 gpurun_out/gpu_suite.log; exit 1; }
    tail -1 gpurun_out/gpu_suite.log
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log ;;
  abq)
    CFG=${1:-c3} STEPS=${2:-3} bash tools/abq.sh default ;;
  bench)
    timeout -k 10 900 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
    tail -1 gpurun_out/bench.log ;;
  rccl1)
    rm -f gpurun_out/rccl1.uid
    timeout -k 10 600 python -u tools/native_multi_check.py --world 1 --rank 0 --comm rccl --uid-file gpurun_out/rccl1.uid \
      --config ${1:-c3} --repeat 2 --digest gpurun_out/rccl1.json > gpurun_out/rccl1.log 2>&1 || { tail -30 gpurun_out/rccl1.log; exit 1; }
    rm -f gpurun_out/rccl1.uid
    tail -2 gpurun_out/rccl1.log ;;
  shardn)  # bash tools/gpu_check.sh shardn <config> <world>: WORLD shm ranks vs one GPU (full dataset)
    VERB=${VERB:-1} WORLD=${2:-4} bash tools/shard_compare.sh ${1:-c3} ;;
  shard2)
    PROF=1 VERB=1 WORLD=2 bash tools/shard_compare.sh ${1:-c3} && python3 tools/prof_compare.py > gpurun_out/prof_w2.txt ;;
  *) echo "unknown job $what"; exit 2 ;;
esac
