set -e
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || { tail -40 gpurun_out/gpu_suite.log; exit 1; }
tail -1 gpurun_out/gpu_suite.log
CFG=c3 STEPS=3 bash tools/abq.sh default ab/wpipe2.so default ab/wpipe2.so
timeout -k 10 300 python tools/native_multi_check.py --world 1 --rank 0 --comm shm --name /mcaat_r4w1 --config c3 --digest gpurun_out/w1.json > gpurun_out/w1.log 2>&1
grep "rank 0" gpurun_out/w1.log | cut -c1-600
