set -e
mkdir -p gpurun_out
rm -f /tmp/mcaat_r4_uid
timeout -k 10 500 python tools/native_multi_check.py --world 1 --rank 0 --comm rccl --name /mcaat_r4r1 --uid-file /tmp/mcaat_r4_uid --config c3 --repeat 2 --digest gpurun_out/w1r.json > gpurun_out/w1r.log 2>&1 || { tail -20 gpurun_out/w1r.log; exit 1; }
grep "rank 0" gpurun_out/w1r.log | sed 's/.*build_stages_ms/build_stages_ms/'
rm -f /tmp/mcaat_r4_uid
timeout -k 10 500 python tools/native_multi_check.py --world 1 --rank 0 --comm rccl --name /mcaat_r4r2 --uid-file /tmp/mcaat_r4_uid --config c3 --repeat 2 --knob dist.desc=0 --digest gpurun_out/w1r0.json > gpurun_out/w1r0.log 2>&1 || { tail -20 gpurun_out/w1r0.log; exit 1; }
grep "rank 0" gpurun_out/w1r0.log | sed 's/.*build_stages_ms/build_stages_ms/'
