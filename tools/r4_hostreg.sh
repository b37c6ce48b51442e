set -e
mkdir -p gpurun_out
timeout -k 10 300 python - <<'PY'
import sys; sys.path.insert(0, '.')
import mcaat_amd as M, bench
cfg = bench.CONFIGS['c3']; spec = M.SynthSpec(**cfg['spec'].__dict__); spec.n_reads = 30_000_000
with M.Context(0) as ctx:
    r = M.Reads.synth(ctx, spec); r.write_fastq('/dev/shm/hostreg_probe.fq', threads=16); r.free()
PY
cat /dev/shm/hostreg_probe.fq > /dev/null
rc=0
timeout -k 10 300 ./tools/hostreg_probe /dev/shm/hostreg_probe.fq 256 16 > gpurun_out/hostreg.log 2>&1 && \
timeout -k 10 300 ./tools/hostreg_probe /dev/shm/hostreg_probe.fq 1024 16 >> gpurun_out/hostreg.log 2>&1 || rc=$?
rm -f /dev/shm/hostreg_probe.fq
cat gpurun_out/hostreg.log
exit $rc
