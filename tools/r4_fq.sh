set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fastq_ingest.py tests/test_cli.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t14.log 2>&1 || { tail -30 gpurun_out/t14.log; exit 1; }
tail -1 gpurun_out/t14.log
MCAAT_PACK_SPLIT=4 timeout -k 10 900 python -u -m pytest tests/test_fastq_ingest.py -m gpu -x -q --timeout 600 --timeout-method thread -k host_pack > gpurun_out/t15.log 2>&1 || { tail -30 gpurun_out/t15.log; exit 1; }
tail -1 gpurun_out/t15.log
timeout -k 10 900 python tools/e2e_probe.py --config c3 --preread --settle 30 --gap 40 --verbose --variants "MCAAT_PACK_SPLIT=16;MCAAT_PACK_SPLIT=8;MCAAT_PACK_SPLIT=1;MCAAT_PACK_SPLIT=16;MCAAT_PACK_SPLIT=8;MCAAT_PACK_SPLIT=1" > gpurun_out/fq.log 2>&1
grep -E "variant|fq: |fq\.pack" gpurun_out/fq.log | sed 's/TIMING_GROW.*//' | cut -c1-170
