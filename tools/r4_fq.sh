set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fastq_ingest.py tests/test_cli.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t14.log 2>&1 || { tail -30 gpurun_out/t14.log; exit 1; }
tail -1 gpurun_out/t14.log
timeout -k 10 900 python tools/e2e_probe.py --config c3 --preread --settle 30 --gap 40 --verbose --variants "X=1;X=2" > gpurun_out/fq.log 2>&1
grep -E "variant|fq\.concat|fq\.pack" gpurun_out/fq.log | sed 's/TIMING_GROW.*//' | cut -c1-170
