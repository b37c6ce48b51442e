set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fastq_ingest.py tests/test_cli.py tests/test_downstream.py tests/test_read_mapping.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t16.log 2>&1 || { tail -30 gpurun_out/t16.log; exit 1; }
tail -1 gpurun_out/t16.log
timeout -k 10 400 python bench.py > gpurun_out/r04_c3_bench_final.json 2> gpurun_out/r04_c3_bench_final.err
tail -1 gpurun_out/r04_c3_bench_final.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['e2e']['T_s'], d['e2e']['build_lib_s'], d['e2e']['sdbg_build_s'], d['e2e']['cycle_finder_s'], d['e2e']['planted_recall'])"
