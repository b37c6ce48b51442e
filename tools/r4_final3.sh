set -e
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/r04_c3_bench_final.json 2> gpurun_out/r04_c3_bench_final.err
tail -1 gpurun_out/r04_c3_bench_final.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['e2e']['T_s'], d['e2e']['build_lib_s'], d['e2e']['sdbg_build_s'], d['e2e']['cycle_finder_s'], d['roofline']['frac'])"
