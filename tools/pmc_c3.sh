# PMC counters for the node_counter kernels (one rocprofv3 pass per counter group).
# Usage on the GPU box: bash tools/pmc_c3.sh [reads]
R=$PWD; N=${1:-3000000}; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp; cd /tmp
B="python $R/bench.py --config c3 --reads $N --steps 1 --warmup 0 --no-cpu-baseline"
run() { name=$1; shift; timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/pmc/$name -o $name -- $B > $R/gpurun_out/pmc/$name.log 2>&1; }
run f FETCH_SIZE && run w WRITE_SIZE && run s1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES && run s2 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
echo exit=$?
