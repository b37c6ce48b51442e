# PMC counters for the hot-path kernels, one rocprofv3 pass per counter group
# (never combined with --sys-trace / runtime traces). Usage: bash tools/pmc_c3.sh [reads] [groups]
# CFG=c5 (or c2) profiles that config instead (its full read count unless N is given)
R=$PWD; CFG=${CFG:-c3}; N=${1:-0}; G=${2:-"f w"}; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp; cd /tmp
B="python $R/bench.py --config $CFG --reads $N --steps 1 --warmup 0 --no-cpu-baseline --no-post --ingest-reads 0 --no-e2e"
run() { name=$1; shift; timeout -k 10 400 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/pmc/$name -o $name -- $B > $R/gpurun_out/pmc/$name.log 2>&1; }
for g in $G; do
  case $g in
    f) run f FETCH_SIZE ;;
    w) run w WRITE_SIZE ;;
    s1) run s1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES ;;
    s2) run s2 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY ;;
    s3) run s3 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS ;;
    s4) run s4 SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH ;;
    s5) run s5 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS ;;
    u1) run u1 TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum ;;
    u2) run u2 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum ;;
    u3) run u3 TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum ;;
    u4) run u4 TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_sum ;;
  esac || exit $?
done
echo exit=0
