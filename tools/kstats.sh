# rocprofv3 kernel statistics of one bench step: bash tools/kstats.sh <name> (CFG=c5 / c2: that
# config instead of C3)
R=$PWD; N=${1:-run}; CFG=${CFG:-c3}; export TMPDIR=/tmp; mkdir -p gpurun_out/kstats; cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kstats/$N -o $N -- python $R/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-post --ingest-reads 0 --no-e2e > $R/gpurun_out/kstats/$N.log 2>&1 || exit $?
python - "$R/gpurun_out/kstats/$N" <<'PY'
import csv, glob, re, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:22]:
    m = re.search(r"(k_[a-z0-9_]+)", r["Name"]); n = m.group(1) if m else r["Name"][:40]
    print("%-34s calls %6s  total %9.2f ms  avg %9.3f ms" % (n, r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e6))
PY
