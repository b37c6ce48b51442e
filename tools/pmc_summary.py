#!/usr/bin/env python3
"""Per-kernel sums of the counters in gpurun_out/pmc/<group>/*counter_collection.csv.
usage: python tools/pmc_summary.py group [group...]"""
import csv, glob, os, re, sys, collections

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for g in sys.argv[1:]:
    files = glob.glob(os.path.join(ROOT, "gpurun_out", "pmc", g, "**", "*counter_collection.csv"), recursive=True)
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for fn in files:
        for row in csv.DictReader(open(fn)):
            m = re.search(r"\b(k_\w+)", row["Kernel_Name"])
            k = (m.group(1) if m else row["Kernel_Name"])[:40]
            tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
    print(f"== {g}")
    for k, d in sorted(tot.items(), key=lambda kv: -max(kv[1].values())):
        print(f"{k:42s} " + " ".join(f"{c}={v:.3e}" for c, v in sorted(d.items())))
