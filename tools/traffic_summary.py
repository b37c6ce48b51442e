"""Per-kernel HBM traffic from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/pmc_c3.sh).

Units and gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
FETCH_SIZE / WRITE_SIZE are in KiB; FETCH_SIZE reads exactly half of the bytes of a wide
(16 B/lane) coalesced stream, so reads are doubled. Output: profiles/traffic.json, keyed by the
bench's kernel names, with bytes per launch.
Usage: python tools/traffic_summary.py gpurun_out/pmc profiles/traffic.json
"""
import collections
import csv
import json
import re
import sys

src, dst = sys.argv[1], sys.argv[2]
NAMES = {"k_sk_scatter": "sk_scatter", "k_lds_count": "lds_count", "k_l2_scatter": "l2_partition",
         "k_l2_hist": "l2_hist"}
fetch = collections.defaultdict(float)
write = collections.defaultdict(float)
launches = collections.defaultdict(set)
for name, acc in (("f", fetch), ("w", write)):
    for r in csv.DictReader(open(f"{src}/{name}/{name}_counter_collection.csv")):
        m = re.search(r"(k_[a-z0-9_]+)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:40]
        acc[k] += float(r["Counter_Value"]) * 1024.0
        launches[k].add(r["Dispatch_Id"])
out = {}
for k in sorted(set(fetch) | set(write), key=lambda x: -(fetch[x] + write[x])):
    n = max(1, len(launches[k]))
    rec = {"launches": n, "fetch_bytes_raw": fetch[k] / n, "write_bytes": write[k] / n,
           "hbm_bytes_per_launch": (2.0 * fetch[k] + write[k]) / n}
    out[k] = rec
    if k in NAMES:
        agg = out.setdefault(NAMES[k] + "@", {"hbm_bytes_per_launch": 0.0})
        agg["hbm_bytes_per_launch"] += rec["hbm_bytes_per_launch"]
for k in list(out):
    if k.endswith("@"):
        out[k[:-1]] = out.pop(k)
json.dump(out, open(dst, "w"), indent=1)
for k, v in list(out.items())[:16]:
    print("%-28s %12.2f GB/launch" % (k, v["hbm_bytes_per_launch"] / 1e9))
