"""Per-kernel HBM traffic from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/pmc_c3.sh).

Units and the gfx950 correction (MI355X_MICROARCH.md §HBM, line "On gfx950 FETCH_SIZE reports
exactly 1/2 of the bytes of a wide coalesced streaming read"): FETCH_SIZE / WRITE_SIZE are in
KiB; FETCH_SIZE = TCC_EA0_RDREQ x 64 B, and a wide (16 B/lane) coalesced stream issues 128-B
requests tallied at 64 B, so ONLY those reads are doubled. Gathers (8 B or less per lane at
scattered addresses: peel walks, FindCycle, DLS, adjacency searches, the MSD scatter levels'
8-B items) issue 64-B requests and are taken as counted. Per kernel:
  stream   : every read a 16-B/lane stream       -> fetch x 2
  mixed    : k_sk_scatter (the 2-bit read stream, 0.25 B/base, is a 16-B/lane stream; the
             write phase's base re-fetches are gathers) -> fetch + 0.5 x stream bytes
  gather   : everything else                      -> fetch x 1
Both raw and corrected bytes are written side by side.
Output: profiles/traffic_<config>.json keyed by kernel (and the bench's short names), bytes
per launch. Usage: python tools/traffic_summary.py gpurun_out/pmc profiles/traffic_c3.json [n_bases]
"""
import collections
import csv
import json
import re
import sys

src, dst = sys.argv[1], sys.argv[2]
n_bases = float(sys.argv[3]) if len(sys.argv) > 3 else 300e6 * 150  # C3
NAMES = {"k_sk_scatter": "sk_scatter", "k_lds_count": "lds_count", "k_l2_scatter": "l2_partition",
         "k_l2_hist": "l2_hist"}
STREAM = {"k_lds_count", "k_l2_scatter", "k_l2_hist", "k_fallback", "k_part_occ", "k_tips_filter",
          "k_recount_candidates", "k_fq_nlcount", "k_fq_nlpos", "k_concat_parts"}
MIXED_STREAM_BYTES = {"k_sk_scatter": 0.25 * n_bases}
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
    raw = fetch[k] / n
    if k in STREAM:
        cls, corr = "stream", 2.0 * raw
    elif k in MIXED_STREAM_BYTES:
        cls, corr = "mixed", raw + 0.5 * MIXED_STREAM_BYTES[k]
    else:
        cls, corr = "gather", raw
    rec = {"launches": n, "read_class": cls, "fetch_bytes_raw": raw, "fetch_bytes_corrected": corr,
           "write_bytes": write[k] / n, "hbm_bytes_raw": raw + write[k] / n,
           "hbm_bytes_per_launch": corr + write[k] / n}
    out[k] = rec
    if k in NAMES:
        agg = out.setdefault(NAMES[k] + "@", {"hbm_bytes_per_launch": 0.0, "hbm_bytes_raw": 0.0})
        agg["hbm_bytes_per_launch"] += rec["hbm_bytes_per_launch"]
        agg["hbm_bytes_raw"] += rec["hbm_bytes_raw"]
for k in list(out):
    if k.endswith("@"):
        out[k[:-1]] = out.pop(k)
json.dump(out, open(dst, "w"), indent=1)
for k, v in list(out.items())[:16]:
    print("%-28s %12.2f GB/launch (raw %.2f)" % (k, v["hbm_bytes_per_launch"] / 1e9, v.get("hbm_bytes_raw", 0) / 1e9))
