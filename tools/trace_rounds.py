"""Timeline of a window of a rocprofv3 run (kernel + HIP API traces): the calls and kernels
between the n-th and (n+k)-th launch of a named kernel, with their start offsets and durations,
to see where a bulk-synchronous round's time goes.
usage: python tools/trace_rounds.py <trace dir> <kernel name> <n> <k>"""
import csv
import glob
import re
import sys

d, name, n0, k = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
kr = list(csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0])))
ar = list(csv.DictReader(open(glob.glob(d + "/**/*hip_api_trace.csv", recursive=True)[0])))
ev = []
for r in kr:
    m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + (m.group(1) if m else r["Kernel_Name"][:30])))
for r in ar:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "A " + r["Function"]))
ev.sort()
hits = [e for e in ev if e[2] == "K " + name]
t0, t1 = hits[n0][0], hits[n0 + k][0]
for s, e, nm in ev:
    if t0 - 20000 <= s <= t1:
        print("%9.1f us  %8.1f us  %s" % ((s - t0) / 1e3, (e - s) / 1e3, nm))
