import csv, glob, collections, sys
d = sys.argv[1]
api = glob.glob(d + "/**/*hip_api_trace.csv", recursive=True)
ker = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
print(api, ker)
rows = list(csv.DictReader(open(api[0])))
tot = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r["Function"]
    t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    tot[n][0] += 1
    tot[n][1] += t
for n, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1])[:25]:
    print(f"{n:40s} {c:8d} {t:10.2f} ms  avg {1000*t/c:8.1f} us")
