import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import mcaat_amd as M
from test_scale_parity import CASES, _oracle
ctx = M.Context(0)
spec, k, prm = CASES["c1_k27"]
ref = _oracle("c1_k27")
reads = M.Reads.synth(ctx, spec)
for extra in [dict(), dict(nc__split_max=2), dict(nc__split_first=2, nc__split_max=2), dict(nc__split_first=1), dict(nc__big_table=0)]:
    kn = dict(nc__l1_slots=64, nc__fine_bits=12); kn.update(extra)
    with ctx.knobs(**kn):
        gk, gc = M.count_edges(ctx, reads, k)
    ok = np.array_equal(gk, ref["ck"]) and np.array_equal(gc, ref["cc"])
    a = dict(zip(gk.tolist(), gc.tolist())); b = dict(zip(ref["ck"].tolist(), ref["cc"].tolist()))
    miss = len(set(b) - set(a)); extra_k = len(set(a) - set(b)); diff = sum(1 for x in a if x in b and a[x] != b[x])
    print(extra, ok, len(gk), len(ref["ck"]), "missing", miss, "extra", extra_k, "count diffs", diff, "dup", len(gk) - len(a), flush=True)
