"""Size of the DepthLevelSearch / FindCycle search region at a bench config (the
sparse-replica design): after CycleFinder, the valid edges within `hops` undirected hops of the
start candidates (mcaat_graph_keep_region), against the post-peel valid edges and D.
usage: python tools/region_probe.py [--config c3] [--hops 77]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mcaat_amd as M  # noqa: E402
from mcaat_amd.configs import CONFIGS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--hops", type=int, default=77)
a = ap.parse_args()
cfg = CONFIGS[a.config]
ctx = M.Context(0)
reads = M.Reads.synth(ctx, cfg["spec"])
g = M.Graph.build(ctx, reads, cfg["k"])
reads.free()
res = g.cycle_finder(M.CfParams(threshold_multiplicity=cfg["thr"]))
D = g.size
cand = np.array(sorted(res.candidates), dtype=np.uint64)
out = {"config": a.config, "D": D, "post_peel_valid": res.stats[2], "candidates": int(cand.size)}
t0 = time.time()
g.keep_region(cand, a.hops)
dt = time.time() - t0
ids1, _, _ = g.valid_subgraph()
out.update({"hops": a.hops, "region_edges": int(ids1.size),
            "region_fraction_of_D": ids1.size / D, "keep_region_s": round(dt, 3)})
print("REGION", out, flush=True)
