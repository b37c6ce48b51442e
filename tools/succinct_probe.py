"""The succinct (BOSS) view at a bench config's full size: bytes of both layouts,
the neighbour check over every edge, and the out-/in-degree scans timed on both, on the fresh
graph and after CycleFinder. usage: python tools/succinct_probe.py --config c3 --out FILE"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import mcaat_amd as M  # noqa: E402
from mcaat_amd.configs import CONFIGS  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--out", default="")
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    t0 = time.time()
    with M.Context(0) as ctx:
        r = M.Reads.synth(ctx, cfg["spec"])
        g = M.Graph.build(ctx, r, cfg["k"])
        r.free()
        D = g.size
        held_arrays = ctx.arena_usage()[0]
        fresh = g.succinct_check(not a.no_check)
        print("fresh", fresh, flush=True)
        g.cycle_finder(M.CfParams(threshold_multiplicity=cfg["thr"]))
        after = g.succinct_check(not a.no_check)
        print("after CycleFinder", after, flush=True)
        g.free()
    d = {"config": a.config, "D": D, "graph_hbm_bytes": held_arrays, "fresh": fresh, "after_cycle_finder": after,
         "view_B_per_edge": fresh["view_bytes"] / D, "arrays_B_per_edge": fresh["array_bytes"] / D,
         "seconds": round(time.time() - t0, 1)}
    print(json.dumps(d), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(d, f, indent=1)
    return 0 if fresh["out_mismatch"] == 0 and fresh["in_mismatch"] == 0 and after["out_mismatch"] == 0 \
        and after["in_mismatch"] == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
