#!/usr/bin/env python3
"""Peel stage time at C3 for several Kahn walk budgets (cf.walk_budget knob): how long the
pending chains are decides whether the list-ranking peel pays. usage: python tools/peel_probe.py b1 b2 ..."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import mcaat_amd as M  # noqa: E402

cfg = bench.CONFIGS["c3"]
with M.Context(0) as ctx:
    reads = M.Reads.synth(ctx, cfg["spec"])
    prm = M.CfParams(threshold_multiplicity=cfg["thr"])
    ref = None
    for b in [int(x) for x in sys.argv[1:]] or [512]:
        ctx.set_knob("cf.walk_budget", b)
        for rep in range(2):
            g = M.Graph.build(ctx, reads, cfg["k"])
            res = g.cycle_finder(prm, as_arrays=True)
            st = ctx.stage_times()
            _, _, valid = g.download_range(0, g.size, keys=False, mult=False, valid=True)
            h = int(valid.sum())
            g.free()
            print(f"budget {b} rep {rep}: peel {st['peel']:.2f} ms, valid {h}, stats {res.stats}", flush=True)
