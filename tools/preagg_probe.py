"""How much a sender-side collapse of identical descriptors would shrink the sharded build's
descriptor all-to-all (SURVEY §8e.1 "count locally first"). One rank of an
N-rank C3 run holds 1/N of the reads: pass C's LDS collapse over that slice reports its distinct
descriptors (MCAAT_PROF_C=1, node_counter.hip prof[6] / prof[7]), which is what the rank would
send after collapsing (a 16-B descriptor + a 4-B weight each) instead of every 16-B descriptor and
its 2-B sub row. usage: MCAAT_PROF_C=1 python tools/preagg_probe.py --config c3 --fractions 8,4,2,1"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import mcaat_amd as M  # noqa: E402
from mcaat_amd.configs import CONFIGS  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--fractions", default="8,4,2,1")
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    spec = cfg["spec"]
    with M.Context(0) as ctx:
        for n in [int(x) for x in a.fractions.split(",")]:
            r = M.Reads.synth_range(ctx, spec, 0, spec.n_reads // n)
            print(f"== 1/{n} of the reads ({spec.n_reads // n})", flush=True)
            sys.stderr.flush()
            c = M.Counts.count(ctx, r, cfg["k"])
            print(f"   distinct edges {c.n}", flush=True)
            c.free()
            r.free()
    return 0


if __name__ == "__main__":
    sys.exit(main())
