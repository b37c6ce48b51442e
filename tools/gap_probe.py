import sys, time
sys.path.insert(0, '.')
import bench, mcaat_amd as M
import torch
cfg = dict(bench.CONFIGS['c3'])
spec = M.SynthSpec(**cfg['spec'].__dict__)
prm = M.CfParams()
with M.Context(0) as ctx:
    reads = M.Reads.synth(ctx, spec)
    for it in range(6):
        t0 = time.perf_counter()
        g = M.Graph.build(ctx, reads, 27)
        t1 = time.perf_counter()
        sb = ctx.stage_times()
        res = g.cycle_finder(prm, as_arrays=True)
        t2 = time.perf_counter()
        sc = ctx.stage_times()
        g.free()
        t3 = time.perf_counter()
        print(sb, flush=True)
        print(f"build {1e3*(t1-t0):.1f} (stages {sum(sb.values()):.1f})  cf {1e3*(t2-t1):.1f} (stages {sum(sc.values()):.1f})  free {1e3*(t3-t2):.1f}", flush=True)
