"""Microbenchmark of the DoA scan variants on one cfg2 batch (same cells, same process, interleaved)."""
import os, sys, time, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch, rsl
from bench import make_cubes
F = int(os.environ.get('F', '200'))
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=8, num_chirps=128, chirp_duration=51.2e-6)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(torch, torch.device('cuda', 0), 1, F, 8, 128, 512, 5)[0]
ch.run(cube)
torch.cuda.synchronize()
ne, nc = ch.totals()
L = ch.lists
out = {}
variants = {'argmax': {}, 'full': {'RSL_DOA_FULL': '1'}}
ref = None
for rnd in range(3):
    for name, env in variants.items():
        for k in ('RSL_DOA_FULL',):
            os.environ.pop(k, None)
        os.environ.update(env)
        idx = torch.empty_like(ch.gidx)
        ctx.doa(ch.rds, L['c_frame'], L['c_rc'], ch.steer, 1, n=ch.cell_cap, n_dev=ch.ncell_dev, out_idx=idx)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            ctx.doa(ch.rds, L['c_frame'], L['c_rc'], ch.steer, 1, n=ch.cell_cap, n_dev=ch.ncell_dev, out_idx=idx)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        h = idx[:nc].cpu().numpy()
        if ref is None:
            ref = h
        same = bool((h == ref).all())
        flops = nc * 361 * 69
        out.setdefault(name, []).append(ms)
        print(f'{name}: {ms:.3f} ms  {flops / ms / 1e9:.1f} TFLOP/s  same={same}', flush=True)
print(json.dumps({k: min(v) for k, v in out.items()}))
