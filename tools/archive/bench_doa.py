"""Microbenchmark of the DoA scan variants on one cfg2 batch (same cells, same process, interleaved):
'toep' = Toeplitz f16-MFMA hi/lo argmax (default), 'f32' = [Re; Im] f32-MFMA argmax, 'full' = f32 scan kernel."""
import os, sys, json
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
variants = {'toep': ({}, True), 'f32': ({}, False), 'full': ({'RSL_DOA_FULL': '1'}, False)}
out, res = {}, {}
for rnd in range(3):
    for name, (env, fast) in variants.items():
        os.environ.pop('RSL_DOA_FULL', None)
        os.environ.update(env)
        idx = torch.empty_like(ch.gidx)
        gm = torch.empty((ch.cell_cap,), dtype=torch.float32, device=idx.device)
        run = lambda: ctx.doa(ch.rds, L['c_frame'], L['c_rc'], ch.steer, 1, n=ch.cell_cap, n_dev=ch.ncell_dev,
                              out_idx=idx, fast=fast)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        res[name] = idx[:nc].cpu().numpy()
        flops = nc * 361 * 69
        out.setdefault(name, []).append(ms)
        print(f'{name}: {ms:.3f} ms  {flops / ms / 1e9:.1f} f32-equiv TFLOP/s', flush=True)
d = res['toep'] != res['f32']
print(f'cells {nc}; toep vs f32 argmax mismatches: {int(d.sum())} (adjacent {int((np.abs(res["toep"] - res["f32"])[d] == 1).sum())})')
print(json.dumps({k: min(v) for k, v in out.items()}))
