"""Time the DoA kernel's ablation variants (RSL_DOA_DBG=0..4) on one cfg2 batch: 1 = no record-tile copies,
2 = no MFMA, 3 = no signature loads, 4 = no Toeplitz operand math, 7 = one of the eight record-tile copies.  Results are wrong by construction for 1-4."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch, rsl
from bench import make_cubes
F = int(os.environ.get('F', '1000'))
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=8, num_chirps=128, chirp_duration=51.2e-6)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(ctx, 1, F, 8, 128, 51.2e-6, 0)[0]
ch.run(cube)
torch.cuda.synchronize()
L = ch.lists
res = {}
for rnd in range(2):
    for v in ['0', '1', '2', '3', '4', '7']:
        os.environ['RSL_DOA_DBG'] = v
        idx = torch.empty_like(ch.gidx)
        run = lambda: ctx.doa(ch.rds, L['c_frame'], L['c_rc'], ch.steer, 1, n=ch.cell_cap, n_dev=ch.ncell_dev, out_idx=idx)
        run(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            run()
        e1.record(); torch.cuda.synchronize()
        res.setdefault(v, []).append(e0.elapsed_time(e1) / 5)
print(json.dumps({k: round(min(x), 4) for k, x in res.items()}))
