"""Run only the DoA scan a few times on one cfg2 batch (for rocprofv3 counter passes)."""
import os, sys
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
L = ch.lists
for _ in range(int(os.environ.get('REPS', '3'))):
    ctx.doa(ch.rds, L['c_frame'], L['c_rc'], ch.steer, 1, n=ch.cell_cap, n_dev=ch.ncell_dev, out_idx=ch.gidx)
torch.cuda.synchronize()
print('cells', ch.totals())
