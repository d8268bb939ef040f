"""Run only the DoA scan (the bench's fused DoA + ESPRIT + phase launch) a few times on one cfg2 batch, for
rocprofv3 counter passes (tools/doa_counters.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

F = int(os.environ.get('F', '200'))
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=8, num_chirps=128, chirp_duration=51.2e-6)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(ctx, 1, F, 8, 128, 51.2e-6, 0)[0]
ch.run(cube)
L = ch.lists
for _ in range(int(os.environ.get('REPS', '3'))):
    ctx.doa_extras(ch.rds, L['c_frame'], L['c_rc'], ch.steer, ch.method, n=ch.cell_cap, n_dev=ch.ncell_dev,
                   esprit_scale=ch.esprit_scale, out_idx=ch.gidx, esprit=ch.ext['esprit'], phase=ch.ext['phase'])
torch.cuda.synchronize()
print('entries, cells', ch.totals())
