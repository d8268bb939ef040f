"""Run the RDS + detection launch (K1 + K2) a few times on one cfg2 batch (CFG=cfg5: 100 configs[4]-shape frames), for rocprofv3 counter passes
(tools/dd_counters.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

A, C, TC, F0 = {'cfg2': (8, 128, 51.2e-6, 1000), 'cfg5': (16, 256, 102.4e-6, 100), 'cfg1': (8, 64, 25.6e-6, 2000)}[os.environ.get('CFG', 'cfg2')]
F = int(os.environ.get('F', str(F0)))
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=TC)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(ctx, 1, F, A, C, TC, 0)[0]
for _ in range(int(os.environ.get('REPS', '3'))):
    ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                   row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)
torch.cuda.synchronize()
print('done', flush=True)
