"""Run the whole batched chain (ch.run: RDS + detection, offsets, compaction, DoA + ESPRIT + phase, velocity) a few
times on one cfg2 batch, one stream, for rocprofv3 counter passes over every kernel (tools/chain_counters.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

F = int(os.environ.get('F', '1000'))
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=8, num_chirps=128, chirp_duration=51.2e-6, ridge=0.01)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(ctx, 1, F, 8, 128, 51.2e-6, 0)[0]
for _ in range(int(os.environ.get('REPS', '3'))):
    ch.run(cube)
torch.cuda.synchronize()
print('entries, cells', ch.totals(), flush=True)
