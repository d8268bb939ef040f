"""RDS + detection over 1000 cfg2 frames in one launch pair vs in chunks whose `work` intermediate (4 MiB per frame)
fits the 256 MiB Infinity Cache, so K2 may read K1's output from the cache instead of HBM.  GPU box."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

F = 1000
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=8, num_chirps=128, chirp_duration=51.2e-6)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(ctx, 1, F, 8, 128, 51.2e-6, 0)[0]


def run(chunk):
    for f0 in range(0, F, chunk):
        f1 = min(F, f0 + chunk)
        ctx.rds_detect(cube[f0:f1], ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds[f0:f1], work=ch.work[f0:f1],
                       mask=ch.mask[f0:f1], row_count=ch.row_count[f0:f1], peak_pow=ch.peak_pow[f0:f1],
                       dc_removal=True)


best = {}
for rep in range(3):
    for chunk in (1000, 100, 50, 25):
        run(chunk)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            run(chunk)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 5 * 1e3
        best[chunk] = min(best.get(chunk, 1e9), ms)
for chunk, ms in best.items():
    print(f'chunk {chunk:5d} frames: RDS + detection {ms:.3f} ms per 1000 frames (wall, min of 3)', flush=True)
