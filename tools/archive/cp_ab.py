"""Cache-policy A/B of the two RDS kernels on one cfg2 batch, min of 4 rotations: RSL_RF_CP (K1; bit 0 nt cube
loads, bit 1 nt work stores) x RSL_DD_CP (K2; bit 0 nt interior loads, bit 1 nt RDS stores, bit 2 nt halo
loads).  GPU box:  python tools/cp_ab.py"""
import os
import sys

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
PAIRS = [(4, 0), (0, 0), (1, 0), (2, 0), (3, 0), (6, 0), (0, 2), (2, 2), (3, 2), (0, 3)]


def run():
    ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                   row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)


best = {}
for rep in range(4):
    for rf, dd in PAIRS:
        os.environ['RSL_RF_CP'], os.environ['RSL_DD_CP'] = str(rf), str(dd)
        run()
        torch.cuda.synchronize()
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        t = ctx.timing_read()
        ctx.timing(False)
        k1, k2 = t['range_fft'][0] / 5, t['doppler_fft'][0] / 5
        b = best.get((rf, dd), (1e9, 1e9, 1e9))
        best[(rf, dd)] = (min(b[0], k1), min(b[1], k2), min(b[2], k1 + k2))
for (rf, dd), (k1, k2, s) in best.items():
    print(f'RF_CP={rf} DD_CP={dd}: range {k1:.3f} ms, doppler/detect {k2:.3f} ms, sum {s:.3f} ms', flush=True)
