"""Doppler/detect (K2) ablation on one cfg2 batch: the kernel's time with one part removed at a time
(RSL_DD_DBG: 1 no FFT, 2 no RDS store, 3 no detection, 4 no peak-power stores, 5 no mask stores; results are wrong
in the variants, only their times matter).  GPU box:  python tools/dd_ablation.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

F = int(os.environ.get('F', '1000'))
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=8, num_chirps=128, chirp_duration=51.2e-6)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(ctx, 1, F, 8, 128, 51.2e-6, 0)[0]


def run():
    ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                   row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)


best = {}
for rep in range(4):  # variants in rotation; the minimum over rotations (clock / warm-up noise is ~10 %)
    for v in ['0', '1', '2', '3', '4', '5']:
        os.environ['RSL_DD_DBG'] = v
        run()
        torch.cuda.synchronize()
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        t = ctx.timing_read()
        ctx.timing(False)
        d = t["doppler_fft"][0] / 5
        best[v] = min(best.get(v, 1e9), d)
names = {'0': 'full', '1': 'no FFT', '2': 'no RDS store', '3': 'no detection', '4': 'no peak-power stores',
         '5': 'no mask stores'}
for v, d in best.items():
    print(f'RSL_DD_DBG={v} ({names[v]}): doppler/detect {d:.3f} ms (min of 4)', flush=True)
