"""K1 tile scheduling A/B on one cfg2 batch: static persistent walk (default) vs per-XCD dequeue (RSL_RF_DYN=1).
Checks that the range spectra / RDS / peaks are bit-identical (again after 30+ launches, so every queue slot has been
reused), then min of 6 rotations.  GPU box:  python tools/dyn_ab.py"""
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
VARS = ['0', '1']


def run():
    ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                   row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)


def outputs(v):
    os.environ['RSL_RF_DYN'] = v
    ch.work.zero_()
    ch.rds.zero_()
    run()
    torch.cuda.synchronize()
    return (ch.work.clone(), ch.rds.clone(), ch.mask.clone(), ch.row_count.clone())


ref = outputs('0')
print(f'outputs bit-identical: {all(torch.equal(a, b) for a, b in zip(ref, outputs("1")))}', flush=True)
best = {}
for rep in range(6):
    for v in VARS:
        os.environ['RSL_RF_DYN'] = v
        run()
        torch.cuda.synchronize()
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        t = ctx.timing_read()
        ctx.timing(False)
        best[v] = min(best.get(v, 1e9), t['range_fft'][0] / 5)
print(f'after reuse bit-identical: {all(torch.equal(a, b) for a, b in zip(ref, outputs("1")))}', flush=True)
for v, d in best.items():
    print(f'RSL_RF_DYN={v}: range fft {d:.3f} ms (min of 6)', flush=True)
