"""K2 peak-power store A/B on one cfg2 batch: per-wave compacted stores (RSL_DD_CP=2, default) vs the tile's run
staged in LDS and stored block-wide (RSL_DD_CP=10); checks the outputs are bit-identical, then min of 6 rotations.
GPU box:  python tools/pk_ab.py"""
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
VARS = ['10', '26']


def run():
    ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                   row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)


outs = {}
for v in VARS:
    os.environ['RSL_DD_CP'] = v
    ch.peak_pow.zero_()
    run()
    torch.cuda.synchronize()
    outs[v] = (ch.peak_pow.clone(), ch.mask.clone(), ch.row_count.clone(), ch.rds.clone())
same = all(torch.equal(a, b) for a, b in zip(outs[VARS[0]], outs[VARS[1]]))
print(f'outputs bit-identical: {same}', flush=True)
best = {}
for rep in range(6):
    for v in VARS:
        os.environ['RSL_DD_CP'] = v
        run()
        torch.cuda.synchronize()
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        t = ctx.timing_read()
        ctx.timing(False)
        best[v] = min(best.get(v, 1e9), t['doppler_fft'][0] / 5)
for v, d in best.items():
    print(f'RSL_DD_CP={v}: doppler/detect {d:.3f} ms (min of 6)', flush=True)
