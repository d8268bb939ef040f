"""Doppler-detect tile height A/B on one cfg2 batch: RSL_DD_KB=32 (34-row tiles; the 512-thread register-form
variant measured is described in DESIGN.md §5)
against the default 16-row tiles.  RDS, peak masks and row counts must be bit-identical (the Doppler FFT of a range
bin does not depend on its tile); then both are timed (min of 4 rotations).  GPU box:  python tools/kb_check.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

F, A, C, TC = int(os.environ.get('F', '1000')), 8, 128, 51.2e-6
KB = os.environ.get('KB', '32')
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=TC)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(ctx, 1, F, A, C, TC, 0)[0]


def run():
    return ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                          row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)


def setkb(kb):
    if kb:
        os.environ['RSL_DD_KB'] = kb
    else:
        os.environ.pop('RSL_DD_KB', None)


out = {}
for kb in ('', KB):
    setkb(kb)
    g = run()
    torch.cuda.synchronize()
    out[kb] = (ch.rds.clone(), ch.mask.clone(), ch.row_count.clone(), g)
(r0, m0, c0, g0), (r1, m1, c1, g1) = out[''], out[KB]
print('rds equal', bool(torch.equal(r0, r1)), 'mask equal', bool(torch.equal(m0, m1)),
      'row_count equal', bool(torch.equal(c0, c1)), 'groups', g0, g1, flush=True)
best = {}
for rep in range(4):
    for kb in ('', KB):
        setkb(kb)
        run()
        torch.cuda.synchronize()
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        t = ctx.timing_read()
        ctx.timing(False)
        best[kb] = min(best.get(kb, 1e9), t['doppler_fft'][0] / 5)
for kb, ms in best.items():
    print(f'RSL_DD_KB={kb or "default"}: doppler/detect {ms:.3f} ms per {F} cfg2 frames', flush=True)
