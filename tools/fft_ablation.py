"""K1 / K2 ablations on one cfg2 batch (CFG=cfg5: one configs[4]-shape batch of 100 frames), c64 and packed `work` (development library, RSL_LIBRARY=librsl_dev.so):
the standalone time of each kernel with one part removed (results are wrong in the variants; only times matter).
  RSL_RF_DBG: 1 no FFT, 2 no cube loads, 3 loads + LDS staging only
  RSL_DD_DBG: 1 no FFT, 4 no peak-power stores, 5 no mask stores, 6 no work loads, 7 loads + LDS staging only,
              8 no RDS stores, 9 RDS stores only (no detection) -- 8 and 9 in the packed (register-form) kernel only
RSL_WORK_C64=1 keeps c64 rows.  GPU box:  RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so python tools/fft_ablation.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

A, C, TC, F0 = {'cfg2': (8, 128, 51.2e-6, 2000), 'cfg5': (16, 256, 102.4e-6, 100), 'cfg1': (8, 64, 25.6e-6, 4000)}[os.environ.get('CFG', 'cfg2')]
F = int(os.environ.get('F', str(F0)))
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=TC)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(ctx, 1, F, A, C, TC, 0)[0]


def run():
    ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                   row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)


def timed(env):
    for k in ('RSL_RF_DBG', 'RSL_DD_DBG', 'RSL_WORK_C64'):
        os.environ.pop(k, None)
    os.environ.update(env)
    run()
    torch.cuda.synchronize()
    ctx.timing(True)
    ctx.timing_reset()
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    t = ctx.timing_read()
    ctx.timing(False)
    return t['range_fft'][0] / 5, t['doppler_fft'][0] / 5


variants = []
for c64 in (os.environ.get('C64', '1,0')).split(','):
    only0 = os.environ.get('ONLY0') == '1'  # the full kernels only (A/B of two libraries)
    rfl = os.environ.get('RF_LIST')  # explicit variant lists, e.g. RF_LIST=0,5
    ddl = os.environ.get('DD_LIST')
    for rf in rfl.split(',') if rfl else ('0',) if only0 else ('0', '1', '2', '3'):
        variants.append(('K1', {'RSL_WORK_C64': c64, 'RSL_RF_DBG': rf}))
    for dd in ddl.split(',') if ddl else ('0',) if only0 else ('0', '1', '4', '5', '6', '7') + (('8', '9') if c64 == '0' else ()):
        variants.append(('K2', {'RSL_WORK_C64': c64, 'RSL_DD_DBG': dd}))
best = {}
for rep in range(3):
    for i, (k, env) in enumerate(variants):
        t1, t2 = timed(env)
        best[i] = min(best.get(i, 1e9), t1 if k == 'K1' else t2)
for i, (k, env) in enumerate(variants):
    print(f"{k} {'c64   ' if env['RSL_WORK_C64'] == '1' else 'packed'} "
          f"{'RSL_RF_DBG=' + env['RSL_RF_DBG'] if k == 'K1' else 'RSL_DD_DBG=' + env['RSL_DD_DBG']}: "
          f"{best[i]:.3f} ms per {F} frames (min of 3)", flush=True)
