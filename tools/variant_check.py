"""Bit-identity of a K2 development variant against the default kernel on one cfg2 batch (development library):
    RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so VAR=<knob> python tools/variant_check.py
(VAR: a 0 / 1 development switch; round 3 used it for RSL_R128_X2, a variant since removed)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

F = int(os.environ.get('F', '200'))
var = os.environ['VAR']
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=8, num_chirps=128, chirp_duration=51.2e-6)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(ctx, 1, F, 8, 128, 51.2e-6, 0)[0]
outs = []
for v in ('0', '1'):
    os.environ[var] = v
    bufs = [ch.rds, ch.mask, ch.row_count, ch.peak_pow]
    for t in bufs:
        t.zero_()
    ctx.rds_detect(cube, ch.table, ch.thr_p, ch.i_lo, ch.i_hi, rds=ch.rds, work=ch.work, mask=ch.mask,
                   row_count=ch.row_count, peak_pow=ch.peak_pow, dc_removal=True)
    torch.cuda.synchronize()
    outs.append([t.clone() for t in bufs])
ok = True
for name, a, b in zip(('rds', 'mask', 'row_count', 'peak_pow'), *outs):
    av = a.view(torch.int32) if a.dtype in (torch.float32,) else (a.view(torch.float32).view(torch.int32) if a.is_complex() else a)
    bv = b.view(torch.int32) if b.dtype in (torch.float32,) else (b.view(torch.float32).view(torch.int32) if b.is_complex() else b)
    eq = torch.equal(av, bv)
    ok &= eq
    print(name, 'identical' if eq else 'DIFFERS', flush=True)
sys.exit(0 if ok else 1)
