"""DoA kernel variants timed on one cfg2 batch (hipEvents): the bench's fused DoA + ESPRIT + phase launch against
the argmax-only launch (what the fused extras cost).  GPU box:  python tools/doa_ab.py"""
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
ch.run(cube)
L = ch.lists


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ctx.timing(True)
    ctx.timing_reset()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    t = ctx.timing_read()['doa_scan']
    ctx.timing(False)
    return t[0] / max(t[1], 1)


full = lambda: ctx.doa_extras(ch.rds, L['c_frame'], L['c_rc'], ch.steer, ch.method, n=ch.cell_cap,
                              n_dev=ch.ncell_dev, esprit_scale=ch.esprit_scale, out_idx=ch.gidx,
                              esprit=ch.ext['esprit'], phase=ch.ext['phase'])
argmax = lambda: ctx.doa_extras(ch.rds, L['c_frame'], L['c_rc'], ch.steer, ch.method, n=ch.cell_cap,
                                n_dev=ch.ncell_dev, esprit_scale=ch.esprit_scale, out_idx=ch.gidx)
for name, fn in (('doa+esprit+phase', full), ('doa argmax only', argmax), ('doa+esprit+phase', full)):
    print(f'{name}: {timed(fn):.3f} ms per {F} frames', flush=True)
