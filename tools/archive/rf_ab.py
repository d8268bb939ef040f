"""Range FFT (K1) variants on one cfg2 batch, min of 4 rotations: RSL_RF_CB (chirp rows per tile) and RSL_RF_DBG=1
(no FFT: the kernel's load/store floor).  GPU box:  python tools/rf_ab.py"""
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
VARS = [('CB8', {}), ('CB16', {'RSL_RF_CB': '16'}), ('CB8 noFFT', {'RSL_RF_DBG': '1'}),
        ('CB16 noFFT', {'RSL_RF_CB': '16', 'RSL_RF_DBG': '1'})]
best = {}
for rep in range(4):
    for name, env in VARS:
        for k in ('RSL_RF_CB', 'RSL_RF_DBG'):
            os.environ.pop(k, None)
        os.environ.update(env)
        ctx.rds(cube, ch.table, out=ch.rds, work=ch.work)
        torch.cuda.synchronize()
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(5):
            ctx.rds(cube, ch.table, out=ch.rds, work=ch.work)
        torch.cuda.synchronize()
        t = ctx.timing_read()['range_fft']
        ctx.timing(False)
        best[name] = min(best.get(name, 1e9), t[0] / max(t[1], 1))
for name, ms in best.items():
    print(f'{name}: range FFT {ms:.3f} ms per 1000 frames ({8.389 / ms:.2f} TB/s of cube + work bytes)', flush=True)
