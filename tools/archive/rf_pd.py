"""Range FFT (K1) tiles in flight per workgroup: RSL_RF_PD 1 (default) or 2 (two register sets, capped at 3 waves per
SIMD), K1 before the plain Doppler kernel; results must be identical.  GPU box:  python tools/rf_pd.py"""
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
best = {}
for rep in range(4):
    for pd in ('1', '2'):
        os.environ['RSL_RF_PD'] = pd
        ctx.rds(cube, ch.table, out=ch.rds, work=ch.work)
        torch.cuda.synchronize()
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(5):
            ctx.rds(cube, ch.table, out=ch.rds, work=ch.work)
        torch.cuda.synchronize()
        t = ctx.timing_read()['range_fft']
        ctx.timing(False)
        best[pd] = min(best.get(pd, 1e9), t[0] / max(t[1], 1))
os.environ['RSL_RF_PD'] = '1'
ctx.rds(cube, ch.table, out=ch.rds, work=ch.work)
torch.cuda.synchronize()
ref = ch.work.clone()
for pd in ('2',):
    os.environ['RSL_RF_PD'] = pd
    ctx.rds(cube, ch.table, out=ch.rds, work=ch.work)
    torch.cuda.synchronize()
    print('PD', pd, 'work identical to PD 1:', bool(torch.equal(ch.work, ref)), flush=True)
for pd, ms in best.items():
    print(f'RSL_RF_PD={pd}: range FFT {ms:.3f} ms per 1000 frames ({8.389 / ms:.2f} TB/s)', flush=True)
