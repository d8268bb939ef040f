"""How many cells k_doa_toep marks ambiguous (re-scanned in fp64 by k_doa_fixup) on the bench workload: one 2000-frame
cfg2 chain (CFG=cfg5: 400 configs[4]-shape frames) with the fixup skipped (development library, RSL_DOA_NOFIX=1: marked cells keep -1 - index), and the DoA
time (K5 + fixup, hipEvent scope) with and without the fixup.
GPU box:  RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so python tools/doa_fix_count.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

F, A, C, TC = {'cfg2': (2000, 8, 128, 51.2e-6), 'cfg5': (400, 16, 256, 102.4e-6)}[os.environ.get('CFG', 'cfg2')]
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=TC)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(ctx, 1, F, A, C, TC, 0)[0]


def doa_ms(reps=5):
    ch.run(cube)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        ch.run_back(emit=False, offsets=False, velocity=False)
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) / reps


for nofix in ('0', '1', '0', '1'):
    os.environ['RSL_DOA_NOFIX'] = nofix
    ms = doa_ms()
    nc = int(ch.ncell_dev.item()) if hasattr(ch, 'ncell_dev') else -1
    g = ch.gidx[:nc].cpu().numpy() if nc > 0 else np.zeros(0)
    mk = g[g < 0]
    full = int(((((-1 - mk) >> 28) & 1) == 0).sum()) if mk.size else 0
    print(f'nofix {nofix}: back half {ms:.3f} ms per {F} frames; cells {nc}; marked {mk.size} '
          f'({(g < 0).mean() * 100:.3f} %), whole-grid re-scans {full}', flush=True)
