"""K5 timing variants on the bench workload (development library): one 2000-frame cfg2 chain, then the fused DoA
(rsl_doa_extras) alone, repeated, for each RSL_DOA_DBG value given (0 = the shipping kernel; 13 = no second-best
tracking; 14 = no in-tile count), with and without the fp64 fixup (RSL_DOA_NOFIX), 3 rounds interleaved.
GPU box:  RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so python tools/doa_var_time.py [dbg ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

F, A, C, TC = 2000, 8, 128, 51.2e-6
VARS = [int(x) for x in sys.argv[1:]] or [0, 13, 14]
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=TC)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(ctx, 1, F, A, C, TC, 0)[0]
ch.run(cube)
torch.cuda.synchronize()


def doa_ms(reps=6):
    ch.run_back(velocity=False)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        ch.run_back(velocity=False)
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) / reps


res = {}
for rnd in range(3):
    for v in VARS:
        for nofix in ('1', '0'):
            os.environ['RSL_DOA_DBG'] = str(v)
            os.environ['RSL_DOA_NOFIX'] = nofix
            res.setdefault((v, nofix), []).append(doa_ms())
for k, t in sorted(res.items()):
    print(f'dbg {k[0]:2d} nofix {k[1]}: ' + ' '.join(f'{x:.3f}' for x in t) + f'  min {min(t):.3f} ms', flush=True)
