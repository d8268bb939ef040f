"""Is a tighter ambiguity bound safe?  One 2000-frame cfg2 chain (development library); the fused DoA run with the
shipping bound (2e-6) and with 1e-6 (RSL_DOA_DBG=16): marked cells of each (RSL_DOA_NOFIX=1), and, with the fixup, the
number of cells whose final grid index differs (the 2e-6 result is the exact one: any difference is a scan-caused
flip the tighter bound lets through), plus both DoA times.
GPU box:  RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so python tools/doa_bound_study.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

F, A, C, TC = 2000, 8, 128, 51.2e-6
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=TC)
ch = rsl.RadarChain(cfg, F, ctx)
res = {}
for seed_batch in range(2):  # two different 2000-frame blocks (rank 0 / rank 1 generators)
    cube = make_cubes(ctx, 1, F, A, C, TC, seed_batch)[0]
    ch.run(cube)
    torch.cuda.synchronize()
    nc = int(ch.ncell_dev.item())
    out = {}
    for dbg in ('0', '16'):
        os.environ['RSL_DOA_DBG'] = dbg
        os.environ['RSL_DOA_NOFIX'] = '1'
        ch.run_back(velocity=False)
        torch.cuda.synchronize()
        marked = int((ch.gidx[:nc] < 0).sum().item())
        os.environ['RSL_DOA_NOFIX'] = '0'
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ch.run_back(velocity=False)
        t0.record()
        for _ in range(4):
            ch.run_back(velocity=False)
        t1.record()
        torch.cuda.synchronize()
        out[dbg] = (ch.gidx[:nc].clone(), marked, t0.elapsed_time(t1) / 4)
    diff = int((out['0'][0] != out['16'][0]).sum().item())
    print(f'block {seed_batch}: cells {nc}; marked shipping {out["0"][1]} / study {out["16"][1]}; '
          f'DoA {out["0"][2]:.3f} / {out["16"][2]:.3f} ms; cells whose index differs: {diff}', flush=True)
