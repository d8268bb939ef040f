"""A/B of the one-pass RDS kernel (K12 + K3', default) against the two-kernel path (RSL_FUSED=0) on the same
device-synthesised cfg2 cubes: RDS difference, detection decisions, entry/cell totals, and per-kernel times.
Run on the GPU box:  python tools/fused_check.py [frames]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'radar-slam_amd'))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import SCENE  # noqa: E402


def run(ch, cube, fused):
    os.environ['RSL_FUSED'] = '1' if fused else '0'
    ch.run(cube)
    torch.cuda.synchronize()
    return (ch.rds.clone(), ch.mask.clone(), ch.row_count.clone(), ch.totals(), ch.gidx.clone())


def timed(ch, cube, fused, ctx, reps=5):
    os.environ['RSL_FUSED'] = '1' if fused else '0'
    ctx.timing(True)
    ctx.timing_reset()
    for _ in range(reps):
        ch.run(cube)
    torch.cuda.synchronize()
    t = ctx.timing_read()
    ctx.timing(False)
    return {k: ms / reps for k, (ms, n) in t.items()}


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    ctx = rsl.get_context(0)
    cfg = rsl.ChainConfig()
    gen = rsl.SyntheticCubes(ctx, SCENE, chirp_duration=cfg.chirp_duration, num_chirps=cfg.num_chirps,
                             num_antennas=cfg.num_antennas, noise_power=0.01)
    cube = gen.generate(F, seed=77, frame0=0)
    ch = rsl.RadarChain(cfg, F, ctx)
    r0 = run(ch, cube, False)
    r1 = run(ch, cube, True)
    ref = r0[0]
    err = ((r1[0] - ref).abs().max() / ref.abs().max()).item()
    bits0 = r0[1].view(torch.uint8).cpu().numpy()
    bits1 = r1[1].view(torch.uint8).cpu().numpy()
    nd = int(np.unpackbits(bits0 ^ bits1).sum())
    npk = int(np.unpackbits(bits0).sum())
    print(f'F={F}: rds rel err {err:.3e}; mask bits differing {nd} of {npk} peaks; '
          f'totals two-kernel {r0[3]} one-pass {r1[3]}; row_count equal {bool((r0[2] == r1[2]).all())}', flush=True)
    for fused in (False, True, False, True):
        t = timed(ch, cube, fused, ctx)
        print(('one-pass ' if fused else 'two-kernel'), {k: round(v, 4) for k, v in t.items() if v > 0}, flush=True)


if __name__ == '__main__':
    main()
