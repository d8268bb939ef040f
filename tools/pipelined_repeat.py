"""Repeat tests/test_gpu_pipelined.py's pipelined-vs-serial comparison R times per placement in one process and report
every mismatch with the first stage that differs (RDS, mask / row counts, offsets, lists), to localise a
non-deterministic difference.  GPU box:  python tools/pipelined_repeat.py [R]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsl  # noqa: E402

A, C, TC, F, NB = 8, 64, 25.6e-6, 3, 4
R = int(sys.argv[1]) if len(sys.argv) > 1 else 10
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=TC)
g = torch.Generator(device='cuda').manual_seed(11)
S = int(round(TC * 10e6))
cubes = [torch.complex(torch.randn(F, A, C, S, device='cuda', generator=g),
                       torch.randn(F, A, C, S, device='cuda', generator=g)) * 0.1 for _ in range(NB)]
ser = rsl.RadarChain(cfg, F, ctx)
want = []
for cube in cubes:
    ser.run(cube)
    torch.cuda.synchronize()
    want.append(dict(rds=ser.rds.clone(), mask=ser.mask.clone(), row_count=ser.row_count.clone(),
                     res=ser.results()))


def stage_diff(ch, w):
    if not torch.equal(ch.rds, w['rds']):
        d = (ch.rds != w['rds']).nonzero()
        return f"rds ({d.shape[0]} values, first {d[:3].tolist()})"
    if not torch.equal(ch.mask, w['mask']):
        return 'mask'
    if not torch.equal(ch.row_count, w['row_count']):
        return 'row_count'
    return None


bad = 0
for rep in range(R):
    for placement in (0, 1, 2):
        chains = [rsl.RadarChain(cfg, F, ctx) for _ in range(2)]
        sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
        evA = [torch.cuda.Event() for _ in range(2)]
        evB = [torch.cuda.Event() for _ in range(2)]
        used = [False, False]
        main = torch.cuda.current_stream()
        msgs = []

        def check(i, ch):
            res = ch.results()
            st = stage_diff(ch, want[i])
            for key, w in want[i]['res'].items():
                if not np.array_equal(w, res[key], equal_nan=True):
                    msgs.append(f'batch {i}: {key} differs; first differing stage: {st}')
                    break
        for i, cube in enumerate(cubes):
            k = i % 2
            ch = chains[k]
            if used[k]:
                evB[k].synchronize()
                check(i - 2, ch)
            sA.wait_stream(main)
            with torch.cuda.stream(sA):
                ch.run_front(cube, emit=placement == 0, offsets=placement < 2)
                evA[k].record(sA)
            with torch.cuda.stream(sB):
                sB.wait_event(evA[k])
                ch.run_back(emit=placement > 0, offsets=placement == 2)
                evB[k].record(sB)
            used[k] = True
        torch.cuda.synchronize()
        for i in (NB - 2, NB - 1):
            check(i, chains[i % 2])
        if msgs:
            bad += 1
            print(f'rep {rep} placement {placement}: ' + '; '.join(msgs), flush=True)
    print(f'rep {rep} done', flush=True)
print(f'{bad} mismatching runs of {3 * R}', flush=True)
