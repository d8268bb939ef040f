"""Repeat tests/test_gpu_pipelined.py's pipelined-vs-serial comparison R times per placement in one process and report
every mismatch with the first stage that differs (work = K1's range spectra, then RDS, masks / row counts, lists),
the guard canary of both chains, and for a work / RDS mismatch the differing positions with their serial and
pipelined values (to tell a K1, a K2 and a foreign store apart).  GPU box:  python tools/pipelined_repeat.py [R] [noguard]
(noguard: plain allocations, the memory layout of the bench and of the failures recorded in round 3)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT, os.path.join(ROOT, 'tests')]
import torch  # noqa: E402

import rsl  # noqa: E402
import test_gpu_pipelined as T  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 10
GUARD = 'noguard' not in sys.argv[2:]
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=T.A, num_chirps=T.C, chirp_duration=T.TC)
cubes = T._cubes()
want = T.serial_reference(ctx, cfg, cubes)

_orig = T.first_stage_diff


def first_stage_diff_verbose(ch, w):
    st = _orig(ch, w)
    if st and (st.startswith('work') or st.startswith('rds')):
        name = st.split()[0]
        a, b = getattr(ch, name), w[name]
        d = (a != b).nonzero()
        vals = [(idx, complex(b[tuple(idx)].item()), complex(a[tuple(idx)].item())) for idx in d[:64].tolist()]
        st += f"; [index, serial, pipelined]: {vals}"
    return st


T.first_stage_diff = first_stage_diff_verbose
bad = 0
for rep in range(R):
    for placement in (0, 1, 2):
        errs = T.run_pipelined(ctx, cfg, cubes, placement, want, guard=GUARD)
        if errs:
            bad += 1
            print(f'rep {rep} placement {placement}: ' + '; '.join(errs), flush=True)
    print(f'rep {rep} done', flush=True)
print(f'{bad} mismatching runs of {3 * R}', flush=True)
