"""Does K1's time depend on where the cube sits in HBM?  (Round 4: K1 alone took either 2.31 or 2.52 ms per 2000 cfg2
frames depending on the process.)  One process: the same synthetic cube copied to views at several element offsets
of one larger allocation, the front half (rsl_rds_detect: K1 + K2, K2's input unchanged) timed on each, 3 rounds.
GPU box:  python tools/k1_align.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

F, A, C, TC = 2000, 8, 128, 51.2e-6
S = int(round(TC * 10e6))
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=TC)
ch = rsl.RadarChain(cfg, F, ctx)
src = make_cubes(ctx, 1, F, A, C, TC, 0)[0]
n = src.numel()
OFFS = [0, 256, 512, 4096, 8192, 65536, 131072, 262144]  # complex64 elements: 2 KiB .. 2 MiB
store = torch.empty(n + max(OFFS), dtype=torch.complex64, device=src.device)


def front_ms(cube, reps=4):
    ch.run_front(cube, emit=False, offsets=False)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        ch.run_front(cube, emit=False, offsets=False)
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) / reps


res = {}
for rnd in range(3):
    for off in OFFS:
        v = store[off:off + n].view(F, A, C, S)
        v.copy_(src)
        res.setdefault(off, []).append(front_ms(v))
print('cube base address mod 2 MiB of offset 0:', store.data_ptr() % (2 << 20), flush=True)
for off, t in res.items():
    print(f'offset {off * 8:8d} B: ' + ' '.join(f'{x:.3f}' for x in t) + f'  min {min(t):.3f} ms', flush=True)
