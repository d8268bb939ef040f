"""The fused front half (development library, RSL_FRONT_FUSED=1: rsl_fft.hip k_front_r512; MODE=pair:
RSL_FRONT_PAIR=1, the concurrent k_front_k1p / k_front_k2p pair) against the two-kernel path on the same cfg2 batch:
RDS, masks, row counts and peak powers must be bit-identical, the queue's error word 0; then both timed.
GPU box:  RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so [MODE=pair] python tools/front_fused_check.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT]
import torch  # noqa: E402

import rsl  # noqa: E402
from bench import make_cubes  # noqa: E402

F = int(os.environ.get('F', '2000'))
PAIR = os.environ.get('MODE') == 'pair'
KNOB = 'RSL_FRONT_PAIR' if PAIR else 'RSL_FRONT_FUSED'
ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=8, num_chirps=128, chirp_duration=51.2e-6)
ch = rsl.RadarChain(cfg, F, ctx)
cube = make_cubes(ctx, 1, F, 8, 128, 51.2e-6, 0)[0]


def front():
    ch.run_front(cube, emit=False, offsets=False)


def snap():
    torch.cuda.synchronize()
    return [t.clone() for t in (ch.rds, ch.mask, ch.row_count, ch.peak_pow)]


def timed(reps=6):
    front()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        front()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


os.environ[KNOB] = '0'
for t in (ch.rds, ch.mask, ch.row_count, ch.peak_pow):
    t.zero_()
front()
ref = snap()
os.environ[KNOB] = '1'
for t in (ch.rds, ch.mask, ch.row_count, ch.peak_pow):
    t.zero_()
front()
got = snap()
ring_bytes = 8 * 6 * 16 * 24576
heads = 2 if PAIR else 1
err = int(ch.work.reshape(-1).view(torch.uint8)[ring_bytes + 4 * (heads * 8 * 32 + 2 * 8 * 6 * 32):][:4]
          .view(torch.int32).item())
names = ('rds', 'mask', 'row_count', 'peak_pow')
same = {n: bool(torch.equal(a, b)) for n, a, b in zip(names, ref, got)}
print(('pair' if PAIR else 'fused'), 'vs two kernels bit-identical:', same, 'queue error word', err, flush=True)
WGS = os.environ.get('PAIR_WG_LIST', '2,3').split(';') if PAIR else ['-']
for rnd in range(3):
    os.environ[KNOB] = '0'
    t2 = timed()
    os.environ[KNOB] = '1'
    for wg in WGS:  # PAIR: workgroups per CU of (K1, K2)
        os.environ['RSL_FRONT_PAIR_WG'] = wg
        t1 = timed()
        print(f"round {rnd}: two kernels {t2:.3f} ms, {'pair ' + wg if PAIR else 'fused'} {t1:.3f} ms per {F} frames",
              flush=True)
