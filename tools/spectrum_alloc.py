"""configs[1] spectrum-scan bimodality study: the same spectrum chain, re-allocated several times
in one process at different positions in the caching allocator (pads of various sizes in front, with and without
empty_cache), each run timed per launch with hipEvents; prints the spectrum buffer's address, its alignment and the
scan's ms per 1000 frames, so that a placement dependence shows up as a per-allocation (not per-process) split.

    python tools/spectrum_alloc.py [--frames 1000] [--reps 6]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'radar-slam_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--frames', type=int, default=1000)
    ap.add_argument('--reps', type=int, default=6)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--contig', type=int, default=0, help='1: the spectrum in a physically contiguous allocation '
                    '(RadarChain(spec_out=\'contiguous\'))')
    ap.add_argument('--pre-chain', type=int, default=0, help='first run the cfg2 chain bench.measure_chain (as the '
                    'default bench line does) before the spectrum allocations')
    args = ap.parse_args()
    import torch
    import rsl
    import bench
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    ctx = rsl.get_context(0)
    A, C, Tc, F = 8, 128, 51.2e-6, args.frames
    if args.pre_chain:
        r = bench.measure_chain(ctx, dev, A, C, Tc, 2000, 5, 2, 0, 1, collective=False)
        print(json.dumps({'pre_chain_fps': 2000 * 5 / r['elapsed']}), flush=True)
        del r
        torch.cuda.empty_cache()
    cubes = bench.make_cubes(ctx, 2, F, A, C, Tc, 0)
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc, spectrum=True, cell_frac=0.6)
    pads = [0, 1 << 30, 3 << 29, (1 << 30) + (2 << 20), 7 << 30, 0]
    for rep in range(args.reps):
        pad = pads[rep % len(pads)]
        hold = torch.empty(pad, dtype=torch.uint8, device=dev) if pad else None
        t_alloc = time.perf_counter()
        ch = rsl.RadarChain(cfg, F, ctx, spec_out='contiguous' if args.contig else None)
        torch.cuda.synchronize()
        t_alloc = time.perf_counter() - t_alloc
        ms = []
        for i in range(args.steps + 1):
            torch.cuda.synchronize()
            ctx.timing(True)
            ctx.timing_reset()
            t0 = time.perf_counter()
            ch.run(cubes[i % 2], esprit=False, velocity=False)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3
            kt = ctx.timing_read()
            ctx.timing(False)
            if i:
                ms.append({'wall': round(wall, 3), 'scan': round(kt['doa_scan'][0], 3),
                           'k1': round(kt['range_fft'][0], 3), 'k2': round(kt['doppler_fft'][0], 3)})
        p = ch.spec.data_ptr()
        out = {'rep': rep, 'pad_MiB': pad >> 20, 'contiguous': ch.spec_contiguous, 'alloc_s': round(t_alloc, 3), 'spec_ptr': hex(p), 'spec_GB': ch.spec.numel() * 4 / 1e9,
               'ptr_mod_2M': p % (2 << 20), 'ptr_mod_1G': p % (1 << 30), 'rds_ptr': hex(ch.rds.data_ptr()),
               'steps': ms}
        print(json.dumps(out), flush=True)
        del ch, hold
        if rep % 2:
            torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
