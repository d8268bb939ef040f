"""configs[1] spectrum-scan bimodality, second study: which buffer's placement decides the scan's speed?  One spectrum
chain runs once (RDS, lists); then the spectrum scan alone (ctx.doa with the cell-blocked spectrum, exactly as
RadarChain.run_back issues it) is timed reading the RDS from several copies of it in fresh allocations, and writing
the spectrum to several output buffers.  A per-RDS-copy split with stable times per copy points at the RDS gather.

    python tools/spectrum_rds.py [--frames 1000] [--copies 6] [--outs 2]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'radar-slam_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--frames', type=int, default=1000)
    ap.add_argument('--copies', type=int, default=6)
    ap.add_argument('--outs', type=int, default=2)
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    import torch
    import rsl
    import bench
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    ctx = rsl.get_context(0)
    A, C, Tc, F = 8, 128, 51.2e-6, args.frames
    cube = bench.make_cubes(ctx, 1, F, A, C, Tc, 0)[0]
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc, spectrum=True, cell_frac=0.6)
    ch = rsl.RadarChain(cfg, F, ctx)
    ch.run(cube, esprit=False, velocity=False)
    torch.cuda.synchronize()
    del cube
    L = ch.lists
    rdss = [ch.rds] + [ch.rds.clone() for _ in range(args.copies - 1)]
    outs = [ch.spec] + [torch.empty_like(ch.spec) for _ in range(args.outs - 1)]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def scan(rds, out):
        ev[0].record()
        ctx.doa(rds, L['c_frame'], L['c_rc'], ch.steer, ch.method, n=ch.cell_cap, n_dev=ch.ncell_dev,
                out_idx=ch.gidx, want_spec=True, spec_blocked=True, out_spec=out)
        ev[1].record()
        torch.cuda.synchronize()
        return round(ev[0].elapsed_time(ev[1]), 3)

    scan(rdss[0], outs[0])
    for rnd in range(2):
        for i, r in enumerate(rdss):
            for j, o in enumerate(outs):
                ms = [scan(r, o) for _ in range(args.reps)]
                print(json.dumps({'round': rnd, 'rds': i, 'rds_ptr': hex(r.data_ptr()), 'out': j,
                                  'out_ptr': hex(o.data_ptr()), 'scan_ms': ms}), flush=True)


if __name__ == '__main__':
    main()
